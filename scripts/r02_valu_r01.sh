#!/bin/bash
# VALU counters of the round-1 rows kernels (tree at 63d22a9 in _ab_r01, built here) for the
# before/after comparison in profiles/r02_pmc_valu_c2.txt
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/r01_pmc_valu_c2 -o run -- python3 _ab_r01/bench.py --cpu-seconds 0 --steps 5 --warmup 2 --no-timers > gpurun_out/r01_pmc_valu_c2.log 2>&1
echo "r01 valu rc=$?"
