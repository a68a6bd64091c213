#!/bin/bash
# Round-4 PMC passes (one counter group per rocprofv3 run, MI355X_MICROARCH.md §HBM / PMC slots):
#   c2_fp32 HBM traffic of the fp32-logits bench line (FETCH_SIZE, WRITE_SIZE in separate passes)
#   MFMA-busy of the fused loss side vs the hipBLASLt route (tools/lossside_bench.py, C2)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_pmc
mkdir -p $O
B="python3 $R/bench.py --cpu-seconds 0 --no-fp32-line --config c2 --logits-dtype fp32 --steps 5 --warmup 2 --settle-ms 0 --no-timers"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_fp32 -o p -- $B > $O/fetch_fp32.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_fp32 -o p -- $B > $O/write_fp32.log 2>&1
L="python3 $R/tools/lossside_bench.py --config c2 --rounds 1 --iters 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mfma_c2 -o p -- $L > $O/mfma_c2.log 2>&1
L3="python3 $R/tools/lossside_bench.py --config c3 --rounds 1 --iters 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mfma_c3 -o p -- $L3 > $O/mfma_c3.log 2>&1
echo done
