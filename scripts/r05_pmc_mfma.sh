#!/bin/bash
# MFMA-busy PMC of the fused loss side vs the hipBLASLt route (tools/lossside_bench.py, C2 and C3),
# one counter group per rocprofv3 run (the mfma passes of scripts/r05_pmc.sh without the HBM passes).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_pmc
mkdir -p $O
for cfg in c2 c3; do
    L="python3 $R/tools/lossside_bench.py --config $cfg --rounds 1 --iters 3"
    timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mfma_$cfg -o p -- $L > $O/mfma_$cfg.log 2>&1
    echo "mfma $cfg done"
done
