#!/bin/bash
# Round-6 loss-side profile at C2 and C3: per-kernel durations (kernel trace + stats, csv) and the
# MFMA-busy PMC pass (one counter group per run), both over tools/lossside_bench.py.
# usage: scripts/r06_prof.sh <tag> [cfgs...]
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-r06}
shift || true
CFGS=${@:-c2 c3}
O=$R/gpurun_out/${TAG}_prof
mkdir -p $O
for cfg in $CFGS; do
    L="python3 $R/tools/lossside_bench.py --config $cfg --rounds 1 --iters 5"
    timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$cfg -o k -- $L > $O/kt_$cfg.log 2>&1
    echo "kernel trace $cfg done"
    timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mfma_$cfg -o p -- $L > $O/mfma_$cfg.log 2>&1
    echo "mfma $cfg done"
done
