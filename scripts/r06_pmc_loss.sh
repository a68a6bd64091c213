#!/bin/bash
# HBM traffic of the fused loss side's kernels (tools/lossside_bench.py, fused route): FETCH_SIZE
# and WRITE_SIZE in separate rocprofv3 passes (MI355X_MICROARCH.md §HBM), C2 and C3.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_pmc_loss
mkdir -p $O
for cfg in c2 c3; do
    L="python3 $R/tools/lossside_bench.py --config $cfg --routes fused --rounds 1 --iters 4"
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$cfg -o p -- $L > $O/fetch_$cfg.log 2>&1
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$cfg -o p -- $L > $O/write_$cfg.log 2>&1
    echo "pmc $cfg done"
done
