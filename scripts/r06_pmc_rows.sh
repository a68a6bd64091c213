#!/bin/bash
# Round-6 HBM traffic of the bench lines' row kernels at HEAD (one counter per rocprofv3 run,
# FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md §HBM) -> gpurun_out/r06_pmc/
# {fetch,write}_<cfg>; tools/pmc_summary.py folds them into profiles/pmc_traffic.json.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_pmc
mkdir -p $O
for cfg in c2 c2_fp32 c3 c4 c5; do
    extra="--config $cfg"
    [ $cfg = c2_fp32 ] && extra="--config c2 --logits-dtype fp32"
    B="python3 $R/bench.py --cpu-seconds 0 --no-fp32-line --no-from-hidden $extra --steps 5 --warmup 2 --settle-ms 0 --no-timers"
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$cfg -o p -- $B > $O/fetch_$cfg.log 2>&1
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$cfg -o p -- $B > $O/write_$cfg.log 2>&1
    echo "pmc $cfg done"
done
