#!/bin/bash
# A/B of the current tree against an older checkout in ab/old (its own library and bench.py),
# interleaved rounds on one box.   bash scripts/ab_trees.sh "<bench args>" [rounds]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
args=${1:-"--config c4"}; rounds=${2:-2}
out=gpurun_out/ab_trees.log
: > $out
for r in $(seq 1 $rounds); do
  for t in old new; do
    d=$PWD; [ $t = old ] && d=$PWD/ab/old
    line=$(cd $d && timeout -k 10 300 python3 bench.py $args --cpu-seconds 0 --no-fp32-line 2>/dev/null | grep '^{') || exit 3
    echo "$line" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('round $r tree $t ms', d['ms_per_step'], 'kern', r['kernels_avg_us'])" | tee -a $out
  done
done
