#!/bin/bash
# C4 at 1024 rollouts on one GPU (the strong-scaling N = 1 point): store policy / residency
# variants interleaved in one call.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r03_strong_check.log
: > $out
B="python3 bench.py --cpu-seconds 0 --no-fp32-line --config c4 --global-batch 1024 --steps 30 --warmup 3"
for r in 1 2; do
  for v in "default:" "nt:--tune store_policy=5" "split_mid:--tune split_mid=3" "split_mid_nt:--tune split_mid=3 --tune store_policy=5"; do
    name=${v%%:*}; flags=${v#*:}
    line=$(timeout -k 10 200 $B $flags 2>/dev/null | grep '^{') || exit 3
    echo "$line" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('round $r $name ms', d['ms_per_step'], 'kern', r['kernels_avg_us'])" | tee -a $out
  done
done
