#!/bin/bash
# A/B on one box: round-1 tree (_ab_r01, built here) vs this tree, C2 and C4, interleaved.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 120 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"kernels_avg_us": {[^}]*}' gpurun_out/$name.log | head -1)"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
  for cfg in c2 c4; do
    run ab_r01_$cfg python3 _ab_r01/bench.py --config $cfg --steps 200 --warmup 50 --cpu-seconds 0 --no-overlap
    run ab_r02_$cfg python3 bench.py --config $cfg --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line
    run ab_r02nd_$cfg python3 bench.py --config $cfg --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line --no-defer-tail
  done
done
