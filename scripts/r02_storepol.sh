#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 120 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"kernels_avg_us": {[^}]*}' gpurun_out/$name.log | head -1)"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do
  for sp in 0 1 2 3 4; do
    run sp${sp}_c2 python3 bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line --tune store_policy=$sp
  done
done
