#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 120 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"kernels_avg_us": {[^}]*}' gpurun_out/$name.log | head -1)"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_c4.py -x -q -p no:cacheprovider > gpurun_out/sm_c4test.log 2>&1 || { echo c4test_fail; tail -5 gpurun_out/sm_c4test.log; }
for i in 1 2; do
  for sm in 1 2 3; do
    run sm${sm}_c4 python3 bench.py --config c4 --steps 200 --warmup 5 --cpu-seconds 0 --tune split_mid=$sm
    run sm${sm}_c3 python3 bench.py --config c3 --steps 200 --warmup 5 --cpu-seconds 0 --tune split_mid=$sm
  done
done
