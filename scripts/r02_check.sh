#!/bin/bash
# GPU check: gpu tests (one process), then the driver's exact bench command.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 5 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -n 2 gpurun_out/bench_driver.log
exit $rc
