#!/bin/bash
# The ragged order launch: tests, then C3 under ragged_probe with the round's first order
# kernel (ab/lib_old.so) vs this tree's, then a C3 kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ragged.py tests/test_gpu_lmhead.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/order_tests.log 2>&1 || exit 1
for r in 1 2; do
  for l in old new; do
    lib=$PWD/ab/lib_old.so; [ $l = new ] && lib=$PWD/trlx-t5_amd/libtrlx_t5_amd.so
    echo "== $l $r" >> gpurun_out/order_ab.log
    TRLX_T5_AMD_LIB=$lib timeout -k 10 200 python3 -u tools/ragged_probe.py --rounds 2 --steps 60 2>/dev/null | grep median >> gpurun_out/order_ab.log || exit 3
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03j_prof_c3 -o run -- python3 bench.py --cpu-seconds 0 --no-fp32-line --config c3 --steps 200 --warmup 5 > gpurun_out/r03j_prof_c3.log 2>&1
