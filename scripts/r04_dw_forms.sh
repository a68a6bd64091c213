#!/bin/bash
# dW kernel forms (tuning lmloss_dw_stage 0..3): parity tests, in-kernel stamps, C2 A/B.
set -e
O=gpurun_out/r04_dw
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lmhead_loss.py tests/test_gpu_lmhead.py > $O/tests.txt 2>&1
for st in 0 1 2 3; do
  LL_TUNE=lmloss_dw_stage=$st LL_STAMPS=1 timeout -k 10 120 python3 tools/lmloss_ablate.py --libs abl/lib_stamp.so > $O/stamps_$st.txt 2>&1
  LL_TUNE=lmloss_dw_stage=$st timeout -k 10 120 python3 tools/lmloss_ablate.py > $O/time_$st.txt 2>&1
done
for st in 0 1 2 3; do
  timeout -k 10 200 python3 tools/lossside_bench.py --config c2 --tune lmloss_dw_stage=$st > $O/c2_$st.txt 2>&1
done
echo done
