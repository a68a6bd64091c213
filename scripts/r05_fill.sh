#!/bin/bash
# Round 5: forward fill variants (LL_FWD_FILL 1 / 2 builds under stamp/): parity of each, stamps, A/B.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fill
mkdir -p $O
cd $R
for L in fill1 fill2; do
  TRLX_T5_AMD_LIB=$R/stamp/lib_$L.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lmhead_loss.py > $O/tests_$L.log 2>&1 || { tail -20 $O/tests_$L.log; exit 1; }
  echo "$L tests $(tail -1 $O/tests_$L.log)"
done
for L in stamp sfill1 sfill2 sa2048; do
  TRLX_T5_AMD_LIB=$R/stamp/lib_$L.so timeout -k 10 120 python tools/dwp_stamps.py --config c2 > $O/stamps_$L.json 2>$O/stamps_$L.err || exit 1
  echo "$L $(cat $O/stamps_$L.json)"
done
bash scripts/r05_ab_libs.sh c2 fill1 fill2
