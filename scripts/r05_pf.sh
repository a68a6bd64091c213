#!/bin/bash
# Round 5: forward S-loop prefetch depth (LL_FWD_PF builds under stamp/): parity of the default, stamps, A/B.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pf
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lmhead_loss.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
TRLX_T5_AMD_LIB=$R/stamp/lib_stamp.so timeout -k 10 120 python tools/dwp_stamps.py --config c2 > $O/stamps.json 2>$O/stamps.err || exit 1
echo "stamps $(cat $O/stamps.json)"
bash scripts/r05_ab_libs.sh c2 pf4 pf6 pf12
