#!/bin/bash
# Round 5: k_lmloss_dwp dS without the per-value label test (LL_DWP_FASTDS=1 build under stamp/): parity, stamps, A/B.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fds
mkdir -p $O
cd $R
TRLX_T5_AMD_LIB=$R/stamp/lib_fds.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lmhead_loss.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
TRLX_T5_AMD_LIB=$R/stamp/lib_sfds.so timeout -k 10 120 python tools/dwp_stamps.py --config c2 > $O/stamps.json 2>$O/stamps.err || exit 1
echo "stamps $(cat $O/stamps.json)"
bash scripts/r05_ab_libs.sh c2 fds && bash scripts/r05_ab_libs.sh c3 fds
