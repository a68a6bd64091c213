#!/bin/bash
# Saved-P plan check: focused parity tests, interleaved A/B (gemm / saved-P / recompute), kernel trace.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/savep
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_lmhead_loss.py -k "hot_path or saved_p" > $O/tests.log 2>&1
echo "tests rc=$?"; tail -3 $O/tests.log
timeout -k 10 200 python tools/lossside_bench.py --config c2 --routes gemm,fused,fused_recompute --rounds 3 --iters 10 > $O/ab_c2.log 2>&1 || exit 1
timeout -k 10 200 python tools/lossside_bench.py --config c3 --routes gemm,fused,fused_recompute --rounds 3 --iters 10 > $O/ab_c3.log 2>&1 || exit 1
cat $O/ab_c2.log $O/ab_c3.log | grep config
if [ -f $R/stamp/lib_nostag.so ]; then
  TRLX_T5_AMD_LIB=$R/stamp/lib_nostag.so timeout -k 10 200 python tools/lossside_bench.py --config c2 --routes fused --rounds 3 --iters 10 > $O/ab_c2_nostag.log 2>&1 || exit 1
  timeout -k 10 200 python tools/lossside_bench.py --config c2 --routes fused --rounds 3 --iters 10 > $O/ab_c2_stag.log 2>&1 || exit 1
  echo "nostag $(grep config $O/ab_c2_nostag.log)"; echo "stag $(grep config $O/ab_c2_stag.log)"
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof -o p -- python3 $R/tools/lossside_bench.py --config c2 --routes fused,fused_recompute --rounds 1 --iters 5 > $O/prof.log 2>&1 || exit 1
echo done
export TRLX_T5_AMD_LIB=$R/stamp/lib_stamp.so
cd $R && timeout -k 10 120 python tools/dwp_stamps.py --config c2 > $O/stamps.json 2>$O/stamps.err && cat $O/stamps.json
