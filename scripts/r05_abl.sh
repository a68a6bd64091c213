cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for L in default abl32 abl64; do
  if [ $L = default ]; then unset TRLX_T5_AMD_LIB; else export TRLX_T5_AMD_LIB=$R/stamp/lib_$L.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/abl_$L -o p -- python3 $R/tools/lossside_bench.py --config c2 --routes fused --rounds 1 --iters 5 > $R/gpurun_out/abl_$L.log 2>&1 || exit 1
done
