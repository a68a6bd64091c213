#!/bin/bash
# Per-kernel A/B of library builds: for each lib (base = the in-tree one, else stamp/lib_<name>.so)
# and round, a kernel trace of tools/lossside_bench.py's fused route and the median duration of
# every loss kernel (tools/kernel_median.py).   scripts/r06_kab.sh <config> <name> [<name> ...]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/kab
mkdir -p $O
cfg=$1; shift
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for L in base "$@"; do
    if [ $L = base ]; then unset TRLX_T5_AMD_LIB; else export TRLX_T5_AMD_LIB=$R/stamp/lib_$L.so; fi
    D=$O/${cfg}_${L}_$round
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D -o k -- python3 $R/tools/lossside_bench.py --config $cfg --routes fused --rounds 1 --iters 12 > $D.log 2>&1 || exit 1
    echo "$cfg $L round $round $(python3 $R/tools/kernel_median.py $D/k_kernel_trace.csv)"
  done
done
