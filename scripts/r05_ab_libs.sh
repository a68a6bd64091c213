#!/bin/bash
# A/B of library builds (stamp/lib_<name>.so vs the in-tree one), alternating processes:
#   scripts/r05_ab_libs.sh <config> <name> [<name> ...]
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_libs
mkdir -p $O
cd $R
cfg=$1; shift
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for L in base "$@"; do
    if [ $L = base ]; then unset TRLX_T5_AMD_LIB; else export TRLX_T5_AMD_LIB=$R/stamp/lib_$L.so; fi
    timeout -k 10 200 python tools/lossside_bench.py --config $cfg --routes fused --rounds 3 --iters 10 > $O/${cfg}_${L}_$round.log 2>&1 || exit 1
    echo "$cfg $L round $round $(grep -o '"fused": \[[^]]*\]' $O/${cfg}_${L}_$round.log)"
  done
done
