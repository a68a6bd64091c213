#!/bin/bash
# Saved-P dW kernel ablations (stamp builds; results wrong): 128 no P loads, 256 no h DMA, 512 no dS.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dwp_abl
mkdir -p $O
cd $R
for L in stamp sa128 sa256 sa512; do
  TRLX_T5_AMD_LIB=$R/stamp/lib_$L.so timeout -k 10 120 python tools/dwp_stamps.py --config c2 > $O/$L.json 2>$O/$L.err || exit 1
  echo "$L $(cat $O/$L.json)"
done
