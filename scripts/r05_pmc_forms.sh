#!/bin/bash
# PMC of the fused loss kernels' forms (row-split fwd1/dw1 vs H-sliced fwd3/dw2): MFMA busy, wait
# breakdown, L2 hit rate, LDS conflicts — one counter pass per run (rocprofv3 does not split).
set -u
O=${O:-gpurun_out/r05_pmc}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
PASSES=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
        "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES")
for form in "lmloss_fwd=1,lmloss_dw=1" "lmloss_fwd=3,lmloss_dw=2" ${EXTRA_FORMS:-}; do
  tag=$(echo $form | tr -d 'a-z_=' | tr ',' '_')
  i=0
  for p in "${PASSES[@]}"; do
    LL_TUNE=$form timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $R/$O/f${tag}_p$i -o p -- \
      python3 $R/tools/lmloss_ablate.py --child --iters 3 --shape ${SHAPE:-6144,768,50257} > $R/$O/f${tag}_p$i.log 2>&1
    rc=$?; echo "form $form pass $i rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
    i=$((i+1))
  done
  python3 $R/tools/pmc_kernels.py $(find $R/$O -path "*f${tag}_p*" -name "*counter_collection.csv") > $R/$O/f${tag}_summary.json
  cat $R/$O/f${tag}_summary.json
done
