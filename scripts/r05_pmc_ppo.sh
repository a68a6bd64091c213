#!/bin/bash
# PMC of the PPO loss side's kernels (tools/lossside_bench.py fused, C2): MFMA busy, waits, L2,
# LDS — one counter group per rocprofv3 run (rocprofv3 does not split passes).
set -u
R=$GRAFT_REPO_ROOT
O=${O:-$R/gpurun_out/r05_pmc_ppo}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PASSES=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
        "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES"
        "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_WAVE_CYCLES GRBM_GUI_ACTIVE")
i=0
for p in "${PASSES[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d $O/p$i -o p -- \
    python3 $R/tools/lossside_bench.py --config ${CFG:-c2} --routes fused --rounds 1 --iters 3 ${TUNE:-} > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then break; fi
  i=$((i+1))
done
python3 $R/tools/pmc_kernels.py $(find $O -name "*counter_collection.csv") > $O/summary.json
cat $O/summary.json
