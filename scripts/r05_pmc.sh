#!/bin/bash
# Round-5 PMC passes at HEAD (one counter group per rocprofv3 run, MI355X_MICROARCH.md §HBM):
#   HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes) of the bench lines c2, c2_fp32, c3, c4, c5
#   -> gpurun_out/r05_pmc/{fetch,write}_<cfg>; summarised into profiles/pmc_traffic.json by
#   tools/pmc_summary.py (run afterwards in the container with --commit <HEAD>).
#   MFMA-busy of the fused loss side vs the hipBLASLt route (tools/lossside_bench.py, C2 and C3).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_pmc
mkdir -p $O
for cfg in c2 c2_fp32 c3 c4 c5; do
    extra="--config $cfg"
    [ $cfg = c2_fp32 ] && extra="--config c2 --logits-dtype fp32"
    B="python3 $R/bench.py --cpu-seconds 0 --no-fp32-line --no-from-hidden $extra --steps 5 --warmup 2 --settle-ms 0 --no-timers"
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$cfg -o p -- $B > $O/fetch_$cfg.log 2>&1
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$cfg -o p -- $B > $O/write_$cfg.log 2>&1
    echo "pmc $cfg done"
done
for cfg in c2 c3; do
    L="python3 $R/tools/lossside_bench.py --config $cfg --rounds 1 --iters 3"
    timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mfma_$cfg -o p -- $L > $O/mfma_$cfg.log 2>&1
    echo "mfma $cfg done"
done
echo done
