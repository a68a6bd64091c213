#!/bin/bash
# Round-6 measurement pass at HEAD: bench lines (C2 with the from_hidden sub-object, C3, C4, C5),
# the C2 rocprof kernel trace, the PPO loss side's interleaved A/B and kernel trace.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06f}
mkdir -p $O
cd $R
step() {  # name limit cmd...
    local n=$1 lim=$2; shift 2
    timeout -k 10 $lim "$@" > $O/$n.log 2>&1
    local rc=$?; echo "$n rc=$rc"; tail -c 1500 $O/$n.log | tail -2
    if [ $rc -ne 0 ]; then exit $rc; fi
}
step bench_c2 300 python bench.py --steps 20 --warmup 5
step bench_c3 300 python bench.py --config c3 --cpu-seconds 10
step lossside_c2 200 python tools/lossside_bench.py --config c2 --routes gemm,fused,fused_recompute --rounds 5 --iters 10
step lossside_c3 200 python tools/lossside_bench.py --config c3 --routes gemm,fused,fused_recompute --rounds 5 --iters 10
step dropin_c2 200 python tools/dropin_update.py --config c2
cd /tmp && export TMPDIR=/tmp
step prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $R/bench.py --steps 20 --warmup 5 --cpu-seconds 0
step prof_lossside 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lossside -o run -- python3 $R/tools/lossside_bench.py --config c2 --routes fused,gemm --rounds 2 --iters 10
step prof_lossside_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lossside_c3 -o run -- python3 $R/tools/lossside_bench.py --config c3 --routes fused,gemm --rounds 2 --iters 10
step mfma_c2 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mfma_c2 -o p -- python3 $R/tools/lossside_bench.py --config c2 --rounds 1 --iters 5
step mfma_c3 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mfma_c3 -o p -- python3 $R/tools/lossside_bench.py --config c3 --rounds 1 --iters 5
echo done
