#!/bin/bash
# Kernel trace of the loss side's two routes at C2 (durations + inter-kernel gaps).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_trace
mkdir -p $O
for route in fused gemm; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/$route -o t -- python3 $R/tools/lossside_bench.py --config c2 --rounds 1 --iters 3 --routes $route > $O/$route.log 2>&1
  f=$(ls $O/$route/*/t_kernel_trace.csv 2>/dev/null || ls $O/$route/t_kernel_trace.csv)
  python3 $R/tools/trace_gaps.py $f --last 24 > $O/${route}_gaps.txt
done
echo done
