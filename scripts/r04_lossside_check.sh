#!/bin/bash
# Loss side check: parity tests, dW stamps + fwd/bwd times, C2/C3 A/B, kernel trace of the fused route.
set -e
O=gpurun_out/r04_ls
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lmhead_loss.py tests/test_gpu_lmhead.py > $O/tests.txt 2>&1
LL_STAMPS=1 timeout -k 10 120 python3 tools/lmloss_ablate.py --libs abl/lib_stamp.so > $O/stamps.txt 2>&1
timeout -k 10 120 python3 tools/lmloss_ablate.py > $O/time.txt 2>&1
timeout -k 10 200 python3 tools/lossside_bench.py --config c2 > $O/c2.txt 2>&1
timeout -k 10 200 python3 tools/lossside_bench.py --config c3 > $O/c3.txt 2>&1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o t -- python3 $R/tools/lossside_bench.py --config c2 --rounds 1 --iters 5 --routes fused > $R/$O/trace.log 2>&1
f=$(ls $R/$O/trace/*/t_kernel_trace.csv 2>/dev/null || ls $R/$O/trace/t_kernel_trace.csv)
python3 $R/tools/trace_gaps.py $f --last 12 > $R/$O/trace_gaps.txt
echo done
