#!/bin/bash
# 16x16 image swizzle: parity, fwd/bwd times (both forward forms), C2/C3 A/B, LDS bank-conflict PMC.
set -e
O=gpurun_out/r04_swz
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lmhead_loss.py tests/test_gpu_lmhead.py > $O/tests.txt 2>&1
timeout -k 10 120 python3 tools/lmloss_ablate.py > $O/time.txt 2>&1
LL_TUNE=lmloss_fwd=2 timeout -k 10 120 python3 tools/lmloss_ablate.py >> $O/time.txt 2>&1
timeout -k 10 300 python3 tools/lossside_bench.py --config c2 --rounds 5 > $O/c2.txt 2>&1
timeout -k 10 200 python3 tools/lossside_bench.py --config c3 --rounds 3 > $O/c3.txt 2>&1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/$O/lds -o p -- python3 $R/tools/lmloss_ablate.py --child --iters 3 --shape 6144,768,50257 > $R/$O/lds.log 2>&1
echo done
