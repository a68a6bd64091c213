#!/bin/bash
# Verdict r02 item 7: the fp32 long-row R+W ceiling (tools/rowpipe_probe: one workgroup per
# 201-KB row, nt loads + nt stores) and the product's fp32 row kernels (C5 ILQL rows, C2 fp32
# PPO loss rows) interleaved in ONE call on one box, three rounds.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r03_fp32_ceiling.log
: > $out
for i in 1 2 3; do
    timeout -k 10 120 ./tools/rowpipe_probe >> $out 2>&1 || exit $?
    timeout -k 10 200 python3 bench.py --config c5 --steps 100 --warmup 5 --cpu-seconds 0 >> $out 2>&1 || exit $?
    timeout -k 10 200 python3 bench.py --config c2 --logits-dtype fp32 --steps 100 --warmup 5 --cpu-seconds 0 --no-fp32-line >> $out 2>&1 || exit $?
    echo "round $i done"
done
