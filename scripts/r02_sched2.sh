#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log | head -1)"; [ $rc -eq 0 ] || exit $rc; }
for i in 1 2; do

run s_fold python bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line --schedule serial
run s_nofold python bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line --schedule serial --no-defer-tail

run p_noov python bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line --schedule pipelined
done
