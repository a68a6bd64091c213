#!/bin/bash
# Schedules: N=1 serial vs pipelined; N=2 (gloo, both ranks on the one GPU) serial vs pipelined.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 240 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log; [ $rc -eq 0 ] || exit $rc; }
run n1_serial python bench.py --steps 100 --warmup 5 --cpu-seconds 0 --schedule serial
run n1_pipe python bench.py --steps 100 --warmup 5 --cpu-seconds 0 --schedule pipelined
run n1_serial_b python bench.py --steps 100 --warmup 5 --cpu-seconds 0 --schedule serial
run n2_gloo_pipe python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 40 --warmup 5 --backend gloo --schedule pipelined
run n2_gloo_serial python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 40 --warmup 5 --backend gloo --schedule serial
