#!/bin/bash
# The bench's RCCL path at world size 1 (--dist): serial schedule (blocking whitening
# all-reduce, loss tail folded) vs pipelined (all-reduce behind the next experience rows),
# each through torch.distributed (ProcessGroupNCCL) and through the boundary's RCCL helper.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 120 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log | head -1) $(grep -o '"comm": [a-z"]*' gpurun_out/$name.log | head -1) $(grep -o '"kernels_avg_us": {[^}]*}' gpurun_out/$name.log | head -1)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/$name.log; exit $rc; }; }
B="python3 bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line"
for i in 1 2; do
  run rccl_nodist $B
  run rccl_serial_torch $B --dist --schedule serial --comm torch
  run rccl_pipe_torch $B --dist --schedule pipelined --comm torch
  run rccl_serial_comm $B --dist --schedule serial --comm rccl
  run rccl_pipe_comm $B --dist --schedule pipelined --comm rccl
done
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rccl -o run -- python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-fp32-line --no-timers --dist --schedule serial --comm rccl > gpurun_out/prof_rccl.log 2>&1 || { echo "prof rc=$?"; tail -5 gpurun_out/prof_rccl.log; exit 1; }
echo prof ok
