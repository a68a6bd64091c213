#!/bin/bash
# Where the world-1 cost of the distributed schedules goes: serial vs pipelined without a
# process group (schedule alone: no fold of the loss tail in pipelined), then with the RCCL helper.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 120 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log | head -1)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/$name.log; exit $rc; }; }
B="python3 bench.py --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line"
for i in 1 2; do
  run split_serial_nodist $B --schedule serial
  run split_serial_nodefer $B --schedule serial --no-defer-tail
  run split_pipe_nodist $B --schedule pipelined
  run split_serial_comm $B --dist --schedule serial --comm rccl
  run split_pipe_comm $B --dist --schedule pipelined --comm rccl
done
