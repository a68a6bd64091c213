#!/bin/bash
# Kernel traces of the world-1 pipelined schedule with the RCCL helper: side-stream vs inline all-reduces.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in side inline; do
  SCHED_PROBE_ONLY=pipelined/$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pipe_$v -o run -- python3 tools/sched_probe.py > gpurun_out/prof_pipe_$v.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/prof_pipe_$v.log; exit 1; }
  tail -2 gpurun_out/prof_pipe_$v.log
done
