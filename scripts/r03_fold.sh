#!/bin/bash
# Round 3: the split GAE folded into the loss rows launch (trlx_ppo_loss_rows_split_gae).
# GPU tests of the fold and the schedules it changes, then serial vs pipelined bench lines
# interleaved on one box (C2, C4, C3).  Stops at the first failing step.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 lim=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc ($(( $(date +%s) - t0 ))s) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log | head -1)"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -30 "gpurun_out/$name.log"; exit $rc; fi
}
B="python3 bench.py --cpu-seconds 0 --no-fp32-line"
steps=${@:-tests bench}
for st in $steps; do
    case $st in
        tests) run r03f_tests 600 python3 -u -m pytest tests/test_gpu_gae_fold.py tests/test_gpu_split_beta.py tests/test_gpu_dist.py tests/test_gpu_rccl.py tests/test_gpu_control.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ;;
        all) run r03f_all_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ;;
        bench) for i in 1 2; do
                 for c in c2 c4 c3; do
                   run r03f_${c}_serial_$i 200 $B --config $c --steps 200 --warmup 5 --schedule serial
                   run r03f_${c}_pipe_$i 200 $B --config $c --steps 200 --warmup 5 --schedule pipelined
                 done
               done ;;
        rccl) for i in 1 2; do
                run r03f_rccl_serial_$i 200 $B --steps 200 --warmup 5 --dist --schedule serial
                run r03f_rccl_pipe_$i 200 $B --steps 200 --warmup 5 --dist --schedule pipelined
              done ;;
        ab) for i in 1 2 3; do
              for c in c2 c4; do
                run r03f_ab_${c}_serial_$i 200 $B --config $c --steps 200 --warmup 5 --schedule serial
                run r03f_ab_${c}_serial_split_$i 200 $B --config $c --steps 200 --warmup 5 --schedule serial --split-beta
                run r03f_ab_${c}_pipe_nofold_$i 200 $B --config $c --steps 200 --warmup 5 --schedule pipelined --no-gae-fold
                run r03f_ab_${c}_pipe_$i 200 $B --config $c --steps 200 --warmup 5 --schedule pipelined
              done
            done ;;
        ab2) for i in 1 2 3; do
              for c in c2 c4; do
                run r03f_ab2_${c}_serial_$i 200 $B --config $c --steps 200 --warmup 5 --schedule serial
                run r03f_ab2_${c}_split_derive_$i 200 $B --config $c --steps 200 --warmup 5 --schedule serial --split-beta
                run r03f_ab2_${c}_split_coefl_$i 200 $B --config $c --steps 200 --warmup 5 --schedule serial --split-beta --coef-launch
              done
            done ;;
        multi) run r03f_host_c2 120 python3 tools/host_overhead.py --config c2
               run r03f_host_c4 120 python3 tools/host_overhead.py --config c4
               run r03f_gloo2_c2 300 $B --gpus 2 --backend gloo --steps 40 --warmup 5
               run r03f_gloo2_c4 300 $B --gpus 2 --backend gloo --config c4 --steps 40 --warmup 5
               for i in 1 2; do
                 run r03f_rccl_serial_$i 200 $B --steps 200 --warmup 5 --dist --schedule serial
                 run r03f_rccl_pipe_$i 200 $B --steps 200 --warmup 5 --dist --schedule pipelined
               done ;;
        strong) for i in 1 2; do
                  run r03f_strong_serial_$i 200 $B --config c4 --global-batch 1024 --steps 50 --warmup 5 --schedule serial
                  run r03f_strong_split_$i 200 $B --config c4 --global-batch 1024 --steps 50 --warmup 5 --schedule serial --split-beta
                  run r03f_strong_pipe_$i 200 $B --config c4 --global-batch 1024 --steps 50 --warmup 5 --schedule pipelined
                done ;;
        prof) run r03f_prof_c2_pipe 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03f_prof_c2_pipe -o run -- $B --steps 200 --warmup 5 --schedule pipelined ;;
        *) echo "unknown step $st"; exit 2 ;;
    esac
done
