#!/bin/bash
# Measurement set (TAG=r03 by default) on one MI355X: bench lines (C2 default = the driver's command, C3,
# C4, C5, C4 strong-scaling shape), rocprofv3 kernel traces, PMC HBM bytes (separate FETCH /
# WRITE passes) and VALU counters.  Each GPU step has its own time limit; the script stops at
# the first step that faults / aborts / times out.
#   TAG=r03 bash scripts/measure.sh [steps...]   (default: all)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03}
run() {
    local name=$1 lim=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc ($(( $(date +%s) - t0 ))s) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log | head -1)"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; tail -5 "gpurun_out/$name.log"; exit $rc; fi
}
B="python3 bench.py --cpu-seconds 0 --no-fp32-line"
steps=${@:-bench c3 c4 c5 strong prof prof_c4 prof_c5 pmc}
for st in $steps; do
    case $st in
        bench) run ${TAG}_bench_c2 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
        c3) run ${TAG}_bench_c3 300 $B --config c3 --steps 200 --warmup 5 ;;
        c4) run ${TAG}_bench_c4 300 $B --config c4 --steps 200 --warmup 5 ;;
        c5) run ${TAG}_bench_c5 300 $B --config c5 --steps 100 --warmup 5 ;;
        strong) run ${TAG}_bench_c4_strong1024 300 $B --config c4 --global-batch 1024 --steps 50 --warmup 5 ;;
        prof) run ${TAG}_prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_c2 -o run -- $B --steps 200 --warmup 5 ;;
        prof_c3) run ${TAG}_prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_c3 -o run -- $B --config c3 --steps 200 --warmup 5 ;;
        prof_c4) run ${TAG}_prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_c4 -o run -- $B --config c4 --steps 200 --warmup 5 ;;
        prof_c5) run ${TAG}_prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_c5 -o run -- $B --config c5 --steps 100 --warmup 5 ;;
        pmc)
            for cfg in ${PMC_CFGS:-c2 c3 c4 c5}; do
                run ${TAG}_pmc_fetch_$cfg 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch_$cfg -o run -- $B --config $cfg --steps 5 --warmup 2 --settle-ms 0 --no-timers
                run ${TAG}_pmc_write_$cfg 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write_$cfg -o run -- $B --config $cfg --steps 5 --warmup 2 --settle-ms 0 --no-timers
            done ;;
        valu) run ${TAG}_pmc_valu_c2 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/${TAG}_pmc_valu_c2 -o run -- $B --steps 5 --warmup 2 --settle-ms 0 --no-timers ;;
        tests) run ${TAG}_gpu_tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ;;
        tsplit) run ${TAG}_gpu_tests_split 600 python3 -u -m pytest tests/test_gpu_split_beta.py tests/test_gpu_dist.py tests/test_gpu_rccl.py tests/test_gpu_control.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
        sched) for i in 1 2; do
                 run ${TAG}_sched_serial_$i 200 $B --steps 200 --warmup 5
                 run ${TAG}_sched_pipe_$i 200 $B --steps 200 --warmup 5 --schedule pipelined
                 run ${TAG}_sched_rccl_serial_$i 200 $B --steps 200 --warmup 5 --dist --schedule serial
                 run ${TAG}_sched_rccl_pipe_$i 200 $B --steps 200 --warmup 5 --dist --schedule pipelined
               done ;;
        mfma) run ${TAG}_pmc_mfma_lossside_c2 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/${TAG}_pmc_mfma_c2 -o run -- python3 tools/lossside_bench.py --config c2 --rounds 1 --iters 3 ;;
        smoke) run ${TAG}_smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
        *) echo "unknown step $st"; exit 2 ;;
    esac
done
