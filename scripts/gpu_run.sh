#!/bin/bash
# Runs GPU steps on the gpurun box; each step has its own time limit and the script
# stops at the first step that faults / aborts / times out (any rc other than 0 or 1).
#   scripts/gpu_run.sh smoke tests bench profile pmc
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 lim=$2; shift 2
    local t0=$(date +%s)
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc ($(( $(date +%s) - t0 ))s)"
    tail -n 4 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"; exit $rc
    fi
}
for step in "$@"; do
    case $step in
        smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) run gpu_tests 1100 python -m pytest tests -m gpu -q -x -p no:cacheprovider ;;
        testsall) run gpu_tests 1100 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
        sweep) run sweep 300 python tools/row_sweep.py ;;
        sweep_c4) B=128 T=128 V=32128 run sweep_c4 300 python tools/row_sweep.py ;;
        sweep_f32) DT=f32 run sweep_f32 300 python tools/row_sweep.py ;;
        bench) run bench 400 python bench.py ;;
        bench_c3) run bench_c3 300 python bench.py --config c3 --cpu-seconds 10 ;;
        bench_c5) run bench_c5 300 python bench.py --config c5 --cpu-seconds 10 ;;
        profile_c5) run profile_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 \
                     -o run -- python bench.py --config c5 --cpu-seconds 0 ;;
        ilql) run ilql_tests 300 python -u -m pytest tests/test_gpu_ilql.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        bench_c4) run bench_c4 300 python bench.py --config c4 --cpu-seconds 10 ;;
        profile_nt) run profile_nt 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_nt \
                     -o run -- python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-timers ;;
        bench_nt) run bench_nt 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-timers ;;
        profile) run profile 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof \
                     -o run -- python bench.py --cpu-seconds 0 ;;
        profile_c4) run profile_c4 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 \
                     -o run -- python bench.py --config c4 --cpu-seconds 0 ;;
        profile_c3) run profile_c3 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 \
                     -o run -- python bench.py --config c3 --cpu-seconds 0 ;;
        pmc_fetch_c4) run pmc_fetch_c4 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_c4 \
                     -o run -- python bench.py --steps 5 --warmup 2 --config c4 --cpu-seconds 0 --no-timers ;;
        pmc_write_c4) run pmc_write_c4 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_c4 \
                     -o run -- python bench.py --steps 5 --warmup 2 --config c4 --cpu-seconds 0 --no-timers ;;
        pmc_fetch_c3) run pmc_fetch_c3 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_c3 \
                     -o run -- python bench.py --steps 5 --warmup 2 --config c3 --cpu-seconds 0 --no-timers ;;
        pmc_write_c3) run pmc_write_c3 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_c3 \
                     -o run -- python bench.py --steps 5 --warmup 2 --config c3 --cpu-seconds 0 --no-timers ;;
        pmc_fetch_c5) run pmc_fetch_c5 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_c5 \
                     -o run -- python bench.py --steps 3 --warmup 1 --config c5 --cpu-seconds 0 --no-timers ;;
        pmc_write_c5) run pmc_write_c5 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_c5 \
                     -o run -- python bench.py --steps 3 --warmup 1 --config c5 --cpu-seconds 0 --no-timers ;;
        pmc_fetch) run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch \
                     -o run -- python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-timers ;;
        pmc_write) run pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write \
                     -o run -- python bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-timers ;;
        newtests) run new_tests 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
                     tests/test_gpu_lmhead_loss.py tests/test_gpu_dist_hidden.py tests/test_gpu_dist_world.py ;;
        hstests) run hs_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
                     tests/test_gpu_lmhead_loss.py -k "h_sliced" ;;
        forms) run forms_c2 300 python tools/lmloss_forms.py --config c2 --fwd 1,2,3,4 --dw 1,2,3 &&
               run forms_c3 300 python tools/lmloss_forms.py --config c3 --fwd 1,2,4 --dw 1,3 ;;
        stamps) LL_HS=1 LL_STAMPS=1 LL_TUNE=lmloss_fwd=4,lmloss_dw=3 run stamps 300 python tools/lmloss_ablate.py --libs stamp/lib_stamp.so ;;
        ablate) LL_HS=1 LL_STAMPS=1 LL_TUNE=lmloss_fwd=3,lmloss_dw=2 run ablate 300 python tools/lmloss_ablate.py \
                    --libs stamp/lib_stamp.so,stamp/lib_abl4.so,stamp/lib_abl1.so ;;
        bench20) run bench20 400 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
