# After the store-policy auto rule: default benches C2 / C5 / C4, the C4 strong shape with
# auto (sc1) vs forced nt, and the parity tests that exercise the knobs.
set -u
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1 || { tail -30 gpurun_out/par.log; exit 1; }
tail -2 gpurun_out/par.log
timeout -k 10 120 python bench.py --cpu-seconds 0 > gpurun_out/b_c2.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --config c5 --cpu-seconds 0 > gpurun_out/b_c5.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --config c4 --cpu-seconds 0 > gpurun_out/b_c4.log 2>&1 || exit 1
grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/b_c*.log
ROWS=1024 timeout -k 10 200 python tools/policy_sweep.py c4 store_policy 0,5 || exit 1
