# Store cache policy A/B (nt = 5 vs sc1 = 2): ILQL C5 through bench.py, PPO through
# tools/policy_sweep.py (interleaved) at shapes around the auto threshold (1.5 GB of gradient
# rows per launch).  GPU-box script; each step under its own time limit.
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for p in 5 2; do
    timeout -k 10 120 python bench.py --config c5 --cpu-seconds 0 --tune store_policy=$p > gpurun_out/c5_pol${p}_$i.log 2>&1 || exit 1
  done
done
grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/c5_pol*.log
ROWS=384 timeout -k 10 150 python tools/policy_sweep.py c2 store_policy 5,2 || exit 1
DT=fp32 ROWS=256 timeout -k 10 150 python tools/policy_sweep.py c2 store_policy 5,2 || exit 1
ROWS=192 timeout -k 10 150 python tools/policy_sweep.py c4 store_policy 5,2 || exit 1
