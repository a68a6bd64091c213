set -u
cd /root/repo
mkdir -p gpurun_out
: > gpurun_out/ab_c5.log
for r in 1 2 3; do for l in A B C; do
  TRLX_T5_AMD_LIB=$PWD/ab/lib_$l.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_c5_$l$r -o run -- python3 bench.py --config c5 --steps 50 --warmup 5 --cpu-seconds 0 > gpurun_out/ab_c5_$l$r.log 2>&1 || exit 3
  echo "round $r lib $l $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_c5_$l$r.log) $(python3 tools/kernel_stats.py gpurun_out/ab_c5_$l$r/run_kernel_stats.csv | grep -E 'prep|finalize' | awk '{print $1, $4}' | tr '\n' ' ')" >> gpurun_out/ab_c5.log
done; done
