for i in 1 2; do
  timeout -k 10 120 python bench.py --config c5 --cpu-seconds 0 > gpurun_out/c5_split$i.log 2>&1 || exit 1
  timeout -k 10 120 python bench.py --config c5 --cpu-seconds 0 --tune split_lds=1 > gpurun_out/c5_nosplit$i.log 2>&1 || exit 1
done
grep -h -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*' gpurun_out/c5_split*.log gpurun_out/c5_nosplit*.log
