#!/bin/bash
# fp32-logits experience rows (streaming forward): stream_threads x stream_unroll sweep at C2
# (the GPT path, bench --logits-dtype fp32), two interleaved rounds on one box.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/r03_fp32_fwd_sweep.log
: > $out
for r in 1 2; do
  for thr in 128 256; do
    for un in 2 4 8; do
      line=$(timeout -k 10 200 python3 bench.py --logits-dtype fp32 --steps 100 --warmup 5 --cpu-seconds 0 --no-fp32-line \
             --tune stream_threads=$thr --tune stream_unroll=$un 2>/dev/null | grep '^{') || exit 3
      echo "$line" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('round $r threads $thr unroll $un ms', d['ms_per_step'], 'kern', r['kernels_avg_us'])" | tee -a $out
    done
  done
done
