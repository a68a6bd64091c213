#!/bin/bash
# Full GPU suite, then bench lines for the listed configs (default c2 c3 c4).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/full_tests.log 2>&1 || { tail -60 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
for c in ${CFGS:-c2 c3 c4}; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 5 --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/chk_bench_$c.log 2>&1 || { tail -20 gpurun_out/chk_bench_$c.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/chk_bench_$c.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; f=d.get('fp32_logits')
        print('$c', d['value'], d['ms_per_step'], r['frac'], r.get('step_frac'), r['kernels_avg_us'], ('fp32', f['ms_per_step'], f['roofline']['kernels_avg_us']) if f else '')
"
done
