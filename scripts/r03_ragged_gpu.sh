#!/bin/bash
# Ragged batches on one GPU: the ragged tests (+ the suites whose oracle comparisons changed),
# then the C3 length-pattern probe and C3 / C2 bench lines.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ragged.py ${TESTS:-} > gpurun_out/rag_tests.log 2>&1 || { tail -40 gpurun_out/rag_tests.log; exit 1; }
tail -3 gpurun_out/rag_tests.log
timeout -k 10 400 python3 -u tools/ragged_probe.py --rounds 2 --steps 40 > gpurun_out/ragged_probe.log 2>&1 || { tail -20 gpurun_out/ragged_probe.log; exit 1; }
grep median gpurun_out/ragged_probe.log
for c in ${CFGS:-c3 c2}; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --cpu-seconds 0 --no-fp32-line > gpurun_out/rag_bench_$c.log 2>&1 || { tail -20 gpurun_out/rag_bench_$c.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/rag_bench_$c.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$c', d['value'], d['ms_per_step'], r['frac'], r.get('step_frac'), r['kernels_avg_us'])
"
done
