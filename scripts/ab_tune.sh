#!/bin/bash
# A/B of bench flag sets (trlx_set_tuning knobs etc.), interleaved rounds in ONE call.
#   bash scripts/ab_tune.sh "<cfg>" <rounds> "name:flags" "name:flags" ...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
cfg=$1; rounds=$2; shift 2
out=gpurun_out/ab_tune.log
: > $out
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    name=${v%%:*}; flags=${v#*:}
    line=$(timeout -k 10 200 python3 bench.py --config $cfg --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line $flags 2>/dev/null | grep '^{') || exit 3
    echo "$line" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('round $r cfg $cfg $name ms', d['ms_per_step'], 'kern', r['kernels_avg_us'])" | tee -a $out
  done
done
