#!/bin/bash
# A/B of library builds (ab/lib_*.so via TRLX_T5_AMD_LIB) on the bench configs, interleaved
# rounds in ONE call on one box.   bash scripts/ab_rows.sh "A B C" "c2 c4" [rounds]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
libs=${1:-"A B"}; cfgs=${2:-"c2"}; rounds=${3:-3}
out=gpurun_out/ab_rows.log
: > $out
for r in $(seq 1 $rounds); do
  for c in $cfgs; do
    for l in $libs; do
      line=$(TRLX_T5_AMD_LIB=$PWD/ab/lib_$l.so timeout -k 10 200 python3 bench.py --config $c --steps 200 --warmup 5 --cpu-seconds 0 --no-fp32-line 2>/dev/null | grep '^{') || exit 3
      echo "$line" | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('round $r cfg $c lib $l ms', d['ms_per_step'], 'kern', r['kernels_avg_us'])" | tee -a $out
    done
  done
done
