#!/bin/bash
# Cost of the skipped rows of a ragged batch: ragged_probe under variant builds (ab/lib_*.so)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/ragged_ab.log
: > $out
for l in ${1:-X0 X1 X2}; do
  echo "== lib $l" >> $out
  TRLX_T5_AMD_LIB=$PWD/ab/lib_$l.so timeout -k 10 300 python3 -u tools/ragged_probe.py --rounds 2 --steps 40 2>/dev/null | grep median >> $out || exit 3
done
cat $out
