#!/bin/bash
# Per-kernel VGPR/SGPR/occupancy report for one source file (gfx950).
f=${1:-vocab_rows.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I../../include -c "$f" -o /dev/null \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: //p' | awk '
  /Function Name/ {name=$3} /VGPRs:/ {v=$2} /AGPRs:/ {ag=$2} /Occupancy/ {occ=$4} /LDS Size/ {lds=$5; printf "%-60s vgpr=%s occ=%s lds=%s\n", name, v, occ, lds}' | c++filt
