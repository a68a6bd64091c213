#!/bin/bash
# Per-kernel VGPR / occupancy report for one source file (gfx950): "kernel vgpr occ lds".
f=${1:-vocab_rows.hip}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I../../include -c "$f" -o /dev/null \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: //p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' | awk '
  /Function Name:/ {name=$3} /^ *VGPRs:/ {v=$2} /Occupancy/ {occ=$NF} /LDS Size/ {printf "%s vgpr=%s occ=%s lds=%s\n", name, v, occ, $NF}' | c++filt | sed 's/(trlx::[A-Za-z]*Args)//'
