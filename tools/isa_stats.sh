#!/bin/bash
# VGPR / SGPR / spill / instruction counts per kernel of a gfx950 build:  tools/isa_stats.sh [src.hip] [extra flags]
src=$(realpath "${1:-vvc-extension-mm_amd/csrc/mm_kernels.hip}"); shift || true
d=$(mktemp -d)
(cd "$d" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -c "$src" \
  --save-temps -o k.o "$@" 2>/dev/null)
s=$(ls "$d"/*gfx950.s 2>/dev/null); [ -n "$s" ] || { echo "compile failed"; rm -rf "$d"; exit 1; }
awk '/^_Z.*: *;/ {name=$1; n=0} /^\t[sv]_|^\t(global|buffer|ds|flat|scratch)_/ {n++} /-- End function/ {if (name!="") {sub(/^_ZN12_GLOBAL__N_1[0-9]+/,"",name); sub(/E.*/,"",name); ins[name]=n}; name=""}
     /^[ \t]+\.name:/ {kn=$2; sub(/^_ZN12_GLOBAL__N_1[0-9]+/,"",kn); sub(/E.*/,"",kn)}
     /^[ \t]+\.vgpr_count:/ {vg[kn]=$2} /^[ \t]+\.sgpr_count:/ {sg[kn]=$2} /^[ \t]+\.vgpr_spill_count:/ {sp[kn]=$2}
     END {for (k in vg) printf "%-16s vgpr %4d sgpr %4d spill %3d instrs %6d\n", k, vg[k], sg[k], sp[k], ins[k]}' "$s" | sort
rm -rf "$d"
