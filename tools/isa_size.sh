#!/bin/bash
# Instruction count per kernel of the gfx950 build (I-cache footprint check):  tools/isa_size.sh [src.hip]
src=$(realpath "${1:-vvc-extension-mm_amd/csrc/mm_kernels.hip}")
d=$(mktemp -d)
(cd "$d" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -c "$src" \
  --save-temps -o k.o 2>/dev/null)
awk '/^_Z.*: *;/ {name=$1; n=0} /^\t[sv]_|^\t(global|buffer|ds|flat|scratch)_/ {n++} /-- End function/ {if (name!="") {sub(/^_ZN12_GLOBAL__N_1[0-9]+/,"",name); printf "%8d %s\n", n, substr(name,1,40)}; name=""}' "$d"/*gfx950.s
rm -rf "$d"
