#!/bin/bash
# Build the library as of git revision REV into ab_variants/NAME (A/B against older code):
#   tools/build_rev.sh REV NAME
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2
d=ab_variants/$name
rm -rf "$d"; mkdir -p "$d"
git archive "$rev" vvc-extension-mm_amd/csrc include | tar -x -C "$d"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared -mllvm -amdgpu-use-amdgpu-trackers=1 \
  -Wno-unused-function "$d/vvc-extension-mm_amd/csrc/mm_kernels.hip" -o "$d/libmm360.so"
echo "built $d/libmm360.so"
