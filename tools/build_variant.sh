#!/bin/bash
# Build an experimental variant of the library with extra compiler flags / a patched source:
#   tools/build_variant.sh NAME [sed-expression-for-mm_kernels.hip] [extra hipcc flags...]
# Output: ab_variants/NAME/libmm360.so (git-ignored; travels to the GPU box for A/B benches).
set -e
cd "$(dirname "$0")/.."
name=$1; expr=${2:-}; shift; shift || true
d=ab_variants/$name
rm -rf "$d"; mkdir -p "$d/csrc" "$d/include"
cp vvc-extension-mm_amd/csrc/* "$d/csrc/"; cp include/mm360.h "$d/include/"
sed -i 's|"../../include/mm360.h"|"../include/mm360.h"|' "$d"/csrc/*.h "$d"/csrc/*.hip
if [ -n "$expr" ]; then sed -i "$expr" "$d/csrc/mm_kernels.hip" "$d"/csrc/*.h; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fPIC -shared -mllvm -amdgpu-use-amdgpu-trackers=1 \
  -Wno-unused-function "$@" "$d/csrc/mm_kernels.hip" -o "$d/libmm360.so"
echo "built $d/libmm360.so"
