#!/bin/bash
# Kernel statistics of library variants on the C3 DMVR workload (plan-ahead off, so that kernels
# do not overlap):  tools/ab_prof.sh default mc_w3 ...  -> gpurun_out/abp_<variant>/
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in "$@"; do
  L=ab_variants/$v/libmm360.so; [ "$v" = default ] && L=vvc-extension-mm_amd/lib/libmm360.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/abp_$v" -o run --output-format csv -- \
    python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --dmvr-share 0.3 --plan-ahead 0 --no-mvp --no-c5 --lib "$L" \
    > "gpurun_out/abp_$v.log" 2>&1 || exit 1
  echo "ok $v"
done
