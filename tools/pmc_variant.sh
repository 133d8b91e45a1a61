#!/bin/bash
# One rocprofv3 --pmc pass per variant over a short C3 bench (no side records):
#   tools/pmc_variant.sh TAG "<counters>" variant...      (variant "default" = the in-tree library)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; ctrs=$2; shift 2
mkdir -p gpurun_out
for v in "$@"; do
  lib=ab_variants/$v/libmm360.so; [ "$v" = default ] && lib=vvc-extension-mm_amd/lib/libmm360.so
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/pmcv_${tag}_$v -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-steps 1 --no-mvp --no-c5 --no-dmvr --no-multi \
    --lib $lib > gpurun_out/pmcv_${tag}_$v.log 2>&1 \
    || { echo "pmc $v failed"; tail -5 gpurun_out/pmcv_${tag}_$v.log; exit 1; }
  echo "== $tag $v"; python3 tools/pmc_summary.py "gpurun_out/pmcv_${tag}_$v/*counter_collection.csv" | grep -A12 "^k_mc_dev"
done
