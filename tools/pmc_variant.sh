#!/bin/bash
# One rocprofv3 --pmc pass per variant over a short C3 bench:  tools/pmc_variant.sh "<counters>" variant...
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ctrs=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  lib=ab_variants/$v/libmm360.so
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/pmcv_$v -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --kernel-steps 1 --lib $lib > gpurun_out/pmcv_$v.log 2>&1 \
    || { echo "pmc $v failed"; tail -5 gpurun_out/pmcv_$v.log; exit 1; }
  echo "== $v"; python3 tools/pmc_summary.py "gpurun_out/pmcv_$v/*counter_collection.csv" | grep -A12 "^k_mc_dev"
done
