#!/bin/bash
# One rocprofv3 --pmc pass over a short C3 bench run of a library variant:
#   tools/pmc_lib.sh TAG LIB COUNTER...   -> gpurun_out/pmc_TAG/
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; lib=$2; shift 2
timeout -s KILL 120 rocprofv3 --pmc "$@" -d "gpurun_out/pmc_$tag" -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-steps 1 --lib "$lib" > "gpurun_out/pmc_$tag.log" 2>&1
