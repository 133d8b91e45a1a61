#!/bin/bash
# rocprofv3 kernel statistics of library variants (tools/build_variant.sh) on a short C3 bench:
#   tools/trace_variants.sh NAME...   -> gpurun_out/tr_NAME/run_kernel_stats.csv (+ a summary line per kernel)
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel-steps 1 --lib ab_variants/$v/libmm360.so > gpurun_out/tr_$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import csv, sys
v = sys.argv[1]
for r in csv.DictReader(open(f'gpurun_out/tr_{v}/run_kernel_stats.csv')):
    if 'k_' in r['Name']:
        print(v, r['Name'].split('(')[1 if r['Name'].startswith('(') else 0][:30], r['Calls'], r['AverageNs'])
PY
done
