#!/bin/bash
# A/B of library variants (tools/build_variant.sh) on the C3 bench: wall time per picture with and
# without plan-ahead, plus a rocprofv3 kernel-statistics pass per variant.
#   [AB_ARGS='extra bench flags'] tools/ab_prof.sh VARIANT...   (results: gpurun_out/abp_<variant>_*.log / _stats.csv)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  lib=tmp_variants/$v/libmm360.so
  for pa in 1 0; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --kernel-steps 6 --no-cpu-baseline --plan-ahead $pa --lib $lib $AB_ARGS \
      > gpurun_out/abp_${v}_pa$pa.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/abp_${v}_pa$pa.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abp_${v}_pa$pa.log').read().strip().splitlines()[-1]); print('$v pa=$pa', d['ms_per_step'], d['stages_ms'])"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_prof_$v -o run --output-format csv -- \
    python3 bench.py --steps 8 --warmup 2 --kernel-steps 2 --no-cpu-baseline --lib $lib $AB_ARGS > gpurun_out/abp_${v}_prof.log 2>&1 \
    || { echo "prof $v failed"; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
f = glob.glob(f"gpurun_out/abp_prof_{v}/**/run_kernel_stats.csv", recursive=True) + glob.glob(f"gpurun_out/abp_prof_{v}/run_kernel_stats.csv")
for r in csv.DictReader(open(f[0])):
    n = r["Name"]
    if "k_" in n and "rocclr" not in n:
        print(f"  {v} {n.split('(')[0].replace('(anonymous namespace)::', '')[:40]:40s} {float(r['AverageNs']) / 1000:8.2f} us x{r['Calls']}")
PY
done
echo "ab_prof done"
