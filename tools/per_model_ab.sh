#!/bin/bash
# Per-model k_reproj for library variants: tools/per_model_ab.sh MODEL VARIANT...
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
m=$1; shift
for v in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --kernel-steps 10 --no-cpu-baseline --no-mvp --uniform-model $m \
    --lib ab_variants/$v/libmm360.so > gpurun_out/pm_${v}_$m.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/pm_${v}_$m.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/pm_${v}_$m.log').read().strip().splitlines()[-1]); print('$v model $m', d['value'], d['stages_ms'])"
done
