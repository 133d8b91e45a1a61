#!/bin/bash
# A/B the per-stage device times of library variants (tools/build_variant.sh) on the C3 bench.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --kernel-steps 10 --no-cpu-baseline --lib ab_variants/$v/libmm360.so > gpurun_out/ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['stages_ms'])"
done
