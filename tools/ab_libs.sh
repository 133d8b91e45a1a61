#!/bin/bash
# A/B of library variants on the C3 bench with the bench's default settings (plan-ahead on),
# alternating runs: tools/ab_libs.sh NAME... (ab_variants/NAME/libmm360.so)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --kernel-steps 5 --no-cpu-baseline \
      --lib ab_variants/$v/libmm360.so > gpurun_out/abl_${v}_$r.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/abl_${v}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abl_${v}_$r.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['stages_ms'])"
  done
done
