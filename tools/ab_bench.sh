#!/bin/bash
# Alternating headline runs of library variants (no side records):  tools/ab_bench.sh ROUNDS v1 v2 ...
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq "$rounds"); do
  for v in "$@"; do
    L=ab_variants/$v/libmm360.so; [ "$v" = default ] && L=vvc-extension-mm_amd/lib/libmm360.so
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --kernel-steps 4 --no-cpu-baseline --no-mvp --no-c5 --no-dmvr --no-multi \
      --lib "$L" > "gpurun_out/abb_${v}_$r.log" 2>&1 || exit 1
    echo "$v $(tail -1 gpurun_out/abb_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'loop_kmc', d['roofline']['kernel_ms'], d['stages_ms'])")"
  done
done
