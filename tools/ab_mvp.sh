#!/bin/bash
# Alternating MM-MVP records of library variants (bench.py's mvp and mvp.in_loop):  tools/ab_mvp.sh ROUNDS v1 v2 ...
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq "$rounds"); do
  for v in "$@"; do
    L=ab_variants/$v/libmm360.so; [ "$v" = default ] && L=vvc-extension-mm_amd/lib/libmm360.so
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --kernel-steps 2 --no-cpu-baseline --no-c5 --no-dmvr \
      --lib "$L" > "gpurun_out/abm_${v}_$r.log" 2>&1 || exit 1
    echo "$v $(tail -1 gpurun_out/abm_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['mvp']; print(d['ms_per_step'], m.get('ms_per_picture'), m.get('kernel_ms'), m['in_loop']['ms_per_picture'])")"
  done
done
