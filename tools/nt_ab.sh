#!/bin/bash
# Non-temporal k_mc output stores (nt) and record loads (ntr) vs the kept library (ab_variants/nt, ntr).
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-mvp "$@" > gpurun_out/nt_$tag.log 2>&1 ||
    { echo "$tag failed"; tail -3 gpurun_out/nt_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/nt_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['stages_ms'])"
}
for round in 1 2; do
  run def_$round --pictures 4
  run nt_$round --pictures 4 --lib ab_variants/nt/libmm360.so
  run ntr_$round --pictures 4 --lib ab_variants/ntr/libmm360.so
done
