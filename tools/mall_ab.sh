#!/bin/bash
# Is k_mc bound below L1?  The C3 bench with 1 picture (its 2 references, 132 MB padded, stay resident in
# the 256 MB MALL) against 4 rotating pictures (529 MB of references), for the kept one-lane k_mc and
# the paired-lane variant (ab_variants/pair, tools/build_rev.sh exp/mc-pair-lanes pair).
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-mvp "$@" > gpurun_out/mall_$tag.log 2>&1 ||
    { echo "$tag failed"; tail -3 gpurun_out/mall_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/mall_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['stages_ms'])"
}
for round in 1 2; do
  run old_p1_$round --pictures 1
  run pair_p1_$round --pictures 1 --lib ab_variants/pair/libmm360.so
  run old_p4_$round --pictures 4
  run pair_p4_$round --pictures 4 --lib ab_variants/pair/libmm360.so
done
