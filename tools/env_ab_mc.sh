#!/bin/bash
# (the MM_AB_* knobs exist only on branch exp/mc-pair-lanes; profiles/r03_ab_mc_pair.txt)
# A/B of the paired-lane k_mc and the plan-ahead gate position through the library's temporary
# MM_AB_* knobs (mm_create): MM_AB_MC_OLD=1 old one-lane k_mc; MM_AB_GATE=1 gate the next picture's
# planning after k_reproj instead of k_mc; MM_AB_MC_LDS=<bytes> dynamic LDS per k_mc_pair_dev
# workgroup (caps its workgroups per CU, leaving room for the planning kernels).
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-mvp > gpurun_out/abmc_$tag.log 2>&1 ||
    { echo "$tag failed"; tail -3 gpurun_out/abmc_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abmc_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['bit_exact'], d['stages_ms'])"
}
for round in 1 2; do
  run old$round MM_AB_MC_OLD=1
  run pair$round A=1
  run pair_g$round MM_AB_GATE=1
  run pair_g_l3$round MM_AB_GATE=1 MM_AB_MC_LDS=40960
  run pair_g_l4$round MM_AB_GATE=1 MM_AB_MC_LDS=29696
  run pair_g_l5$round MM_AB_GATE=1 MM_AB_MC_LDS=23040
  run pair_l4$round MM_AB_MC_LDS=29696
done
