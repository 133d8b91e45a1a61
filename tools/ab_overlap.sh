#!/bin/bash
# A/B of the reproj-ahead pipeline (the next picture's k_reproj on the auxiliary stream beside this
# picture's paired k_mc) against the default, alternating runs of the C3 bench (plan-ahead on).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { tag=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --steps 40 --warmup 4 --kernel-steps 2 --no-cpu-baseline --no-mvp --no-c5 > gpurun_out/ov_$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/ov_$tag.log; exit 1; }; python3 -c "import json; d=json.loads(open('gpurun_out/ov_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'], d['stages_ms'])"; }
for r in 1 2; do
  run def$r A=1
  run pair$r MM_AB_PAIR=1
  run ov$r MM_AB_OVERLAP=1
  run ov_lds40k$r MM_AB_OVERLAP=1 MM_AB_MC_LDS=36864
  run ov_lds24k$r MM_AB_OVERLAP=1 MM_AB_MC_LDS=20480
done
