#!/bin/bash
# A/B of mm_set_plan_ahead on the C3 bench (same library, alternating runs):
#   tools/ab_plan_ahead.sh  -> gpurun_out/ab_pa*.log, one summary line per run
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for pa in 0 1; do
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --kernel-steps 5 --no-cpu-baseline --plan-ahead $pa \
      > gpurun_out/ab_pa${pa}_$r.log 2>&1 || { echo "plan-ahead $pa failed"; tail -5 gpurun_out/ab_pa${pa}_$r.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_pa${pa}_$r.log').read().strip().splitlines()[-1]); print('plan_ahead=$pa', d['value'], d['ms_per_step'], d.get('mvp'))"
  done
done
