#!/bin/bash
# Plan-ahead handoff A/B: MM_AB_HOSTSYNC=1 makes the host wait for the next picture's planning (ev_plan)
# before it issues the context stream's wait, so the runtime can skip the cross-queue barrier packet
# (tools/variants/plan_ahead_hostsync.patch built into ab_variants/hs).
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export TMPDIR=/tmp
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-mvp --lib ab_variants/hs/libmm360.so > gpurun_out/hs_$tag.log 2>&1 ||
    { echo "$tag failed"; tail -3 gpurun_out/hs_$tag.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/hs_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['stages_ms'])"
}
for round in 1 2 3; do
  run def_$round A=1
  run hs_$round MM_AB_HOSTSYNC=1
done
