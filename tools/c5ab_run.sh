#!/bin/bash
# The ME GPU tests, then C5 (Mcandidates/s) of the in-tree library and the ab_variants/ listed, alternating:
#   tools/c5ab_run.sh [ROUNDS] [variant ...]        (on the GPU box; logs gpurun_out/c5ab_<v>_<round>.log)
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rounds=${1:-2}; shift || true
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "sad_window or sad_pattern" --timeout 120 --timeout-method thread > gpurun_out/me_tests.log 2>&1
tail -1 gpurun_out/me_tests.log
for r in $(seq "$rounds"); do for v in default "$@"; do
  L=ab_variants/$v/libmm360.so; [ "$v" = default ] && L=vvc-extension-mm_amd/lib/libmm360.so
  timeout -k 10 200 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu-baseline --lib "$L" > gpurun_out/c5ab_${v}_$r.log 2>&1
  echo "$v $r $(tail -1 gpurun_out/c5ab_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'])")"
done; done
