#!/bin/bash
# Per-model stage times on the C3 picture with uniform 16x16 PUs of one motion model each.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for m in 1 2 3 4 5 6 10; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --kernel-steps 10 --no-cpu-baseline --no-mvp --no-c5 --no-dmvr --uniform-model $m > gpurun_out/model_$m.log 2>&1 || { echo "model $m failed"; tail -5 gpurun_out/model_$m.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/model_$m.log').read().strip().splitlines()[-1]); print($m, d['value'], d['stages_ms'])"
done
