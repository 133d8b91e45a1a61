#!/bin/bash
# C3 bench per stripe count (mm_set_stripes):  tools/ab_stripes.sh 1 2 3 4 ...
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for s in "$@"; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --kernel-steps 3 --no-cpu-baseline --stripes $s > gpurun_out/abs_$s.log 2>&1 || { echo "stripes $s failed"; tail -5 gpurun_out/abs_$s.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abs_$s.log').read().strip().splitlines()[-1]); print('stripes $s', d['value'], d['ms_per_step'])"
done
