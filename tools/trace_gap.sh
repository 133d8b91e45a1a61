#!/bin/bash
# Kernel + HIP-runtime trace of a short C3 bench with and without plan-ahead (host launch times vs
# kernel start times: is the per-picture gap host-bound or a cross-queue wait?).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for pa in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/tg_pa$pa -o run --output-format csv -- \
    python3 bench.py --steps 12 --warmup 3 --kernel-steps 1 --no-cpu-baseline --plan-ahead $pa "$@" \
    > gpurun_out/tg_pa$pa.log 2>&1 || { echo "trace pa=$pa failed"; tail -5 gpurun_out/tg_pa$pa.log; exit 1; }
done
echo "trace_gap done"
