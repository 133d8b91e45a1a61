#!/bin/bash
# The MM_RACE_PROBE diagnostic build (csrc/mm_probe.h): every cross-wave LDS store is preceded by a
# poison store and a delay, so a read that is not ordered behind its __syncthreads() reads poison.
#   tools/race_probe.sh build   -> ab_variants/probe/libmm360.so (here, on the CPU)
#   tools/race_probe.sh run     -> the GPU suite on that library (on the GPU box; tools/gpu_run.sh race_probe)
set -e
cd "$(dirname "$0")/.."
case "${1:-}" in
  build) tools/build_variant.sh probe "" -DMM_RACE_PROBE ;;
  run) MM360_LIB=ab_variants/probe/libmm360.so timeout -k 10 900 python -u -m pytest tests -x -v -m gpu \
         --timeout 300 --timeout-method thread ;;
  *) echo "usage: $0 build|run"; exit 2 ;;
esac
