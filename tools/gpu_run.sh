#!/bin/bash
# GPU-box driver: runs the named steps in order, each under its own time limit, and stops at the
# first failure (no further GPU work after a fault / abort / timeout).
#   tools/gpu_run.sh tests smoke bench prof pmc=<tag>=<counters,...>
set -u
mkdir -p gpurun_out
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[gpu_run] $name: $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[gpu_run] $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
for step in "$@"; do
  case $step in
    tests) run gpu_tests 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ;;
    tests_k=*)  # tests_k=<pytest -k expression>: a subset of the GPU suite
      run gpu_tests_k 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -k "${step#tests_k=}" ;;
    race_probe) run race_probe 900 env MM360_LIB=ab_variants/probe/libmm360.so python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ;;
    probe_ctl)  # positive control: the probe build with the s_ged barriers removed must FAIL (wrong pictures)
      run probe_ctl 300 bash -c 'MM360_LIB=ab_variants/probe_ctl/libmm360.so python -u -m pytest tests/test_gpu.py -q -k "pred_full_frame_vs_oracle or pred_uniform_per_model" --timeout 120 --timeout-method thread; rc=$?; echo "pytest rc=$rc (1 = tests failed as expected)"; test $rc -eq 1' ;;
    abb=*)  # abb=<rounds>=<v1,v2,...>: alternating headline runs of library variants (default = in-tree)
      rounds=$(echo "$step" | cut -d= -f2); vs=$(echo "$step" | cut -d= -f3 | tr ',' ' ')
      run "abb_$(echo "$vs" | tr ' ' '_')" 900 bash tools/ab_bench.sh "$rounds" $vs ;;
    example) run example 120 vvc-extension-mm_amd/lib/example_decode ;;
    dmvrab=*)  # dmvrab=<v1,v2,...>: C3 with a 30 % MM-DMVR share, per library variant (default = in-tree)
      for v in $(echo "$step" | cut -d= -f2 | tr ',' ' '); do
        L=ab_variants/$v/libmm360.so; [ "$v" = default ] && L=vvc-extension-mm_amd/lib/libmm360.so
        run "dmvr_$v" 600 python bench.py --dmvr-share 0.3 --steps 12 --warmup 3 --no-cpu-baseline --no-mvp --no-c5 --lib "$L"
      done ;;
    c5ab=*)  # c5ab=<v1,v2,...>: C5 (Mcandidates/s) of library variants (default = in-tree), one run each
      for v in $(echo "$step" | cut -d= -f2 | tr ',' ' '); do
        L=ab_variants/$v/libmm360.so; [ "$v" = default ] && L=vvc-extension-mm_amd/lib/libmm360.so
        run "c5_$v" 600 python bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --lib "$L"
      done ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench_c4) run bench_c4 600 python bench.py --config C4 ;;
    bench_dmvr) run bench_dmvr 600 python bench.py --dmvr-share 0.3 --cpu-seconds 5 ;;
    bench_c5) run bench_c5 600 python bench.py --config C5 ;;
    prof_dmvr) run prof_dmvr 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dmvr -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --dmvr-share 0.3 --no-mvp --no-c5 ;;
    prof_dmvr0) run prof_dmvr0 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dmvr0 -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --dmvr-share 0.3 --plan-ahead 0 --no-mvp --no-c5 ;;
    prof_c5) run prof_c5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline ;;
    c4_emulate) run c4_emulate 600 python bench.py --config C4 --c4-emulate ;;
    c4_gloo2) run c4_gloo2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 6 --warmup 2 ;;
    per_model) run per_model 900 bash tools/per_model.sh ;;
    coherent) run coherent 600 python bench.py --coherent-mv --steps 20 --warmup 3 --no-cpu-baseline --no-mvp --no-c5 --no-dmvr --no-multi ;;
    ubench) run ubench 300 bash -c "tools/ubench/load_check && tools/ubench/valu_rate2" ;;
    prof_r5) run prof_r5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5 -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-mvp --no-c5 --no-dmvr --no-multi ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 12 --warmup 4 --no-cpu-baseline --no-mvp --no-c5 --no-dmvr --no-multi ;;
    pmc_fetch) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-steps 1 --no-mvp --no-c5 --no-dmvr --no-multi ;;
    pmc_write) run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-steps 1 --no-mvp --no-c5 --no-dmvr --no-multi ;;
    pmc_valu) run pmc_valu 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d gpurun_out/pmc_valu -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-steps 1 --no-mvp --no-c5 --no-dmvr --no-multi ;;
    counters) run counters 300 rocprofv3 -L ;;
    pmc_c5) run pmc_c5 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_c5 -o run --output-format csv -- python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmc_mem) run pmc_mem 600 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_mem -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-steps 1 --no-mvp --no-c5 --no-dmvr --no-multi ;;
    pmc_sq) run pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-steps 1 --no-mvp --no-c5 --no-dmvr --no-multi ;;
    pmc=*)  # pmc=<tag>=<counter,counter,...>: one rocprofv3 --pmc pass over a short bench run
      tag=$(echo "$step" | cut -d= -f2); ctrs=$(echo "$step" | cut -d= -f3 | tr ',' ' ')
      run "pmc_$tag" 600 rocprofv3 --pmc $ctrs -d "gpurun_out/pmc_$tag" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-steps 1 --no-mvp --no-c5 --no-dmvr --no-multi ;;
    pmcv=*)  # pmcv=<tag>=<counter,...>=<v1,v2,...>: one rocprofv3 --pmc pass per library variant (default = in-tree)
      tag=$(echo "$step" | cut -d= -f2); ctrs=$(echo "$step" | cut -d= -f3 | tr ',' ' '); vs=$(echo "$step" | cut -d= -f4 | tr ',' ' ')
      run "pmcv_$tag" 600 bash tools/pmc_variant.sh "$tag" "$ctrs" $vs ;;
    pmcd=*)  # pmcd=<tag>=<counter,...>: one rocprofv3 --pmc pass over a short C3 run with a 30 % MM-DMVR share
      tag=$(echo "$step" | cut -d= -f2); ctrs=$(echo "$step" | cut -d= -f3 | tr ',' ' ')
      run "pmcd_$tag" 600 rocprofv3 --pmc $ctrs -d "gpurun_out/pmcd_$tag" -o run --output-format csv -- python3 bench.py --dmvr-share 0.3 --steps 3 --warmup 1 --no-cpu-baseline --kernel-steps 1 --no-mvp --no-c5 ;;
    pmc5=*)  # pmc5=<tag>=<counter,...>: one rocprofv3 --pmc pass over a short C5 run
      tag=$(echo "$step" | cut -d= -f2); ctrs=$(echo "$step" | cut -d= -f3 | tr ',' ' ')
      run "pmc5_$tag" 600 rocprofv3 --pmc $ctrs -d "gpurun_out/pmc5_$tag" -o run --output-format csv -- python3 bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu_run] all steps ok"
