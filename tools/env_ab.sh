cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
run() { tag=$1; shift; env "$@" timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --kernel-steps 1 --no-cpu-baseline > gpurun_out/env_$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/env_$tag.log; exit 1; }; python3 -c "import json; d=json.loads(open('gpurun_out/env_$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'])"; }
run def A=1
run kpool HSA_KERNARG_POOL_SIZE=33554432
run sigpool ROC_SIGNAL_POOL_SIZE=16384
run aw ROC_ACTIVE_WAIT_TIMEOUT=1000
run def2 A=1
run kpool2 HSA_KERNARG_POOL_SIZE=33554432
run sigpool2 ROC_SIGNAL_POOL_SIZE=16384
run aw2 ROC_ACTIVE_WAIT_TIMEOUT=1000
