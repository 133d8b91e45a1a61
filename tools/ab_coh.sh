cd /root/repo
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --kernel-steps 10 --no-cpu-baseline > gpurun_out/coh_a.log 2>&1 && timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --kernel-steps 10 --no-cpu-baseline --coherent-mv > gpurun_out/coh_b.log 2>&1 && tail -1 gpurun_out/coh_a.log | cut -c1-60 && python3 -c "
import json
for f in ('a','b'):
    d=json.loads(open('gpurun_out/coh_'+f+'.log').read().strip().splitlines()[-1]); print(f, d['value'], d['stages_ms'])"
