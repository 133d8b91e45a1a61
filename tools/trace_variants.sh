cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in noatom2 p_noemit; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --kernel-steps 1 --lib tmp_variants/$v/libmm360.so > gpurun_out/tr_$v.log 2>&1 || exit 1
python3 - <<PY
import csv
for r in csv.DictReader(open('gpurun_out/tr_$v/run_kernel_stats.csv')):
    print('$v', r['Name'][:40], r['Calls'], r['AverageNs'])
PY
done
