#!/bin/bash
# round 6 final tree (with F1a's Xa split handed to F2): the suite against the bounds-checking debug
# library, the default bench line, rocprofv3 trace of the bench command (the product suite + smoke:
# profiles/r06_xsp)
O=gpurun_out/r06_final7; mkdir -p $O
RLKS_LIB=$PWD/rl-k8s-scheduler_amd/rlks/librlks_debug.so timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_debug.log 2>&1 || { tail -30 $O/pytest_gpu_debug.log; exit 1; }
tail -1 $O/pytest_gpu_debug.log
timeout -k 10 400 python3 -u bench.py > $O/bench_default.txt 2>&1 || { tail -20 $O/bench_default.txt; exit 1; }
grep '^{' $O/bench_default.txt | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('bench', round(d['value']/1e6,3), 'M', r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us (pipeline', round(r['avg_launch_ms_pipeline']*1e3,1), ') frac', round(r['frac'],3), 'cpu', round(d['cpu_baseline']['value']))"
R=$(pwd)
T=$R/gpurun_out/r06_trace7; mkdir -p $T
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o c4_bench -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
cd $R
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r06_trace7/**/*kernel_stats.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:7]
for r in rows:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us', r['Percentage'])
PY
