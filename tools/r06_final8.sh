#!/bin/bash
# round 6 final tree, final bench.py (roofline timing: the tighter of the back-to-back and the raw
# in-pipeline bracket): the default bench line and rocprofv3 trace + stats of the bench command, same box
O=gpurun_out/r06_final8; mkdir -p $O
timeout -k 10 400 python3 -u bench.py > $O/bench_default.txt 2>&1 || { tail -20 $O/bench_default.txt; exit 1; }
grep '^{' $O/bench_default.txt | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('bench', round(d['value']/1e6,3), r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us (back-to-back', round(r.get('avg_launch_ms_back_to_back', r['avg_launch_ms'])*1e3,1), ') frac', round(r['frac'],3), 'cpu', round(d['cpu_baseline']['value']))"
R=$(pwd)
T=$R/gpurun_out/r06_trace8; mkdir -p $T
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o c4_bench -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $T/bench.txt 2>&1 || { tail -20 $T/bench.txt; exit 1; }
cd $R
grep '^{' $T/bench.txt | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('under rocprofv3:', round(d['value']/1e6,3), r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us frac', round(r['frac'],3))"
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r06_trace8/**/*kernel_stats.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:6]
for r in rows:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us', r['Percentage'])
PY
