#!/bin/bash
# round 6 evidence on the final tree: rocprofv3 kernel trace + stats of the bench command (c4, the
# default) and the SGD-step PMC anatomy (tools/pmc_sgd.sh: instruction mix, waits, MFMA busy, HBM bytes)
R=$(pwd)
O=$R/gpurun_out/r06_trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c4_bench -- \
  python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench.txt 2>&1 || { tail -20 $O/bench.txt; exit 1; }
cd $R
grep '^{' $O/bench.txt | tail -1 | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']
print('bench', round(d['value']/1e6,3), r['kernel'], round(r['avg_launch_ms']*1e3,1), 'us frac', round(r['frac'],3))"
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r06_trace/**/*kernel_stats.csv', recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:8]
for r in rows:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us', r['Percentage'])
PY
[ -n "$NO_PMC" ] || bash tools/pmc_sgd.sh r06_pmc
