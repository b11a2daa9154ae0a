#!/bin/bash
# rocprofv3 kernel stats of a short default bench run -> gpurun_out/$1/prof
set -e
O=gpurun_out/${1:-prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
python3 - <<PY
import csv,glob
f=glob.glob("$GRAFT_REPO_ROOT/$O/prof/**/c4_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]: print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e3,1), r["Percentage"])
PY
