#!/bin/bash
# rocprofv3 kernel stats of the c5 wide gradient (tools/prof_wide.py) per library: prof_wide_ab.sh <lib>...
set -e
R=$(pwd)
O=$R/gpurun_out/prof_wide_ab; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  RLKS_LIB=$R/rl-k8s-scheduler_amd/rlks/$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$L -o w -- python3 $R/tools/prof_wide.py --reps 3 > $O/$L.log 2>&1
  python3 - <<PY
import csv,glob
f=glob.glob("$O/$L/**/w_kernel_stats.csv", recursive=True)[0]
print("$L")
for r in list(csv.DictReader(open(f)))[:18]: print("  ", r["Name"][:58], r["Calls"], round(float(r["AverageNs"])/1e3,1), round(float(r["TotalDurationNs"])/1e6,3))
PY
done
