#!/bin/bash
# instruction-fetch and wait stalls of F1a (k_sf_fwd): SQ wait and icache counters over tools/prof_step.py
R=$(pwd)
O=$R/gpurun_out/${1:-pmc_ifetch}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for pp in 0; do
  RLKS_F1A_PIPE=$pp timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/sq_p$pp -o p -- python3 $R/tools/prof_step.py --sgd 4 > $O/sq_p$pp.log 2>&1 || exit 1
  RLKS_F1A_PIPE=$pp timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ --output-format csv -d $O/ic_p$pp -o p -- python3 $R/tools/prof_step.py --sgd 4 > $O/ic_p$pp.log 2>&1 || echo "icache pass failed"
done
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for f in sorted(glob.glob(O + "/*/*counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "k_sf_fwd" not in k:
            continue
        acc[k[:40]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, d in acc.items():
        print(f.split("/")[-2], k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
