#!/bin/bash
# SQ wait / instruction-fetch counters of F1a for the libraries named (librlks_xp_<v>.so; "default" =
# librlks.so), each over tools/prof_step.py --sgd 4: tools/pmc_f1a.sh <outdir> <variant>...
R=$(pwd)
O=$R/gpurun_out/$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then L=$R/rl-k8s-scheduler_amd/rlks/librlks.so; else L=$R/rl-k8s-scheduler_amd/rlks/librlks_xp_$v.so; fi
  RLKS_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $O/sq_$v -o p -- python3 $R/tools/prof_step.py --sgd 4 > $O/sq_$v.log 2>&1 || exit 1
  RLKS_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/ic_$v -o p -- python3 $R/tools/prof_step.py --sgd 4 > $O/ic_$v.log 2>&1 || echo "icache pass failed"
done
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for f in sorted(glob.glob(O + "/*/*/*counter_collection.csv") + glob.glob(O + "/*/*counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "k_sf_fwd" not in k:
            continue
        acc[k[:34]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, d in acc.items():
        print(f.split("/")[-3] if f.count("/") > 2 else f, k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
