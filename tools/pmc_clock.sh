#!/bin/bash
# effective clock and MFMA busy of the SGD-step kernels (DVFS check): GRBM_GUI_ACTIVE / 8 / duration,
# SQ_VALU_MFMA_BUSY_CYCLES vs the MFMA count; one --pmc pass plus a kernel-trace pass for durations
R=$(pwd)
O=$R/gpurun_out/${1:-pmc_clock}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES --kernel-trace --output-format csv -d $O/pmc -o p -- python3 $R/tools/prof_step.py --sgd 16 > $O/pmc.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 $R/tools/prof_step.py --sgd 16 > $O/trace.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
dur = collections.defaultdict(list)
for f in glob.glob(O + "/trace/*kernel_stats.csv"):
    for row in csv.DictReader(open(f)):
        dur[row["Name"]] = float(row["AverageNs"])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(O + "/pmc/*counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    if not any(x in k for x in ("k_sf_fwd", "k_sf_bwd", "k_sf_dw2", "k_reduce", "k_sf_roll")):
        continue
    m = {c: sum(v) / len(v) for c, v in d.items()}
    ns = dur.get(k)
    line = {c: round(v) for c, v in m.items()}
    if ns:
        line["avg_ns"] = round(ns)
        line["eff_clock_GHz"] = round(m.get("GRBM_GUI_ACTIVE", 0) / 8 / ns, 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            line["mfma_busy_per_simd_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 3)
    print(k[:50], line)
PY
