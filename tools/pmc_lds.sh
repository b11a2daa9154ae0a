#!/bin/bash
# LDS occupancy and bank conflicts of the SGD-step kernels (one --pmc pass) + GRBM_GUI_ACTIVE
R=$(pwd)
O=$R/gpurun_out/${1:-pmc_lds}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA --output-format csv -d $O/pmc -o p -- python3 $R/tools/prof_step.py --sgd 16 > $O/pmc.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(O + "/pmc/*counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in acc.items():
    if not any(x in k for x in ("k_sf_fwd", "k_sf_bwd", "k_sf_dw2", "k_reduce")):
        continue
    m = {c: sum(v) / len(v) for c, v in d.items()}
    line = {c: round(v) for c, v in m.items()}
    g = m.get("GRBM_GUI_ACTIVE", 0) / 8  # per-XCD cycles
    if g:
        line["lds_active_per_cu_frac"] = round(m.get("SQ_LDS_IDX_ACTIVE", 0) / (256 * g), 3)
        line["lds_conflict_per_cu_frac"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / (256 * g), 3)
    print(k[:44], line)
PY
