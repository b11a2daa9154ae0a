#!/usr/bin/env python3
"""Per-kernel anatomy from tools/pmc_sgd.sh's rocprofv3 passes: duration (kernel trace), effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), MFMA-pipe busy fraction, instruction counts per wave,
wave-cycle split (waiting / issue-stalled / issuing), LDS activity and bank conflicts, and HBM
bytes per launch (FETCH_SIZE x 1024 x 2 for gfx950's half-counted wide reads, WRITE_SIZE x 1024;
MI355X_MICROARCH.md §HBM).  usage: pmc_anatomy.py <dir> [kernel substrings...]"""
import csv
import glob
import json
import sys
from collections import defaultdict

KEEP = ("k_sf_f1", "k_sf_fwd", "k_sf_bwd", "k_sf_dw2", "k_reduce", "k_sf_split", "k_gather")


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main():
    d = sys.argv[1]
    keep = tuple(sys.argv[2:]) or KEEP
    dur = {}
    for f in glob.glob(d + "/trace/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Name"])] = float(r["AverageNs"])
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(d + "/[abcd]/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in per.items():
        if not any(s in k for s in keep):
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        ns = dur.get(k, 0.0)
        res = {"avg_us": ns / 1e3}
        g = m.get("GRBM_GUI_ACTIVE", 0.0) / 8
        if ns and g:
            res["eff_clock_GHz"] = g / ns
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            res["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g)
        waves = m.get("SQ_WAVES", 0.0)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if c in m and waves:
                res[c.lower().replace("sq_insts_", "insts_") + "_per_wave"] = m[c] / waves
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in m:
                    res[c.lower().replace("sq_", "") + "_frac"] = m[c] / wc
            if waves and g:
                res["waves_resident_per_simd"] = wc * 4 / (1024 * g)  # wave-cycles are quad-cycles
        if g and "SQ_LDS_IDX_ACTIVE" in m:
            res["lds_active_per_cu_frac"] = m["SQ_LDS_IDX_ACTIVE"] / (256 * g)
            res["lds_conflict_per_cu_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / (256 * g)
        if "FETCH_SIZE" in m:
            res["hbm_read_bytes_corrected"] = m["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in m:
            res["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        res["counters"] = m
        out[k] = res
    json.dump(out, open(d + "/summary.json", "w"), indent=1, sort_keys=True)
    lines = []
    for k, r in sorted(out.items(), key=lambda kv: -kv[1]["avg_us"]):
        lines.append(k)
        lines.append("   " + "  ".join(f"{a}={v:.4g}" for a, v in r.items() if a != "counters"))
    open(d + "/summary.txt", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
