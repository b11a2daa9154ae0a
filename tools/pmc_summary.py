#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into per-kernel averages.

usage: pmc_summary.py <out.json> <kernel_stats.csv> [<pmc_counter_collection.csv> ...]
Per-dispatch counter values are averaged per kernel name; HBM traffic per launch is derived as the
guide prescribes (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KB) x 1024 x 2 for wide coalesced reads
(gfx950 reports half), WRITE_SIZE (KB) x 1024.
"""
import csv
import json
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").strip()


def main():
    out, stats_csv, pmc_csvs = sys.argv[1], sys.argv[2], sys.argv[3:]
    kern = {}
    for r in csv.DictReader(open(stats_csv)):
        kern[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                  "total_ns": float(r["TotalDurationNs"]), "pct": float(r["Percentage"])}
    per = defaultdict(lambda: defaultdict(list))
    for f in pmc_csvs:
        for r in csv.DictReader(open(f)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in per.items():
        d = kern.setdefault(k, {})
        for c, v in cs.items():
            d[c] = sum(v) / len(v)
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
    json.dump(kern, open(out, "w"), indent=1, sort_keys=True)
    for k, d in sorted(kern.items(), key=lambda kv: -kv[1].get("total_ns", 0))[:14]:
        print(f"{k[:48]:48s} calls={d.get('calls', 0):6d} avg_us={d.get('avg_ns', 0) / 1e3:9.2f} "
              f"pct={d.get('pct', 0):5.1f} rd={d.get('hbm_read_bytes_corrected', 0) / 1e6:8.2f}MB "
              f"wr={d.get('hbm_write_bytes', 0) / 1e6:8.2f}MB")


if __name__ == "__main__":
    main()
