#!/usr/bin/env python3
"""Add k_node_step's per-launch HBM traffic (separate --pmc FETCH_SIZE / WRITE_SIZE passes over
tools/node_step_time.py, gfx950 correction FETCH x 2) to profiles/pmc_traffic.json (key k_node_step:
the c3 stationary-churn case bench.py reports traffic for).

usage: pmc_node_traffic.py <fetch counter csv> <write counter csv> <source> [pmc_traffic.json] [--first-half]"""
import collections
import csv
import json
import sys


def per_kernel(path, counter, first_half=False):
    """per-launch average per kernel name; first_half: only the earlier half of the dispatches (a
    node_step_time.py run over both legs runs the stationary one first, under the same kernel name)"""
    d = collections.defaultdict(list)
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        if r["Counter_Name"] == counter and "k_node_step" in r["Kernel_Name"]:
            d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    if first_half:
        d = {k: v[: max(1, len(v) // 2)] for k, v in d.items()}
    return {k: sum(v) / len(v) for k, v in d.items()}


def main():
    half = "--first-half" in sys.argv
    sys.argv = [a for a in sys.argv if a != "--first-half"]
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE", half), per_kernel(sys.argv[2], "WRITE_SIZE", half)
    dst = sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_traffic.json"
    out = json.load(open(dst))
    keep = list(fetch)
    for k in keep[:1]:
        f = fetch[k]
        key = "k_node_step"
        rd, wr = f * 1024 * 2, write.get(k, 0.0) * 1024
        out[key] = {"kernel": k, "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                    "source": sys.argv[3]}
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in out.items() if k.startswith("k_node_step")}, indent=1))


if __name__ == "__main__":
    main()
