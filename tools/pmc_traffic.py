#!/usr/bin/env python3
"""Write profiles/pmc_traffic.json (read by bench.py for roofline.traffic) from a pmc_summary.py
summary.json: per-launch HBM bytes of the kernels bench.py names, as MI355X_MICROARCH.md §HBM
prescribes (separate --pmc passes; FETCH_SIZE KB x 1024 x 2 for gfx950's half-counted wide
coalesced reads, WRITE_SIZE KB x 1024).

usage: pmc_traffic.py <summary.json> <source-description> [out.json]"""
import json
import sys

# bench.py kernel name -> rocprofv3 kernel-name prefix
NAMES = {"k_sf_f1": "rlks::k_sf_f1<", "k_sf_fwd": "rlks::k_sf_fwd<", "k_sf_split": "rlks::k_sf_split", "k_sf_bwd": "rlks::k_sf_bwd<", "k_sf_dw2": "rlks::k_sf_dw2", "k_reduce": "rlks::k_reduce",
         "k_gather_packed": "rlks::k_gather_packed",
         "k_gae": "rlks::k_gae", "k_fwd_head_pi": "rlks::k_fwd_head<2, 0, 4, 2, 1", "k_dw2": "rlks::k_dw2",
         "k_dh1": "rlks::k_dh1", "k_node_step": "rlks::k_node_step"}


def main():
    summ = json.load(open(sys.argv[1]))
    out = {"source": sys.argv[2]}
    for bench_name, prefix in NAMES.items():
        for k, d in summ.items():
            if k.startswith(prefix) and "hbm_read_bytes_corrected" in d and "hbm_write_bytes" in d:
                out[bench_name] = {"kernel": k, "hbm_read_bytes": d["hbm_read_bytes_corrected"],
                                   "hbm_write_bytes": d["hbm_write_bytes"],
                                   "hbm_bytes_per_launch": d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"],
                                   "avg_us": d.get("avg_us", d.get("avg_ns", 0) / 1e3)}
                break
    dst = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
