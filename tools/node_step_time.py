#!/usr/bin/env python3
"""Time the c3 node step alone (bench.py's k_node_step leg: 65,536 envs x 8 clusters x 256 nodes,
graph-replayed), for comparing library builds via RLKS_LIB.  usage: node_step_time.py [stationary|<p> ...]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))

if __name__ == "__main__":
    import torch

    import bench

    class _A:  # the two attributes node_env_timing reads
        device = torch.device("cuda", 0)

    def timed(fn, n=5):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / n

    dps = [a if a == "stationary" else float(a) for a in sys.argv[1:]] or ["stationary", 0.02]
    for dp in dps:
        r = bench.node_env_timing(_A, torch, timed, depart_prob=dp)
        print(json.dumps({k: r[k] for k in ("depart_prob", "ms", "GBps", "frac_hbm")}))
