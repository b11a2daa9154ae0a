#!/usr/bin/env python3
"""Per-wave phase clocks of the c3 work-list node step (the WL_XP_CLOCK build, RLKS_LIB=.../librlks_xp_CLOCK.so):
s_memrealtime (100 MHz) at kernel entry, after the loads, after the list, after B, before the
counters flush; prints the distributions (us) over the 4 waves of every workgroup of one step."""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))

if __name__ == "__main__":
    import torch
    from rlks import VecK8sMultiCloudEnv, _lib
    from rlks.env import NodeSpec
    from rlks.tables import synthetic_table

    n, Cc, nodes = 65536, 8, 256
    for dp in ("stationary", 0.02):
        spec = NodeSpec(Cc, nodes, arrival_rate=1.0, depart_prob=dp, init_occupancy=0.5)
        venv = VecK8sMultiCloudEnv(n, table=synthetic_table(Cc, 100, seed=42), seed=42, nodes=spec,
                                   device=torch.device("cuda", 0))
        venv.reset()
        acts = [torch.randint(0, Cc, (n,), dtype=torch.int32, device="cuda") for _ in range(8)]
        for t in range(60):
            venv.step(acts[t % 8])
        torch.cuda.synchronize()
        venv.step(acts[0])
        torch.cuda.synchronize()
        nb = n * 8 // 512  # NP = 2: 512 pairs a workgroup
        buf = np.zeros(nb * 4 * 6, dtype=np.uint64)
        _lib.check(_lib.lib().rlks_xp_wl_clock(C.c_void_p(buf.ctypes.data), C.c_size_t(buf.nbytes)))
        c = buf.reshape(nb, 4, 6)[:, :, :5].astype(np.float64) / 100.0  # us
        t0 = c[:, :, 0].min()
        c -= t0
        out = {"depart_prob": spec.depart_prob, "kernel_us": float(c[:, :, 4].max())}
        pct = lambda x: [round(float(np.percentile(x, q)), 2) for q in (0, 10, 50, 90, 99, 100)]
        out["start"] = pct(c[:, :, 0])
        out["loads"] = pct(c[:, :, 1] - c[:, :, 0])
        out["list"] = pct(c[:, :, 2] - c[:, :, 1])
        out["B"] = pct(c[:, :, 3] - c[:, :, 2])
        out["D"] = pct(c[:, :, 4] - c[:, :, 3])
        out["end"] = pct(c[:, :, 4])
        out["life"] = pct(c[:, :, 4] - c[:, :, 0])
        # start time vs block index (dispatch order)
        bs = c[:, 0, 0]
        out["start_by_block_decile"] = [round(float(bs[i * nb // 10:(i + 1) * nb // 10].mean()), 2) for i in range(10)]
        print(json.dumps(out))
        del venv
