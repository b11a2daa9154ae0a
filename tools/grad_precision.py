#!/usr/bin/env python3
"""Per-tensor precision of the SGD-step gradient against the float64 oracle, beside a float32
reference band of the same computation (oracle.ppo_loss_grad_fp32_band, element-wise worst of
three fp32 evaluations; the diagnostic behind tests/parity.py's bias-tensor checks).

  RLKS_LIB=<variant .so> python3 tools/grad_precision.py [--quick] [--json out.json]

For every parameter tensor: the unscaled relative error |g - g64| / |g64| over the elements with
|g64| > 1e-6 max|g64| at the maximum and p99, the fp32 reference's, and their ratios (against the band
and, beside it, against a single plain fp32 evaluation: VERDICT r05 item 7); and the
cancellation-scaled maximum (|g - g64| / sum_rows |terms|).  Test infrastructure (imports the
oracle); never part of the product path."""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "rl-k8s-scheduler_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import oracle  # noqa: E402
from test_gpu_learn import _minibatch, _params  # noqa: E402

CASES = [  # (path, rows, D, H, A)
    ("sf16", 65536, 6, 256, 2), ("sf16", 4096, 6, 256, 2), ("sf16", 512, 12, 256, 4), ("sf16", 512, 24, 256, 8),
    ("wide", 256, 192, 2048, 64), ("wide", 8192, 24, 512, 8), ("wide", 4096, 192, 2048, 64),
]


def run_case(path, rows, D, H, A, seed_off=0):
    from rlks import _lib
    from rlks.policy import TENSOR_NAMES

    d = torch.device("cuda", 0)
    p = _params(d, seed=rows + (A if path == "sf16" else H) + seed_off, D=D, A=A, H=H)
    p.desc.precision = 1 if path == "sf16" else _lib.RLKS_PRECISION_WIDE
    # inputs and oracle results cached per case, so that every library variant sees the same
    # minibatch (its generation runs the library's forward) and the oracle runs once
    cache = Path(os.environ.get("TMPDIR", "/tmp")) / "rlks_grad_precision_cache" / f"{path}_{rows}_{D}_{H}_{A}_{seed_off}.npz"
    z = np.load(cache) if cache.exists() else None
    if z is not None and "band" not in z:  # a cache from before the fp32 band: rebuild it
        z = None
    if z is not None:
        mb = z["mb"]
    else:
        rng = np.random.default_rng(rows + (0 if path == "sf16" else H) + seed_off)
        mb = _minibatch(rows, rng, D=D, A=A, p=p, d=d)
        _, vv = p.forward(torch.from_numpy(mb[:, :D].copy()).to(d))
        mb[:, D + A + 1] = vv.cpu().numpy() + rng.standard_normal(rows).astype(np.float32) * 4
    adv_mean, adv_invstd, klc = 0.3, 0.7, 0.2
    dyn = torch.tensor([adv_mean, adv_invstd, klc, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.01)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
    ws = torch.empty(wsb.value, dtype=torch.uint8, device=d)
    grad = torch.zeros(p.padded, device=d)
    mbt = torch.from_numpy(mb).to(d)
    _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
              rows, grad.data_ptr(), None, ws.data_ptr(), ws.numel(), None)
    g = grad.cpu().numpy().astype(np.float64)
    kw = dict(entropy_coeff=0.01, kl_coeff=klc, adv_mean=adv_mean, adv_inv_std=adv_invstd)
    flat = p.flat.cpu().numpy()
    if z is not None:
        eg, est, band = z["eg"], {"scale": z["scale"]}, list(z["band"])
    else:
        eg, est = oracle.ppo_loss_grad(flat, p.offsets, D, H, A, mb, scale=True, **kw)
        band = oracle.ppo_loss_grad_fp32_band(flat, p.offsets, D, H, A, mb, **kw)
        cache.parent.mkdir(parents=True, exist_ok=True)
        np.savez(cache, mb=mb, eg=eg, scale=est["scale"], band=np.stack(band))
    out = []
    for i, (name, kind, net) in enumerate(TENSOR_NAMES):
        o, n = p.offsets[i], int(np.prod(p.shapes[i]))
        a, b = g[o:o + n], eg[o:o + n]
        c = [np.asarray(r[o:o + n], np.float64) for r in band]
        s = np.asarray(est["scale"][o:o + n], np.float64)
        keep = np.abs(b) > 1e-6 * np.abs(b).max()
        e = np.abs(a - b)[keep] / np.abs(b[keep])
        e32 = np.max([np.abs(r - b)[keep] for r in c], axis=0) / np.abs(b[keep])
        e1 = np.abs(c[0] - b)[keep] / np.abs(b[keep])  # one plain fp32 evaluation (the band's first)
        ks = s > 0
        es = np.abs(a - b)[ks] / s[ks]
        es32 = np.max([np.abs(r - b)[ks] for r in c], axis=0) / s[ks]
        rec = {"tensor": i, "name": f"{'pi' if net == 0 else 'vf'}.{kind}", "n": int(keep.sum()),
               "rel_max": float(e.max()), "rel_max_fp32": float(e32.max()),
               "rel_p99": float(np.percentile(e, 99)), "rel_p99_fp32": float(np.percentile(e32, 99)),
               "rel_p50": float(np.percentile(e, 50)), "rel_p50_fp32": float(np.percentile(e32, 50)),
               "rel_max_fp32_single": float(e1.max()), "rel_p99_fp32_single": float(np.percentile(e1, 99)),
               "rel_p50_fp32_single": float(np.percentile(e1, 50)),
               "scaled_max": float(es.max()), "scaled_max_fp32": float(es32.max())}
        rec["max_ratio"] = rec["rel_max"] / max(rec["rel_max_fp32"], 1e-30)
        rec["p99_ratio"] = rec["rel_p99"] / max(rec["rel_p99_fp32"], 1e-30)
        rec["scaled_ratio"] = rec["scaled_max"] / max(rec["scaled_max_fp32"], 1e-30)
        rec["max_ratio_single"] = rec["rel_max"] / max(rec["rel_max_fp32_single"], 1e-30)
        rec["p99_ratio_single"] = rec["rel_p99"] / max(rec["rel_p99_fp32_single"], 1e-30)
        out.append(rec)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="the small cases only")
    ap.add_argument("--path", choices=["sf16", "wide"], default=None, help="one path's cases only")
    ap.add_argument("--json", default=None)
    ap.add_argument("--seeds", type=int, default=1)
    args = ap.parse_args()
    res = {"lib": os.environ.get("RLKS_LIB", "librlks.so"), "cases": []}
    for case in CASES:
        if (args.quick and case[1] > 4096) or (args.path and case[0] != args.path):
            continue
        for so in range(args.seeds):
            recs = run_case(*case, seed_off=so)
            res["cases"].append({"case": list(case), "seed_off": so, "tensors": recs})
            print(f"== {case} seed+{so}", flush=True)
            for r in recs:
                flag = " <" if (r["name"].split(".")[1].startswith("b") and (r["max_ratio"] > 8 or r["p99_ratio"] > 4)) else ""
                print(f"  {r['tensor']:2d} {r['name']:6s} max {r['rel_max']:.2e}/{r['rel_max_fp32']:.2e}={r['max_ratio']:6.2f}"
                      f"  p99 {r['rel_p99']:.2e}/{r['rel_p99_fp32']:.2e}={r['p99_ratio']:5.2f}"
                      f"  p50 {r['rel_p50']:.1e}/{r['rel_p50_fp32']:.1e}  scaled {r['scaled_ratio']:5.2f}"
                      f"  | one fp32: max x{r['max_ratio_single']:6.2f} p99 x{r['p99_ratio_single']:5.2f}{flag}", flush=True)
    if args.json:
        Path(args.json).parent.mkdir(parents=True, exist_ok=True)
        Path(args.json).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
