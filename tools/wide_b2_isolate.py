#!/usr/bin/env python3
"""Where the generic-width step's policy db2 error comes from, at the elements where the rows cancel
(test infrastructure: imports the oracle; never part of the product path).

  python3 tools/wide_b2_isolate.py [--case rows,D,H,A] [--top 5]

Runs tests/test_gpu_learn.py::test_wide_grad_matches_oracle's minibatch through rlks_ppo_grad, reads
the policy net's H2 and dL/dlogits back from the workspace (rlks_debug_wide_bufs) and, for the tensor's
worst elements, recomputes db2 = sum_rows (dout W3)(1 - H2^2) in float64 from
  (h2, dout) in {float64 oracle, GPU} x {float64 oracle, GPU}
so that the error splits into the forward's (H2), the loss's (dout) and the kernel arithmetic's
(GPU db2 - db2(GPU h2, GPU dout))."""
import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "rl-k8s-scheduler_amd", ROOT / "oracle", ROOT / "tests"):
    sys.path.insert(0, str(p))

import torch  # noqa: E402

import oracle  # noqa: E402
from test_gpu_learn import _minibatch, _params  # noqa: E402


def dout64(logits, mb, D, A, adv_mean, adv_invstd, klc, ent_c, clip=0.3, dtype=torch.float64):
    """dL/dlogits of the policy part of oracle.ppo_loss_grad's loss, float64 autograd (or dtype)"""
    rec = torch.as_tensor(np.asarray(mb, np.float64)).to(dtype)
    lg = torch.tensor(np.asarray(logits)).to(dtype).requires_grad_(True)
    lo = rec[:, D:D + A]
    adv = (rec[:, D + A] - adv_mean) * adv_invstd
    logp_old = rec[:, D + A + 2]
    act = rec[:, D + A + 3].long()
    lpa = torch.log_softmax(lg, 1)
    ratio = torch.exp(lpa.gather(1, act[:, None])[:, 0] - logp_old)
    surr = torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip))
    lpo = torch.log_softmax(lo, 1)
    kl = (lpo.exp() * (lpo - lpa)).sum(1)
    ent = -(lpa.exp() * lpa).sum(1)
    n = rec.shape[0]
    ((-surr - ent_c * ent).sum() / n + klc * kl.sum() / n).backward()
    return lg.grad.double().numpy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="256,192,2048,64")
    ap.add_argument("--top", type=int, default=5)
    args = ap.parse_args()
    rows, D, H, A = (int(v) for v in args.case.split(","))
    from rlks import _lib

    d = torch.device("cuda", 0)
    p = _params(d, seed=rows + H, D=D, A=A, H=H)
    p.desc.precision = _lib.RLKS_PRECISION_WIDE
    rng = np.random.default_rng(rows + H)
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
    torch.cuda.synchronize()
    ptrs = (C.c_void_p * 6)()
    _lib.call("rlks_debug_wide_bufs", C.byref(p.desc), rows, ws.data_ptr(), ptrs)

    def fetch(ptr, n):
        base = ws.data_ptr()
        off = ptr - base
        assert 0 <= off and off + 4 * n <= ws.numel()
        return ws[off:off + 4 * n].view(torch.float32).cpu().numpy().astype(np.float64)

    h2g = fetch(ptrs[0], rows * H).reshape(rows, H)
    lgg = fetch(ptrs[1], rows * A).reshape(rows, A)
    dog = fetch(ptrs[2], rows * A).reshape(rows, A)
    g = grad.cpu().numpy().astype(np.float64)
    flat = p.flat.cpu().numpy().astype(np.float64)
    o = p.offsets
    W1 = flat[o[0]:o[0] + H * D].reshape(H, D)
    b1 = flat[o[1]:o[1] + H]
    W2 = flat[o[2]:o[2] + H * H].reshape(H, H)
    b2 = flat[o[3]:o[3] + H]
    W3 = flat[o[4]:o[4] + A * H].reshape(A, H)
    b3 = flat[o[5]:o[5] + A]
    x = mb[:, :D].astype(np.float64)
    h2 = np.tanh(np.tanh(x @ W1.T + b1) @ W2.T + b2)
    lg = h2 @ W3.T + b3
    do = dout64(lg, mb, D, A, adv_mean, adv_invstd, klc, 0.01)
    kw = dict(entropy_coeff=0.01, kl_coeff=klc, adv_mean=adv_mean, adv_inv_std=adv_invstd)
    g64, est = oracle.ppo_loss_grad(flat, o, D, H, A, mb, scale=True, **kw)
    band = oracle.ppo_loss_grad_fp32_band(flat, o, D, H, A, mb, **kw)

    def db2(hh, dd):
        return ((dd @ W3) * (1 - hh * hh)).sum(0)

    ref = g64[o[3]:o[3] + H]
    assert np.allclose(db2(h2, do), ref, rtol=1e-9, atol=1e-15 * np.abs(ref).max())
    e32 = np.max([np.abs(b[o[3]:o[3] + H] - ref) for b in band], axis=0)
    rel = np.abs(g[o[3]:o[3] + H] - ref) / np.abs(ref)
    print(f"case {args.case}: per-row H2 err max {np.abs(h2g - h2).max():.2e}, logits {np.abs(lgg - lg).max():.2e}, "
          f"dout {np.abs(dog - do).max():.2e} (|dout| max {np.abs(do).max():.2e})")
    xt = torch.tensor(x, dtype=torch.float32)
    t32 = lambda a: torch.tensor(a, dtype=torch.float32)  # noqa: E731
    h1_32 = torch.tanh(xt @ t32(W1).T + t32(b1))
    h2_32 = torch.tanh(h1_32 @ t32(W2).T + t32(b2)).double().numpy()
    z2 = np.tanh(x @ W1.T + b1) @ W2.T + b2
    eg2, eh32 = np.abs(h2g - h2), np.abs(h2_32 - h2)
    i = np.unravel_index(eg2.argmax(), eg2.shape)
    print(f"H2 abs err GPU p50/p99/max {np.percentile(eg2, 50):.2e}/{np.percentile(eg2, 99):.2e}/{eg2.max():.2e}; "
          f"torch fp32 {np.percentile(eh32, 50):.2e}/{np.percentile(eh32, 99):.2e}/{eh32.max():.2e}; worst at {i}: z2 {z2[i]:.6g}")
    print(f"dout(GPU logits) vs GPU dout: {np.abs(dout64(lgg, mb, D, A, adv_mean, adv_invstd, klc, 0.01) - dog).max():.2e}")
    do32 = dout64(lg.astype(np.float32), mb, D, A, adv_mean, adv_invstd, klc, 0.01, dtype=torch.float32)
    dor = do.astype(np.float32).astype(np.float64)
    print(f"torch fp32 dout err max {np.abs(do32 - do).max():.2e}, fp32-rounded dout64 {np.abs(dor - do).max():.2e}")
    parts = {"gpu": g[o[3]:o[3] + H], "h2 gpu+dout gpu": db2(h2g, dog), "h2 gpu": db2(h2g, do), "dout gpu": db2(h2, dog),
             "dout torch32": db2(h2, do32), "dout rnd64": db2(h2, dor), "h2 gpu+dout rnd64": db2(h2g, dor)}
    for n in np.argsort(-rel)[:args.top]:
        canc = est["scale"][o[3] + n] / abs(ref[n])
        s = "  ".join(f"{k} {abs(v[n] - ref[n]) / abs(ref[n]):.2e}" for k, v in parts.items())
        print(f"  n {n:5d} cancellation {canc:9.3g}  band {e32[n] / abs(ref[n]):.2e}  {s}")


if __name__ == "__main__":
    main()
