#!/usr/bin/env python3
"""Where the split-fp16 step's layer-1 gradient error comes from: run the SGD
step on the c4-size minibatch, read F1a's dZ2 hand-off back (rlks_debug_sf_handoff) and compare
  (a) the GPU's dZ2 with the float64 oracle's, element by element;
  (b) the GPU's dW1 / db1 with float64 dW1 / db1 computed from the GPU's own dZ2 (F1b's own error);
  (c) float64 dW1 / db1 from the GPU's dZ2 with the oracle's (the error F1a hands to F1b).
Test infrastructure (imports the oracle); not part of the product path."""
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


def pct(e):
    return f"p50 {np.median(e):.2e} p99 {np.percentile(e, 99):.2e} max {e.max():.2e}"


def rel(a, b, floor=1e-6):
    keep = np.abs(b) > floor * np.abs(b).max()
    return np.abs(a - b)[keep] / np.abs(b[keep])


def main(rows=65536, A=2):
    from rlks import _lib

    D, H = 3 * A, 256
    d = torch.device("cuda", 0)
    p = _params(d, seed=rows + A, D=D, A=A)
    p.desc.precision = 1
    rng = np.random.default_rng(rows)
    mb = _minibatch(rows, rng, D=D, A=A, p=p, d=d)
    _, vv = p.forward(torch.from_numpy(mb[:, :D].copy()).to(d))
    mb[:, D + A + 1] = vv.cpu().numpy() + rng.standard_normal(rows).astype(np.float32) * 4
    adv_mean, adv_invstd, klc = 0.3, 0.7, 0.2
    dyn = torch.tensor([adv_mean, adv_invstd, klc, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.01)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
    ws = torch.zeros(wsb.value, dtype=torch.uint8, device=d)
    grad = torch.zeros(p.padded, device=d)
    mbt = torch.from_numpy(mb).to(d)
    _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
              rows, grad.data_ptr(), None, ws.data_ptr(), ws.numel(), None)
    torch.cuda.synchronize()
    ptrs = (C.c_void_p * 4)()
    _lib.call("rlks_debug_sf_handoff", C.byref(p.desc), rows, ws.data_ptr(), ptrs)
    base = ws.data_ptr()
    T = rows // 16
    g = grad.cpu().numpy().astype(np.float64)
    flat = p.flat.cpu().numpy().astype(np.float64)
    kw = dict(entropy_coeff=0.01, kl_coeff=klc, adv_mean=adv_mean, adv_inv_std=adv_invstd)
    eg, _ = oracle.ppo_loss_grad(flat, p.offsets, D, H, A, mb, **kw)
    eg32, _ = oracle.ppo_loss_grad(flat, p.offsets, D, H, A, mb, dtype=np.float32, **kw)
    # exact intermediates (float64 autograd, as the oracle)
    rec = torch.as_tensor(mb.astype(np.float64))
    f = torch.tensor(flat, requires_grad=True)
    x = rec[:, :D]
    inter = []
    for net in (0, 1):
        w1, b1, w2, b2, w3, b3 = oracle._net(torch, f, p.offsets, D, H, A, net)
        z1 = x @ w1.T + b1
        inter.append((z1.detach().numpy(), w2.detach().numpy()))
    # the oracle's dZ2 of both nets: z2.grad from its own autograd pass
    ex = oracle_dz2(flat, p.offsets, D, H, A, mb, kw)
    for net in (0, 1):
        off_dz = ptrs[net] - base
        off_e = ptrs[2 + net] - base
        planes = ws[off_dz: off_dz + T * 16 * H * 2 * 2].view(torch.float16).cpu().numpy().astype(np.float64)
        edz = ws[off_e: off_e + 4 * T].view(torch.int32).cpu().numpy()
        pl = planes.reshape(T, 8, 2, 4, 16, 8)  # tile, s, plane, g, c, j
        # (odd tiles are handed over negated: the rounding-bias cancellation, sgd_sf16.hip tile_sign)
        sgn = np.where(np.arange(T) & 1, -1.0, 1.0)
        v = (pl[:, :, 0] + pl[:, :, 1]) * (sgn * 2.0 ** -edz)[:, None, None, None, None]  # tile, s, g, c, j
        # j -> nt = 2 s + (j >> 2), i = j & 3: n = 16 nt + 4 g + i, m = 16 tile + c
        v = v.reshape(T, 8, 4, 16, 2, 4)  # tile, s, g, c, jh, i
        dz = np.transpose(v, (0, 3, 1, 4, 2, 5)).reshape(rows, H)  # m, (s, jh, g, i) = n
        Z1, W2 = inter[net]
        H1 = np.tanh(Z1)
        dz1 = (dz @ W2) * (1 - H1 ** 2)
        db1, dw1 = dz1.sum(0), dz1.T @ mb[:, :D].astype(np.float64)
        o1, ob = p.offsets[6 * net], p.offsets[6 * net + 1]
        print(f"net {net}: dZ2 (GPU vs fp64)        {pct(rel(dz, ex[net]))}")
        for nm, gpu, mine, o, n in (("b1", g[ob:ob + H], db1, ob, H), ("w1", g[o1:o1 + H * D], dw1.ravel(), o1, H * D)):
            print(f"  {nm}: (b) F1b alone        {pct(rel(gpu, mine))}")
            print(f"  {nm}: (c) F1a's dZ2        {pct(rel(mine, eg[o:o + n]))}")
            print(f"  {nm}:     GPU total        {pct(rel(gpu, eg[o:o + n]))}")
            print(f"  {nm}:     fp32 reference   {pct(rel(eg32[o:o + n].astype(np.float64), eg[o:o + n]))}")


def oracle_dz2(flat, off, D, H, A, mb, kw):
    rec = torch.as_tensor(np.asarray(mb, np.float64))
    f = torch.tensor(flat, requires_grad=True)
    x = rec[:, :D]
    lo = rec[:, D:D + A]
    adv = (rec[:, D + A] - kw["adv_mean"]) * kw["adv_inv_std"]
    vt, lpo_old, act = rec[:, D + A + 1], rec[:, D + A + 2], rec[:, D + A + 3].long()
    outs, z2s = [], []
    for net in (0, 1):
        w1, b1, w2, b2, w3, b3 = oracle._net(torch, f, off, D, H, A, net)
        z2 = torch.tanh(x @ w1.T + b1) @ w2.T + b2
        z2.retain_grad()
        z2s.append(z2)
        outs.append(torch.tanh(z2) @ w3.T + b3)
    lp = torch.log_softmax(outs[0], 1)
    ratio = torch.exp(lp.gather(1, act[:, None])[:, 0] - lpo_old)
    surr = torch.min(adv * ratio, adv * torch.clamp(ratio, 0.7, 1.3))
    lpo = torch.log_softmax(lo, 1)
    kl = (lpo.exp() * (lpo - lp)).sum(1)
    ent = -(lp.exp() * lp).sum(1)
    vf = torch.clamp((outs[1][:, 0] - vt) ** 2, 0, 10.0)
    n = rec.shape[0]
    ((-surr + vf - kw["entropy_coeff"] * ent).sum() / n + kw["kl_coeff"] * kl.sum() / n).backward()
    return [z.grad.numpy() for z in z2s]


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 65536)
