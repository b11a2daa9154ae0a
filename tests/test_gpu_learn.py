"""GPU parity of GAE (K3), the MLP forward / PPO gradient (K4), Adam, the minibatch gather and one
end-to-end PPO iteration, against the CPU oracle.

Tolerances (north star: "rewards, advantages and gradients within 1e-5 relative"):
  - elementwise outputs (GAE, forward logits/values, Adam): |x - ref| <= 1e-5 * |ref| + atol with
    atol = 1e-5 * max|ref| (fp32 accumulation over K = 256 or T = 128 terms);
  - gradients (sums over the minibatch rows): per tensor, ||g - ref||_2 <= 1e-5 * ||ref||_2 and
    elementwise |g - ref| <= 1e-5 * max|ref| + 1e-5 * |ref|;
  - and, for every fp32 output above, per element (tests/parity.py): over the elements with
    |ref| > 1e-6 max|ref|, the relative error against fp64 no worse than float32 references of the
    same computation (the oracle's fp32 band: three evaluations with hidden units relabelled / rows
    reversed, element-wise worst; the serial fp32 recurrence for GAE) by 4x at p50, p99, p99.9 and
    the maximum, so a near-zero element cannot hide behind max|ref|.  Gradients: 4x pooled at p50 /
    p99 / p99.9; each bias tensor unscaled within 4x at p99 and 8x at the maximum; each weight tensor
    in the cancellation-scaled form within 4x at p99 and 8x at the maximum.
"""
import ctypes as C

import numpy as np
import pytest

import oracle
from parity import close_as_fp32, gae_fp32_serial, grad_close_as_fp32, logp_of

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def close(x, ref, rtol=1e-5):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    atol = rtol * max(1e-30, float(np.abs(ref).max()))
    err = np.abs(x - ref)
    ok = err <= rtol * np.abs(ref) + atol
    assert ok.all(), f"max err {err.max():.3e} vs max|ref| {np.abs(ref).max():.3e}"


# ----------------------------------------------------------------------------- GAE
@pytest.mark.parametrize("T,N,gamma,lam", [(128, 4096, 0.99, 1.0), (64, 1000, 0.995, 0.95), (17, 5, 0.9, 0.0),
                                           (256, 333, 0.99, 1.0), (200, 65, 0.99, 0.9), (1, 40, 0.99, 1.0),
                                           (300, 70, 0.99, 1.0), (4000, 1, 0.99, 1.0), (128, 131072, 0.99, 1.0)])
def test_gae_matches_oracle(T, N, gamma, lam):
    """reverse-scan GAE (T <= 256: 8 / 16-step segments, partial last segment, ragged lane groups)
    and the serial recurrence (T > 256, c1's 4,000-step single lane) vs the float64 oracle"""
    from rlks import _lib

    d = _dev()
    rng = np.random.default_rng(T + N)
    r = rng.random((T, N)).astype(np.float32) * 100
    v = rng.standard_normal((T + 1, N)).astype(np.float32) * 50
    dn = (rng.random((T, N)) < 0.01).astype(np.uint8)
    rt, vt_, dt = (torch.from_numpy(x).to(d) for x in (r, v, dn))
    adv = torch.zeros(T, N, device=d)
    vtg = torch.zeros(T, N, device=d)
    npart = _lib.lib().rlks_gae_partials_count(N)
    part = torch.zeros(npart, 2, dtype=torch.float64, device=d)
    sums = torch.zeros(3, dtype=torch.float64, device=d)
    dyn = torch.zeros(8, device=d)
    _lib.call("rlks_gae", rt.data_ptr(), vt_.data_ptr(), dt.data_ptr(), gamma, lam, T, N, adv.data_ptr(),
              vtg.data_ptr(), part.data_ptr(), None)
    _lib.call("rlks_adv_stats", part.data_ptr(), npart, float(T * N), sums.data_ptr(), None)
    _lib.call("rlks_adv_finalize", sums.data_ptr(), dyn.data_ptr(), None)
    ea, ev = oracle.gae(r, v, dn, gamma, lam)
    fa, fv = gae_fp32_serial(r, v, dn, gamma, lam)
    close_as_fp32(adv.cpu().numpy(), ea, fa)
    close_as_fp32(vtg.cpu().numpy(), ev, fv)
    dd = dyn.cpu().numpy()
    assert abs(dd[0] - ea.mean()) <= 1e-5 * abs(ea).max()
    assert abs(1 / dd[1] - max(1e-4, ea.std())) <= 1e-5 * ea.std()


def test_gae_golden_vectors():
    from conftest import GOLDEN
    from rlks import _lib

    d = _dev()
    g = np.load(GOLDEN / "gae.npz")
    for ci in range(3):
        gamma, lam = g[f"c{ci}_params"]
        r, v, dn = g[f"c{ci}_r"], g[f"c{ci}_v"], g[f"c{ci}_d"]
        T, N = r.shape
        adv = torch.zeros(T, N, device=d)
        vtg = torch.zeros(T, N, device=d)
        rt, vt_, dt = (torch.from_numpy(np.ascontiguousarray(x)).to(d) for x in (r, v, dn))
        _lib.call("rlks_gae", rt.data_ptr(), vt_.data_ptr(), dt.data_ptr(), float(gamma), float(lam), T, N,
                  adv.data_ptr(), vtg.data_ptr(), None, None)
        fa, fv = gae_fp32_serial(r, v, dn, gamma, lam)
        close_as_fp32(adv.cpu().numpy(), g[f"c{ci}_adv"], fa)
        close_as_fp32(vtg.cpu().numpy(), g[f"c{ci}_vt"], fv)


# ----------------------------------------------------------------------------- MLP
def _params(d, seed=0, D=6, A=2, scale_b=0.1, H=None):
    from rlks.policy import PolicyParams

    H = H if H is not None else (256 if (D + 1 <= 32 and A in (2, 4, 8)) else 2048)
    p = PolicyParams(D, H, A, device=d, seed=seed)
    # non-zero biases so that every bias path is exercised
    g = torch.Generator().manual_seed(seed + 1)
    for i in (1, 3, 5, 7, 9, 11):
        v = p.view(i)
        v.copy_((torch.randn(v.shape, generator=g) * scale_b).to(d))
    return p


@pytest.mark.parametrize("n", [1, 31, 1000, 70001])
def test_policy_forward_matches_oracle(n):
    d = _dev()
    p = _params(d, seed=n)
    rng = np.random.default_rng(n)
    obs = rng.random((n, 6)).astype(np.float32)
    lg, v = p.forward(torch.from_numpy(obs).to(d))
    flat = p.flat.cpu().numpy()
    el, ev = oracle.mlp_forward(flat, p.offsets, 6, 256, 2, obs)
    fl, fv = oracle.mlp_forward_fp32_band(flat, p.offsets, 6, 256, 2, obs)
    close(lg.cpu().numpy(), el)
    close(v.cpu().numpy(), ev)
    close_as_fp32(lg.cpu().numpy(), el, fl, what="logits")
    close_as_fp32(v.cpu().numpy(), ev, fv, what="values")


def _minibatch(rows, rng, D=6, A=2, p=None, d=None):
    stride = (D + A + 4 + 3) // 4 * 4
    mb = np.zeros((rows, stride), np.float32)
    mb[:, :D] = rng.random((rows, D))
    if p is not None:  # old logits near the current policy, so that ratios straddle the clip range
        lg, _ = p.forward(torch.from_numpy(mb[:, :D].copy()).to(d))
        lo = lg.cpu().numpy() + rng.standard_normal((rows, A)).astype(np.float32) * 0.3
    else:
        lo = rng.standard_normal((rows, A)).astype(np.float32)
    mb[:, D:D + A] = lo
    mb[:, D + A] = rng.standard_normal(rows) * 3 + 0.5
    mb[:, D + A + 1] = rng.standard_normal(rows) * 2
    act = rng.integers(0, A, rows)
    mb[:, D + A + 3] = act
    lsm = lo - np.log(np.exp(lo - lo.max(1, keepdims=True)).sum(1, keepdims=True)) - lo.max(1, keepdims=True)
    mb[:, D + A + 2] = lsm[np.arange(rows), act]
    return mb


@pytest.mark.parametrize("A", [2, 8])
def test_f16_throughput_mode_gradient(A):
    """RLKS_PRECISION_F16 (the split-fp16 SGD kernels with one product: fp16 operands hi x hi, fp32
    accumulation): a throughput mode below the reference's fp32, never chosen by "auto".  Its gradient
    is within 5e-3 of the fp64 oracle per tensor (norm-wise: fp16's 2^-11 operand rounding), and it is
    not the fp32-accurate result (the mode really drops the lo products)."""
    from rlks import _lib

    d = _dev()
    rows, D = 4096, 3 * A
    p = _params(d, seed=rows + A, D=D, A=A)
    rng = np.random.default_rng(rows)
    mb = _minibatch(rows, rng, D=D, A=A, p=p, d=d)
    dyn = torch.tensor([0.3, 0.7, 0.2, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.01)
    mbt = torch.from_numpy(mb).to(d)
    grads = {}
    for prec in (_lib.RLKS_PRECISION_F16, _lib.RLKS_PRECISION_SF16):
        p.desc.precision = prec
        wsb = C.c_int64()
        _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
        ws = torch.empty(wsb.value, dtype=torch.uint8, device=d)
        grad = torch.zeros(p.padded, device=d)
        _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
                  rows, grad.data_ptr(), None, ws.data_ptr(), ws.numel(), None)
        grads[prec] = grad.cpu().numpy().astype(np.float64)
    eg, _ = oracle.ppo_loss_grad(p.flat.cpu().numpy(), p.offsets, D, 256, A, mb, entropy_coeff=0.01, kl_coeff=0.2,
                                 adv_mean=0.3, adv_inv_std=0.7)
    g16, gsf = grads[_lib.RLKS_PRECISION_F16], grads[_lib.RLKS_PRECISION_SF16]
    assert np.isfinite(g16).all()
    worst = 0.0
    for i, shp in enumerate(p.shapes):
        o, n = p.offsets[i], int(np.prod(shp))
        a, b = g16[o:o + n], eg[o:o + n]
        r = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
        worst = max(worst, r)
        assert r <= 5e-3, (i, r)
        assert np.linalg.norm(gsf[o:o + n] - b) <= 1e-5 * np.linalg.norm(b) + 1e-12, i
    assert worst > 1e-6, worst  # (the one-product mode is not the fp32-accurate kernel)


@pytest.mark.parametrize("A", [2, 8])
def test_sf16_grad_tile_dynamic_range(A):
    """split-fp16 gradient with every other 16-row tile 'quiet': its rows' dlogits / dvalue 2^-20 of the
    others' (old logits = the current ones, standardised advantage and value error scaled by 2^-20),
    so the dZ2 exponents of one F2 row split differ by ~20 (F2 scales a tile's H1 rows
    by the split's smallest dZ2 exponent, pushing a quiet tile's lo plane toward fp16 subnormals).
    Per element against fp64 / fp32 (cancellation-scaled, tests/parity.py) and 1e-5 norm-wise."""
    from rlks import _lib

    d = _dev()
    D, rows = 3 * A, 4096
    p = _params(d, seed=77 + A, D=D, A=A)
    p.desc.precision = 1
    rng = np.random.default_rng(5)
    mb = _minibatch(rows, rng, D=D, A=A, p=p, d=d)
    lg, vv = p.forward(torch.from_numpy(mb[:, :D].copy()).to(d))
    lg, vv = lg.cpu().numpy(), vv.cpu().numpy()
    adv_mean, adv_invstd, klc, tiny = 0.3, 0.7, 0.2, 2.0 ** -20
    quiet = (np.arange(rows) // 16) % 2 == 1
    mb[:, D + A + 1] = vv + rng.standard_normal(rows).astype(np.float32) * 4
    mb[quiet, D:D + A] = lg[quiet]                      # ratio 1, KL gradient 0
    lsm = lg - lg.max(1, keepdims=True)
    lsm = lsm - np.log(np.exp(lsm).sum(1, keepdims=True))
    act = mb[:, D + A + 3].astype(np.int64)
    mb[quiet, D + A + 2] = lsm[quiet, act[quiet]]
    mb[quiet, D + A] = adv_mean + (mb[quiet, D + A] - adv_mean) * tiny
    mb[quiet, D + A + 1] = vv[quiet] + rng.standard_normal(int(quiet.sum())).astype(np.float32) * tiny
    dyn = torch.tensor([adv_mean, adv_invstd, klc, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.0)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
    ws = torch.empty(wsb.value, dtype=torch.uint8, device=d)
    grad = torch.zeros(p.padded, device=d)
    mbt = torch.from_numpy(mb).to(d)
    _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
              rows, grad.data_ptr(), None, ws.data_ptr(), ws.numel(), None)
    g = grad.cpu().numpy()
    kw = dict(kl_coeff=klc, adv_mean=adv_mean, adv_inv_std=adv_invstd)
    eg, est = oracle.ppo_loss_grad(p.flat.cpu().numpy(), p.offsets, D, 256, A, mb, scale=True, **kw)
    eg32 = oracle.ppo_loss_grad_fp32_band(p.flat.cpu().numpy(), p.offsets, D, 256, A, mb, **kw)
    assert np.linalg.norm(g - eg) <= 1e-5 * np.linalg.norm(eg)
    grad_close_as_fp32(g, eg, eg32, p.offsets, p.shapes, scale=est["scale"])


@pytest.mark.parametrize("rows,A,precision", [(256, 2, 0), (4096, 2, 0), (256, 2, 1), (4096, 2, 1), (65536, 2, 1),
                                              (512, 4, 1), (512, 8, 1), (512, 4, 0), (1024, 8, 0)])
def test_ppo_grad_matches_oracle(rows, A, precision):
    """precision 0: fp32 MFMA kernels; 1: split-fp16 MFMA kernels (sgd_sf16.hip) — same 1e-5 bar"""
    from rlks import _lib

    d = _dev()
    D = 3 * A
    p = _params(d, seed=rows + A, D=D, A=A)
    p.desc.precision = precision
    rng = np.random.default_rng(rows)
    mb = _minibatch(rows, rng, D=D, A=A, p=p, d=d)
    # value targets near the current values so that some rows are inside / outside vf_clip
    _, vv = p.forward(torch.from_numpy(mb[:, :D].copy()).to(d))
    mb[:, D + A + 1] = vv.cpu().numpy() + rng.standard_normal(rows).astype(np.float32) * 4
    adv_mean, adv_invstd, klc = 0.3, 0.7, 0.2
    dyn = torch.tensor([adv_mean, adv_invstd, klc, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.01)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
    ws = torch.empty(wsb.value, dtype=torch.uint8, device=d)
    grad = torch.zeros(p.padded, device=d)
    stats = torch.zeros(8, dtype=torch.float64, device=d)
    mbt = torch.from_numpy(mb).to(d)
    _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
              rows, grad.data_ptr(), stats.data_ptr(), ws.data_ptr(), ws.numel(), None)
    g = grad.cpu().numpy()
    eg, est = oracle.ppo_loss_grad(p.flat.cpu().numpy(), p.offsets, D, 256, A, mb, entropy_coeff=0.01,
                                   kl_coeff=klc, adv_mean=adv_mean, adv_inv_std=adv_invstd, scale=True)
    eg32 = oracle.ppo_loss_grad_fp32_band(p.flat.cpu().numpy(), p.offsets, D, 256, A, mb, entropy_coeff=0.01,
                                   kl_coeff=klc, adv_mean=adv_mean, adv_inv_std=adv_invstd)
    grad_close_as_fp32(g, eg, eg32, p.offsets, p.shapes, scale=est["scale"])
    from rlks.policy import TENSOR_NAMES

    for i, (name, _, _) in enumerate(TENSOR_NAMES):
        n = int(np.prod(p.shapes[i]))
        a = g[p.offsets[i]: p.offsets[i] + n]
        b = eg[p.offsets[i]: p.offsets[i] + n]
        assert np.linalg.norm(a - b) <= 1e-5 * np.linalg.norm(b) + 1e-12, name
        close(a, b)
    st = stats.cpu().numpy()
    for k, j in (("policy_loss", 0), ("vf_loss", 1), ("kl", 2), ("entropy", 3)):
        assert abs(st[j] - est[k]) <= 1e-5 * max(abs(est[k]), 1e-3 * rows), k
    assert st[4] == rows


@pytest.mark.parametrize("rows,D,H,A", [(512, 6, 256, 2), (384, 12, 512, 4), (256, 192, 2048, 64), (300, 24, 96, 8),
                                        (8192, 24, 512, 8), (4096, 192, 2048, 64),
                                        (300, 192, 256, 64), (1000, 64, 512, 16)])  # split-K weight gradients;
# obs 192 / 64 at ragged rows: Z1 and dW1 on the pre-split GEMM with zero-padded X / dZ1 plane rows
def test_wide_grad_matches_oracle(rows, D, H, A):
    """generic-width path (wide_mlp.hip: split-fp16 GEMMs with fused epilogues), incl. the c5 shape
    (obs 3 x 64 clusters, 64 actions, hidden 2048) and ragged rows; same 1e-5 bar"""
    from rlks import _lib

    d = _dev()
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
    stats = torch.zeros(8, dtype=torch.float64, device=d)
    mbt = torch.from_numpy(mb).to(d)
    _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
              rows, grad.data_ptr(), stats.data_ptr(), ws.data_ptr(), ws.numel(), None)
    g = grad.cpu().numpy()
    eg, est = oracle.ppo_loss_grad(p.flat.cpu().numpy(), p.offsets, D, H, A, mb, entropy_coeff=0.01,
                                   kl_coeff=klc, adv_mean=adv_mean, adv_inv_std=adv_invstd, scale=True)
    eg32 = oracle.ppo_loss_grad_fp32_band(p.flat.cpu().numpy(), p.offsets, D, H, A, mb, entropy_coeff=0.01,
                                   kl_coeff=klc, adv_mean=adv_mean, adv_inv_std=adv_invstd)
    grad_close_as_fp32(g, eg, eg32, p.offsets, p.shapes, scale=est["scale"])
    from rlks.policy import TENSOR_NAMES

    for i, (name, _, _) in enumerate(TENSOR_NAMES):
        n = int(np.prod(p.shapes[i]))
        a = g[p.offsets[i]: p.offsets[i] + n]
        b = eg[p.offsets[i]: p.offsets[i] + n]
        assert np.linalg.norm(a - b) <= 1e-5 * np.linalg.norm(b) + 1e-12, name
        close(a, b)
    st = stats.cpu().numpy()
    for k, j in (("policy_loss", 0), ("vf_loss", 1), ("kl", 2), ("entropy", 3)):
        assert abs(st[j] - est[k]) <= 1e-5 * max(abs(est[k]), 1e-3 * rows), k
    assert st[4] == rows


@pytest.mark.parametrize("n,D,H,A", [(1000, 192, 2048, 64), (77, 12, 512, 4)])
def test_wide_forward_matches_oracle(n, D, H, A):
    d = _dev()
    p = _params(d, seed=n, D=D, A=A, H=H)
    rng = np.random.default_rng(n)
    obs = rng.random((n, D)).astype(np.float32)
    lg, v = p.forward(torch.from_numpy(obs).to(d))
    el, ev = oracle.mlp_forward(p.flat.cpu().numpy(), p.offsets, D, H, A, obs)
    fl, fv = oracle.mlp_forward_fp32_band(p.flat.cpu().numpy(), p.offsets, D, H, A, obs)
    close(lg.cpu().numpy(), el)
    close(v.cpu().numpy(), ev)
    close_as_fp32(lg.cpu().numpy(), el, fl, what="logits")
    close_as_fp32(v.cpu().numpy(), ev, fv, what="values")


def test_adam_matches_torch():
    from rlks import _lib

    d = _dev()
    rng = np.random.default_rng(0)
    n = 135939 + 61
    p, g = rng.standard_normal(n).astype(np.float32), rng.standard_normal(n).astype(np.float32) * 1e-3
    m, v = rng.standard_normal(n).astype(np.float32) * 1e-4, rng.random(n).astype(np.float32) * 1e-6
    pt, gt, mt, vt = (torch.from_numpy(x.copy()).to(d) for x in (p, g, m, v))
    _lib.call("rlks_adam_step", pt.data_ptr(), gt.data_ptr(), mt.data_ptr(), vt.data_ptr(), n, 3e-4, 0.9, 0.999,
              1e-8, 7, None)
    ep, em, ev = oracle.adam(p, g, m, v, 7, 3e-4)
    close(mt.cpu().numpy(), em, 1e-6)
    close(vt.cpu().numpy(), ev, 1e-6)
    # parameters: the stored value may differ from torch's by the final rounding of p - step
    # (<= 2 ulp of p) plus 1e-5 of the lr-sized update; m and v above agree to 1e-6
    np.testing.assert_allclose(pt.cpu().numpy(), ep, rtol=2.5e-7, atol=1e-5 * 3e-4)


@pytest.mark.parametrize("D,A,T,N", [(6, 2, 128, 4096), (12, 4, 16, 1024), (24, 8, 8, 2048), (192, 64, 4, 512)])
def test_gather_is_a_permutation_per_epoch(D, A, T, N):
    """every epoch's minibatches are a permutation of the train batch, and every record holds its
    source sample's fields (obs, logits, adv, vtarg, logp, action, zero padding) — the row-parallel
    gather (records of 12 / 20 / 36 floats) and the element-parallel one (wide records)"""
    from rlks import _lib

    d = _dev()
    S = T * N
    g = torch.Generator(device=d).manual_seed(D)
    f32 = dict(dtype=torch.float32, device=d)
    b = {"obs": torch.rand(T + 1, N, D, generator=g, **f32), "logits": torch.randn(T, N, A, generator=g, **f32),
         "values": torch.zeros(T + 1, N, **f32),
         "actions": torch.randint(0, A, (T, N), generator=g, dtype=torch.int32, device=d),
         "logp": torch.randn(T, N, generator=g, **f32), "rewards": torch.zeros(T, N, **f32),
         "dones": torch.zeros(T, N, dtype=torch.uint8, device=d),
         "adv": torch.arange(S, dtype=torch.float64, device=d).float().view(T, N),
         "vtarg": torch.randn(T, N, generator=g, **f32)}
    rb = _lib.RolloutBufs(*[b[k].data_ptr() for k in ("obs", "logits", "values", "actions", "logp", "rewards",
                                                       "dones", "adv", "vtarg")], T, N)
    desc = _lib.MlpDesc(D, 256, A, 0)
    stride = _lib.lib().rlks_minibatch_stride(C.byref(desc))
    dyn = torch.tensor([0, 1, 0.2, 1, 0, 0, 0, 0], **f32)
    out = torch.zeros(S, stride, **f32)
    mb = min(S, 65536)
    seen = []
    for epoch in range(2):
        out.fill_(-7.0)
        for row0 in range(0, S, mb):
            _lib.call("rlks_ppo_gather", C.byref(desc), C.byref(rb), 77, epoch, row0, mb, dyn.data_ptr(),
                      out[row0:].data_ptr(), None)
        idx = out[:, D + A].double()
        # adv column carries the sample id (exact in fp32 below 2^24)
        assert torch.equal(torch.sort(idx).values, torch.arange(S, dtype=torch.float64, device=d))
        seen.append(idx.clone())
        t, n = idx.long() // N, idx.long() % N
        assert torch.equal(out[:, :D], b["obs"][t, n])
        assert torch.equal(out[:, D:D + A], b["logits"][t, n])
        assert torch.equal(out[:, D + A + 1], b["vtarg"][t, n])
        assert torch.equal(out[:, D + A + 2], b["logp"][t, n])
        assert torch.equal(out[:, D + A + 3], b["actions"][t, n].float())
        assert bool((out[:, D + A + 4:] == 0).all())
    assert not torch.equal(seen[0], seen[1])


@pytest.mark.parametrize("D,A,T,N,groups", [(6, 2, 128, 4096, 1), (6, 2, 16, 1024, 4), (12, 4, 16, 1024, 2),
                                             (24, 8, 8, 2048, 1)])
def test_packed_gather_equals_direct_gather(D, A, T, N, groups):
    """rlks_ppo_pack + rlks_ppo_gather_packed writes exactly the records of rlks_ppo_gather_grouped
    (same permutation per lane group, same fields), bit for bit"""
    from rlks import _lib

    d = _dev()
    S = T * N
    g = torch.Generator(device=d).manual_seed(D + groups)
    f32 = dict(dtype=torch.float32, device=d)
    b = {"obs": torch.randn(T + 1, N, D, generator=g, **f32), "logits": torch.randn(T, N, A, generator=g, **f32),
         "values": torch.zeros(T + 1, N, **f32),
         "actions": torch.randint(0, A, (T, N), generator=g, dtype=torch.int32, device=d),
         "logp": torch.randn(T, N, generator=g, **f32), "rewards": torch.zeros(T, N, **f32),
         "dones": torch.zeros(T, N, dtype=torch.uint8, device=d), "adv": torch.randn(T, N, generator=g, **f32),
         "vtarg": torch.randn(T, N, generator=g, **f32)}
    rb = _lib.RolloutBufs(*[b[k].data_ptr() for k in ("obs", "logits", "values", "actions", "logp", "rewards",
                                                       "dones", "adv", "vtarg")], T, N)
    desc = _lib.MlpDesc(D, 256, A, 0)
    stride = _lib.lib().rlks_minibatch_stride(C.byref(desc))
    ps = _lib.lib().rlks_packed_stride(C.byref(desc))
    assert ps % 16 == 0 and ps >= stride
    packed = torch.full((S, ps), -3.0, **f32)
    _lib.call("rlks_ppo_pack", C.byref(desc), C.byref(rb), packed.data_ptr(), None)
    rows = min(S, 8192)
    ref = torch.zeros(rows, stride, **f32)
    got = torch.full((rows, stride), -5.0, **f32)
    for epoch, row0 in ((0, 0), (3, rows), (9, S - rows)):
        _lib.call("rlks_ppo_gather_grouped", C.byref(desc), C.byref(rb), 1234, epoch, groups, 1, row0, rows, None,
                  ref.data_ptr(), None)
        _lib.call("rlks_ppo_gather_packed", C.byref(desc), packed.data_ptr(), T, N, 1234, epoch, groups, 1, row0,
                  rows, got.data_ptr(), None)
        assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
    assert bool((packed[:, stride:] == 0).all())


@pytest.mark.parametrize("A,f1", [(2, "split"), (8, "split"), (2, "fused")])
def test_fused_sgd_step_equals_grad_then_adam(A, f1, monkeypatch):
    """rlks_ppo_sgd_step (Adam inside the gradient reduction, the next step's weight maxima from
    its slots) and the multi-rank pair rlks_ppo_grad_step + rlks_ppo_adam_apply (an all-reduce goes
    between them) give the parameters, Adam moments and gradients of rlks_ppo_grad + rlks_adam_step,
    bit for bit, over consecutive steps -- including a first step that claims prev_fused with no
    fused predecessor (the device-side tag check falls back to scanning the weights).  f1 = "fused" /
    "split": every call runs the fused F1 kernel (RLKS_F1_FUSED=1) / the two F1 kernels
    (RLKS_F1_SPLIT=1; by default the library fuses them up to 4 actions)"""
    from rlks import _lib
    from rlks.policy import PolicyParams

    d = _dev()
    D, M = 3 * A, 2048
    desc = _lib.MlpDesc(D, 256, A, _lib.RLKS_PRECISION_SF16)
    stride = _lib.lib().rlks_minibatch_stride(C.byref(desc))
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.0)
    g = torch.Generator(device=d).manual_seed(A)
    p_ref = PolicyParams(D, 256, A, device=d, seed=3)
    p_fus = PolicyParams(D, 256, A, device=d, seed=3)
    p_spl = PolicyParams(D, 256, A, device=d, seed=3)
    p_rs = PolicyParams(D, 256, A, device=d, seed=3)  # the split-kernel reference of the multi-rank pair
    p_ref.desc.precision = p_fus.desc.precision = p_spl.desc.precision = _lib.RLKS_PRECISION_SF16
    p_rs.desc.precision = _lib.RLKS_PRECISION_SF16
    P = p_ref.padded
    dyn = torch.tensor([0.1, 1.3, 0.2, 1.0 / M, 0, 0, 0, 0], dtype=torch.float32, device=d)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(desc), M, C.byref(wsb))
    ws_ref = torch.zeros(wsb.value, dtype=torch.uint8, device=d)
    ws_fus = torch.zeros(wsb.value, dtype=torch.uint8, device=d)
    ws_spl = torch.zeros(wsb.value, dtype=torch.uint8, device=d)
    ws_rs = torch.zeros(wsb.value, dtype=torch.uint8, device=d)
    st = {k: torch.zeros(P, device=d) for k in ("m_ref", "v_ref", "g_ref", "m_fus", "v_fus", "g_fus", "m_spl", "v_spl",
                                                 "g_spl", "m_rs", "v_rs", "g_rs")}
    stats_rs = torch.zeros(8, dtype=torch.float64, device=d)
    stats_ref = torch.zeros(8, dtype=torch.float64, device=d)
    stats_fus = torch.zeros(8, dtype=torch.float64, device=d)
    stats_spl = torch.zeros(8, dtype=torch.float64, device=d)
    monkeypatch.setenv("RLKS_F1_FUSED" if f1 == "fused" else "RLKS_F1_SPLIT", "1")
    for step in range(1, 6):
        mb = torch.zeros(M, stride, device=d)
        mb[:, :D] = torch.rand(M, D, generator=g, device=d)
        mb[:, D:D + A] = torch.randn(M, A, generator=g, device=d)
        mb[:, D + A] = torch.randn(M, generator=g, device=d)
        mb[:, D + A + 1] = torch.randn(M, generator=g, device=d) * 30
        mb[:, D + A + 2] = -torch.rand(M, generator=g, device=d) * 2
        mb[:, D + A + 3] = torch.randint(0, A, (M,), generator=g, device=d).float()
        _lib.call("rlks_ppo_grad", C.byref(desc), C.byref(co), p_ref.flat.data_ptr(), dyn.data_ptr(), mb.data_ptr(), M,
                  st["g_ref"].data_ptr(), stats_ref.data_ptr(), ws_ref.data_ptr(), ws_ref.numel(), None)
        _lib.call("rlks_adam_step", p_ref.flat.data_ptr(), st["g_ref"].data_ptr(), st["m_ref"].data_ptr(),
                  st["v_ref"].data_ptr(), P, 3e-3, 0.9, 0.999, 1e-8, step, None)
        _lib.call("rlks_ppo_grad", C.byref(desc), C.byref(co), p_rs.flat.data_ptr(), dyn.data_ptr(), mb.data_ptr(), M,
                  st["g_rs"].data_ptr(), stats_rs.data_ptr(), ws_rs.data_ptr(), ws_rs.numel(), None)
        _lib.call("rlks_adam_step", p_rs.flat.data_ptr(), st["g_rs"].data_ptr(), st["m_rs"].data_ptr(),
                  st["v_rs"].data_ptr(), P, 3e-3, 0.9, 0.999, 1e-8, step, None)
        _lib.call("rlks_ppo_sgd_step", C.byref(desc), C.byref(co), p_fus.flat.data_ptr(), dyn.data_ptr(),
                  mb.data_ptr(), M, st["g_fus"].data_ptr(), stats_fus.data_ptr(), st["m_fus"].data_ptr(),
                  st["v_fus"].data_ptr(), P, 3e-3, 0.9, 0.999, 1e-8, step, 1, ws_fus.data_ptr(), ws_fus.numel(),
                  None)
        _lib.call("rlks_ppo_grad_step", C.byref(desc), C.byref(co), p_spl.flat.data_ptr(), dyn.data_ptr(),
                  mb.data_ptr(), M, st["g_spl"].data_ptr(), stats_spl.data_ptr(), step, 1, ws_spl.data_ptr(),
                  ws_spl.numel(), None)
        g_summed = st["g_spl"].clone()  # what a one-rank all-reduce leaves
        _lib.call("rlks_ppo_adam_apply", C.byref(desc), p_spl.flat.data_ptr(), st["g_spl"].data_ptr(),
                  st["m_spl"].data_ptr(), st["v_spl"].data_ptr(), P, 3e-3, 0.9, 0.999, 1e-8, step, ws_spl.data_ptr(),
                  ws_spl.numel(), M, None)
        assert torch.equal(st["g_spl"].view(torch.int32), g_summed.view(torch.int32)), step
        for ref, sfx in (("ref", "fus"), ("rs", "spl")):
            for k in ("g", "m", "v"):
                assert torch.equal(st[k + "_" + ref].view(torch.int32), st[k + "_" + sfx].view(torch.int32)), (step, k, sfx)
        assert torch.equal(p_ref.flat.view(torch.int32), p_fus.flat.view(torch.int32)), step
        assert torch.equal(p_rs.flat.view(torch.int32), p_spl.flat.view(torch.int32)), step
        assert torch.equal(stats_ref, stats_fus)
        assert torch.equal(stats_rs, stats_spl)


@pytest.mark.parametrize("A,groups", [(2, 1), (4, 2), (2, 16)])
def test_sgd_step_next_equals_step_then_gather(A, groups):
    """rlks_ppo_sgd_step_next (the next minibatch's packed gather run by extra blocks of the step's
    reduce launch, rewriting the minibatch buffer the step just read) leaves the parameters, Adam
    moments, stats and minibatch buffer of rlks_ppo_sgd_step + rlks_ppo_gather_packed, bit for bit,
    over consecutive steps crossing an epoch, and so does the multi-rank form rlks_ppo_grad_step_next
    + rlks_ppo_adam_apply; 16 lane groups exceed the fused form (two launches)"""
    from rlks import _lib
    from rlks.policy import PolicyParams

    d = _dev()
    D, T, N, M = 3 * A, 8, 2048, 2048
    desc = _lib.MlpDesc(D, 256, A, _lib.RLKS_PRECISION_SF16)
    L = _lib.lib()
    stride, ps = L.rlks_minibatch_stride(C.byref(desc)), L.rlks_packed_stride(C.byref(desc))
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.0)
    g = torch.Generator(device=d).manual_seed(groups)
    packed = torch.zeros(T * N, ps, device=d)
    packed[:, :D] = torch.rand(T * N, D, generator=g, device=d)
    packed[:, D:D + A] = torch.randn(T * N, A, generator=g, device=d)
    packed[:, D + A] = torch.randn(T * N, generator=g, device=d)
    packed[:, D + A + 1] = torch.randn(T * N, generator=g, device=d) * 30
    packed[:, D + A + 2] = -torch.rand(T * N, generator=g, device=d) * 2
    packed[:, D + A + 3] = torch.randint(0, A, (T * N,), generator=g, device=d).float()
    dyn = torch.tensor([0.1, 1.3, 0.2, 1.0 / M, 0, 0, 0, 0], dtype=torch.float32, device=d)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(desc), M, C.byref(wsb))
    run = {}
    for k in ("ref", "nxt", "rk"):
        p = PolicyParams(D, 256, A, device=d, seed=5)
        p.desc.precision = _lib.RLKS_PRECISION_SF16
        run[k] = dict(p=p, m=torch.zeros(p.padded, device=d), v=torch.zeros(p.padded, device=d),
                      grad=torch.zeros(p.padded, device=d), ws=torch.zeros(wsb.value, dtype=torch.uint8, device=d),
                      mb=torch.zeros(M, stride, device=d), stats=torch.zeros(6, 8, dtype=torch.float64, device=d))
    seed = 0x1234ABCD
    steps = [(e, b) for e in range(2) for b in range(3)]  # 3 minibatches of the 8 x 2048 batch, 2 epochs

    def gather(r, e, b):
        _lib.call("rlks_ppo_gather_packed", C.byref(desc), packed.data_ptr(), T, N, seed, e, groups, 0, b * M, M,
                  r["mb"].data_ptr(), None)

    def step_args(r, k):
        return (C.byref(desc), C.byref(co), r["p"].flat.data_ptr(), dyn.data_ptr(), r["mb"].data_ptr(), M,
                r["grad"].data_ptr(), r["stats"][k].data_ptr(), r["m"].data_ptr(), r["v"].data_ptr(), r["p"].padded,
                3e-3, 0.9, 0.999, 1e-8, k + 1, int(k > 0))

    ref, nxt, rk = run["ref"], run["nxt"], run["rk"]
    for r in (ref, nxt, rk):
        gather(r, *steps[0])
    for k in range(len(steps)):
        _lib.call("rlks_ppo_sgd_step", *step_args(ref, k), ref["ws"].data_ptr(), ref["ws"].numel(), None)
        x = xr = None
        if k + 1 < len(steps):
            ne, nb = steps[k + 1]
            gather(ref, ne, nb)
            x = C.byref(_lib.GatherNext(packed.data_ptr(), nxt["mb"].data_ptr(), seed, nb * M, T, N, ne, groups, 0, M))
            xr = C.byref(_lib.GatherNext(packed.data_ptr(), rk["mb"].data_ptr(), seed, nb * M, T, N, ne, groups, 0, M))
        _lib.call("rlks_ppo_sgd_step_next", *step_args(nxt, k), x, nxt["ws"].data_ptr(), nxt["ws"].numel(), None)
        # the multi-rank form (one rank: the all-reduce is the identity)
        a = step_args(rk, k)
        _lib.call("rlks_ppo_grad_step_next", *a[:8], k + 1, int(k > 0), xr, rk["ws"].data_ptr(), rk["ws"].numel(),
                  None)
        _lib.call("rlks_ppo_adam_apply", C.byref(desc), rk["p"].flat.data_ptr(), rk["grad"].data_ptr(),
                  rk["m"].data_ptr(), rk["v"].data_ptr(), rk["p"].padded, 3e-3, 0.9, 0.999, 1e-8, k + 1,
                  rk["ws"].data_ptr(), rk["ws"].numel(), M, None)
        for r in (nxt, rk):
            assert torch.equal(ref["mb"].view(torch.int32), r["mb"].view(torch.int32)), k
            assert torch.equal(ref["p"].flat.view(torch.int32), r["p"].flat.view(torch.int32)), k
            for key in ("m", "v", "grad"):
                assert torch.equal(ref[key].view(torch.int32), r[key].view(torch.int32)), (k, key)
    assert torch.equal(ref["stats"], nxt["stats"])
    assert torch.equal(ref["stats"], rk["stats"])


# ----------------------------------------------------------------------------- end to end
def test_ppo_iteration_parity_and_surface(tmp_path):
    """one iteration at the c2 size (4,096 lanes x 128 steps): the fused rollout's env transitions
    replayed bit-exactly by the C oracle, values / GAE vs the oracle, one SGD step's gradient vs the
    fp64 oracle on the gathered minibatch, then the RLlib-style result surface"""
    from rlks import _lib
    from rlks.ppo import PPO, PPOConfig
    from rlks.tables import load_table

    d = _dev()
    N, T = 4096, 128
    cfg = (PPOConfig().environment("K8sMultiCloudEnv").framework("torch")
           .training(train_batch_size=N * T, sgd_minibatch_size=8192, num_sgd_iter=2, lr=3e-4, gamma=0.99)
           .debugging(seed=11))
    cfg.num_envs = N
    algo = PPO(config=cfg, device=d)
    assert algo.T == T and algo.n_mb == 64
    algo.rollout(explore=True)
    b = {k: v.cpu().numpy() for k, v in algo.buf.items()}
    assert set(np.unique(b["actions"])) <= {0, 1} and 0 < b["actions"].mean() < 1
    assert b["dones"].sum() > 0
    # env transitions of the fused kernel == the C oracle fed the same actions (bit-exact)
    tab = load_table()
    ora = oracle.OracleEnv(oracle.make_cfg(N, tab.n_rows, tab.n_clouds, noise_mode=0, seed=11, autoreset=1),
                           tab.cost, tab.latency)
    np.testing.assert_array_equal(ora.reset().view(np.uint32), b["obs"][0].view(np.uint32))
    for t in range(T):
        o, r, term, _, _, _ = ora.step(b["actions"][t])
        np.testing.assert_array_equal(o.view(np.uint32), b["obs"][t + 1].view(np.uint32))
        np.testing.assert_array_equal(r.astype(np.float32).view(np.uint32), b["rewards"][t].view(np.uint32))
        np.testing.assert_array_equal(term, b["dones"][t])
    # logp consistent with the stored logits (per element, against fp64 and fp32 log-softmax)
    close_as_fp32(b["logp"], logp_of(b["logits"], b["actions"]), logp_of(b["logits"], b["actions"], np.float32),
                  what="logp")
    # logits and values of visited observations recomputed by the oracle (fp64, and torch fp32)
    flat = algo.params.flat.cpu().numpy()
    for t in (0, 57, T):
        el, ev = oracle.mlp_forward(flat, algo.params.offsets, 6, 256, 2, b["obs"][t])
        fl, fv = oracle.mlp_forward_fp32_band(flat, algo.params.offsets, 6, 256, 2, b["obs"][t])
        close(b["values"][t], ev)
        close_as_fp32(b["values"][t], ev, fv, what=f"values[{t}]")
        if t < T:
            close(b["logits"][t], el)
            close_as_fp32(b["logits"][t], el, fl, what=f"logits[{t}]")
    algo.advantages()
    ea, evt = oracle.gae(b["rewards"], b["values"], b["dones"], 0.99, 1.0)
    fa, fvt = gae_fp32_serial(b["rewards"], b["values"], b["dones"], 0.99, 1.0)
    close(algo.buf["adv"].cpu().numpy(), ea)
    close(algo.buf["vtarg"].cpu().numpy(), evt)
    close_as_fp32(algo.buf["adv"].cpu().numpy(), ea, fa, what="adv")
    close_as_fp32(algo.buf["vtarg"].cpu().numpy(), evt, fvt, what="vtarg")
    # one SGD step: gradient vs oracle on the gathered minibatch
    _lib.call("rlks_ppo_gather", C.byref(algo.params.desc), C.byref(algo.bufs), 5, 0, 0, algo.mb,
              algo.dyn.data_ptr(), algo.mbuf.data_ptr(), None)
    mb = algo.mbuf.cpu().numpy()
    dyn = algo.dyn.cpu().numpy()
    wsb = algo.ws
    _lib.call("rlks_ppo_grad", C.byref(algo.params.desc), C.byref(algo.coeffs), algo.params.flat.data_ptr(),
              algo.dyn.data_ptr(), algo.mbuf.data_ptr(), algo.mb, algo.grad.data_ptr(), None, wsb.data_ptr(),
              wsb.numel(), None)
    kw = dict(kl_coeff=float(dyn[2]), adv_mean=float(dyn[0]), adv_inv_std=float(dyn[1]))
    eg, est = oracle.ppo_loss_grad(flat, algo.params.offsets, 6, 256, 2, mb, **kw, scale=True)
    eg32 = oracle.ppo_loss_grad_fp32_band(flat, algo.params.offsets, 6, 256, 2, mb, **kw)
    g = algo.grad.cpu().numpy()
    assert np.linalg.norm(g - eg) <= 1e-5 * np.linalg.norm(eg)
    grad_close_as_fp32(g, eg, eg32, algo.params.offsets, algo.params.shapes, scale=est["scale"])
    # full iterations through the RLlib-named surface
    r1 = algo.train()
    r2 = algo.train()
    for r in (r1, r2):
        assert np.isfinite(r["episode_reward_mean"]) and r["episodes_this_iter"] > 0
        assert 3000 < r["episode_reward_mean"] < 6300  # per-step min/max returns bound it
        ls = r["info"]["learner"]["default_policy"]["learner_stats"]
        assert np.isfinite(ls["policy_loss"]) and np.isfinite(ls["vf_loss"]) and ls["kl"] >= 0
    assert r2["training_iteration"] == algo.iteration and r2["timesteps_total"] == algo.samples * algo.iteration
    a0 = algo.compute_single_action(np.full(6, 0.5, np.float32), explore=False)
    path = algo.save(tmp_path)
    algo2 = PPO.from_checkpoint(path, device=d)
    assert torch.equal(algo2.params.flat, algo.params.flat) and algo2.iteration == algo.iteration
    assert algo2.compute_single_action(np.full(6, 0.5, np.float32), explore=False) == a0


@pytest.mark.parametrize("A", [2, 8])
def test_f2_image_kernel_matches_register_kernel(A, monkeypatch):
    """Round 6's F2 (k_sf_dw2r: H1 in registers, [k / 4][n][4] partials, the default) and rounds 3-5's
    (k_sf_dw2: H1 through an LDS image, [n][k] partials; RLKS_F2_IMAGE=1, kept for same-box A/B runs)
    give the same gradient up to the MFMAs' operand roles (the same products, accumulated in another
    order): every tensor within 1e-6 of its norm, dW2 / db2 included, and both are deterministic"""
    from rlks import _lib
    from rlks.policy import TENSOR_NAMES

    d = _dev()
    rows, D = 16384, 3 * A
    p = _params(d, seed=rows + 7 * A, D=D, A=A)
    p.desc.precision = _lib.RLKS_PRECISION_SF16
    mb = _minibatch(rows, np.random.default_rng(rows + 3), D=D, A=A, p=p, d=d)
    mbt = torch.from_numpy(mb).to(d)
    dyn = torch.tensor([0.3, 0.7, 0.2, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.01)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
    ws = torch.zeros(wsb.value, dtype=torch.uint8, device=d)

    def grad():
        g = torch.zeros(p.padded, device=d)
        _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
                  rows, g.data_ptr(), None, ws.data_ptr(), ws.numel(), None)
        torch.cuda.synchronize()
        return g.cpu().numpy()

    gr = [grad(), grad()]
    monkeypatch.setenv("RLKS_F2_IMAGE", "1")
    gi = [grad(), grad()]
    for a, b in (gr, gi):
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    for i, (name, _, _) in enumerate(TENSOR_NAMES):
        o, n = p.offsets[i], int(np.prod(p.shapes[i]))
        a, b = gi[0][o:o + n].astype(np.float64), gr[0][o:o + n].astype(np.float64)
        assert np.linalg.norm(a - b) <= 1e-6 * np.linalg.norm(b) + 1e-12, name


@pytest.mark.parametrize("A", [2, 4, 8])
def test_fused_f1_is_deterministic_and_matches_split_kernels(A, monkeypatch):
    """F1a + F1b as one kernel (k_sf_f1, 16-wave workgroups, one per CU; the
    default up to 4 actions, RLKS_F1_FUSED=1 forces it).  At the c4 minibatch (65,536 rows: two
    rounds of workgroups) three runs are bit for bit the same, and the gradient equals the two split
    kernels' (8-wave workgroups, RLKS_F1_SPLIT=1) up to the order of the workgroup sums (16 waves' slots
    added in LDS instead of 8, and half as many partials).  (The fused kernel on 8-wave workgroups, two per CU, was measured
    non-deterministic in a few tiles a step: DESIGN.md §15.)"""
    from rlks import _lib
    from rlks.policy import TENSOR_NAMES

    d = _dev()
    rows, D = 65536, 3 * A
    p = _params(d, seed=rows + A, D=D, A=A)
    p.desc.precision = _lib.RLKS_PRECISION_SF16
    mb = _minibatch(rows, np.random.default_rng(rows + 1), D=D, A=A, p=p, d=d)
    mbt = torch.from_numpy(mb).to(d)
    dyn = torch.tensor([0.3, 0.7, 0.2, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.01)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
    ws = torch.zeros(wsb.value, dtype=torch.uint8, device=d)

    def grad():
        g = torch.zeros(p.padded, device=d)
        st = torch.zeros(8, dtype=torch.float64, device=d)
        _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
                  rows, g.data_ptr(), st.data_ptr(), ws.data_ptr(), ws.numel(), None)
        torch.cuda.synchronize()
        return g.cpu().numpy(), st.cpu().numpy()

    monkeypatch.setenv("RLKS_F1_SPLIT", "1")
    gs, ss = grad()
    monkeypatch.delenv("RLKS_F1_SPLIT")
    monkeypatch.setenv("RLKS_F1_FUSED", "1")
    runs = [grad() for _ in range(3)]
    for gf, sf in runs[1:]:
        np.testing.assert_array_equal(gf.view(np.uint32), runs[0][0].view(np.uint32))
        np.testing.assert_array_equal(sf.view(np.uint64), runs[0][1].view(np.uint64))
    gf = runs[0][0]
    for i, (name, _, _) in enumerate(TENSOR_NAMES):
        o, n = p.offsets[i], int(np.prod(p.shapes[i]))
        a, b = gf[o:o + n].astype(np.float64), gs[o:o + n].astype(np.float64)
        assert np.linalg.norm(a - b) <= 1e-6 * np.linalg.norm(b) + 1e-12, name
    np.testing.assert_allclose(runs[0][1], ss, rtol=1e-6)
