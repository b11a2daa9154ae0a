"""Per-element tolerance helpers shared by the GPU parity tests (no GPU needed to import).

North star: rewards, advantages and gradients within 1e-5 relative.  A float32 computation cannot
meet 1e-5 relative on every element of a sum with cancellation, so a fp32 result is checked element
by element against the float64 oracle *and* against what a float32 reference of the same
computation (torch-CPU fp32 / a serial fp32 recurrence) achieves on the same inputs: over the
elements with |ref| > floor * max|ref|, the relative error is no worse than the fp32 reference's by
`factor` at the 50th, 99th and 99.9th percentiles and at the maximum.  Unlike a max-normalised bound,
a near-zero element cannot hide behind max|ref|.
"""
import numpy as np

QS = (50, 99, 99.9, 100)
# an fp32 result is not asked to beat ~2 ulp of relative error per element (a tiny sample's fp32
# reference can be exact by chance)
ULP2 = 2.0 ** -22


def rel_errors(x, ref64, ref32, floor=1e-6):
    x, ref64, ref32 = (np.asarray(a, np.float64).ravel() for a in (x, ref64, ref32))
    assert x.shape == ref64.shape == ref32.shape, (x.shape, ref64.shape, ref32.shape)
    assert np.isfinite(x).all(), "non-finite output"
    keep = np.abs(ref64) > floor * np.abs(ref64).max()
    den = np.abs(ref64[keep])
    return np.abs(x - ref64)[keep] / den, np.abs(ref32 - ref64)[keep] / den


def assert_pcts(e, e32, factor=4.0, what=""):
    if e.size == 0:
        return
    for q in QS:
        a, b = np.percentile(e, q), np.percentile(e32, q)
        assert a <= factor * b + ULP2, f"{what} p{q}: {a:.3e} vs fp32 {b:.3e}"


def close_as_fp32(x, ref64, ref32, factor=4.0, floor=1e-6, what=""):
    """element-wise relative error of x against the float64 reference no worse than the float32
    reference's by `factor` at the 50th / 99th / 99.9th percentiles and the maximum"""
    e, e32 = rel_errors(x, ref64, ref32, floor)
    assert_pcts(e, e32, factor, what)


def grad_close_as_fp32(g, g64, g32, offsets, shapes, factor=4.0, floor=1e-6, tensor_max_factor=10.0):
    """the gradient form of test_sf16_gradient_per_element: over all parameter tensors pooled (the
    floor relative to each tensor's own max), the relative error no worse than the fp32 reference's
    by `factor` at p50 / p99 / p99.9 and the maximum; per tensor, p99 within `factor` (tensors of at
    least 100 elements) and the maximum within `tensor_max_factor` (one worst element of a small
    tensor is a noisy statistic for both precisions)"""
    es, e32s = [], []
    for i, shp in enumerate(shapes):
        o, n = offsets[i], int(np.prod(shp))
        e, e32 = rel_errors(g[o:o + n], g64[o:o + n], g32[o:o + n], floor)
        if e.size:
            assert e.max() <= tensor_max_factor * e32.max() + ULP2, \
                f"tensor {i} max: {e.max():.3e} vs fp32 {e32.max():.3e}"
            if e.size >= 100:
                assert np.percentile(e, 99) <= factor * np.percentile(e32, 99) + ULP2, \
                    f"tensor {i} p99: {np.percentile(e, 99):.3e} vs fp32 {np.percentile(e32, 99):.3e}"
        es.append(e)
        e32s.append(e32)
    assert_pcts(np.concatenate(es), np.concatenate(e32s), factor, "pooled")


def log_softmax(lo, dtype):
    lo = np.asarray(lo, dtype)
    m = lo.max(-1, keepdims=True)
    z = lo - m
    return z - np.log(np.exp(z).sum(-1, keepdims=True))


def logp_of(logits, actions, dtype=np.float64):
    lsm = log_softmax(logits, dtype)
    return np.take_along_axis(lsm, np.asarray(actions)[..., None].astype(np.int64), -1)[..., 0]


def gae_fp32_serial(r, v, dn, gamma, lam):
    """the plain float32 backward recurrence (RLlib's discount_cumsum evaluated in the rollout's
    float32): delta_t = r_t + gamma V_{t+1} (1 - d_t) - V_t, A_t = delta_t + gamma lam (1 - d_t) A_{t+1}"""
    T = r.shape[0]
    f = np.float32
    adv = np.zeros(r.shape, f)
    a = np.zeros(r.shape[1:], f)
    g, gl = f(gamma), f(gamma * lam)
    for t in range(T - 1, -1, -1):
        nd = (1 - dn[t]).astype(f)
        delta = (r[t] + g * v[t + 1] * nd - v[t]).astype(f)
        a = (delta + gl * nd * a).astype(f)
        adv[t] = a
    return adv, (adv + v[:T]).astype(f)
