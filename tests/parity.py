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


def assert_pcts(e, e32, factor=4.0, what="", max_factor=None):
    if e.size == 0:
        return
    for q in QS:
        a, b = np.percentile(e, q), np.percentile(e32, q)
        f = max_factor if (q == 100 and max_factor is not None) else factor
        assert a <= f * b + ULP2, f"{what} p{q}: {a:.3e} vs fp32 {b:.3e} (worst element {int(e.argmax())})"


def close_as_fp32(x, ref64, ref32, factor=4.0, floor=1e-6, what="", max_factor=8.0):
    """element-wise relative error of x against the float64 reference no worse than the float32
    reference's by `factor` at the 50th / 99th / 99.9th percentiles and by `max_factor` at the
    maximum: the worst element of a sample sits where the sum cancels (a logit or value near zero),
    and there the fp32 reference's own error is a matter of luck as much as of precision (the same
    reasoning as grad_close_as_fp32's per-tensor maximum)"""
    e, e32 = rel_errors(x, ref64, ref32, floor)
    assert_pcts(e, e32, factor, what, max_factor)


def grad_close_as_fp32(g, g64, g32, offsets, shapes, factor=4.0, floor=1e-6, scale=None, tensor_factor=4.0,
                       tensor_max_factor=8.0):
    """the gradient form of test_sf16_gradient_per_element.

    Pooled over all parameter tensors (the floor relative to each tensor's own max): the relative
    error |g - g64| / |g64| no worse than the fp32 reference's by `factor` at p50 / p99 / p99.9.

    Per tensor, every element against its own cancellation scale s (oracle.ppo_loss_grad(...,
    scale=True): the sum over the minibatch rows of the absolute per-row terms of that element):
    |g - g64| / s at p99 within `tensor_factor` and at the maximum within `tensor_max_factor` of the
    fp32 reference's.  A gradient element is a sum over the rows; where the rows cancel (|g64| << s,
    typical of bias gradients under PPO's advantage standardisation) the relative error of any
    floating-point evaluation is the per-row error times s / |g64|, so the relative error's extreme
    elements compare the two evaluations' luck at cancellation points, not their precision; the
    scaled error is what a summation's error bound is proportional to (not asked to beat 2^-22 of
    it: the split-fp16 representation's own error per row term).  Without `scale`, the per-tensor
    checks use the relative error (p99 within 6x, max within 10x)."""
    es, e32s = [], []
    for i, shp in enumerate(shapes):
        o, n = offsets[i], int(np.prod(shp))
        e, e32 = rel_errors(g[o:o + n], g64[o:o + n], g32[o:o + n], floor)
        es.append(e)
        e32s.append(e32)
        if scale is not None:
            s = np.asarray(scale[o:o + n], np.float64)
            keep = s > 0
            es_ = np.abs(np.asarray(g[o:o + n], np.float64) - g64[o:o + n])[keep] / s[keep]
            e32_ = np.abs(np.asarray(g32[o:o + n], np.float64) - g64[o:o + n])[keep] / s[keep]
            pf, mf = tensor_factor, tensor_max_factor
        else:
            es_, e32_ = e, e32
            pf, mf = 6.0, 10.0
        if es_.size:
            assert es_.max() <= mf * e32_.max() + ULP2, \
                f"tensor {i} max: {es_.max():.3e} vs fp32 {e32_.max():.3e}{' (scaled)' if scale is not None else ''}"
            if es_.size >= 100:
                a, b = np.percentile(es_, 99), np.percentile(e32_, 99)
                assert a <= pf * b + ULP2, \
                    f"tensor {i} p99: {a:.3e} vs fp32 {b:.3e}{' (scaled)' if scale is not None else ''}"
    e, e32 = np.concatenate(es), np.concatenate(e32s)
    for q in QS[:-1]:
        a, b = np.percentile(e, q), np.percentile(e32, q)
        assert a <= factor * b + ULP2, f"pooled p{q}: {a:.3e} vs fp32 {b:.3e}"


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
