"""Per-element tolerance helpers shared by the GPU parity tests (no GPU needed to import).

North star: rewards, advantages and gradients within 1e-5 relative.  A float32 computation cannot
meet 1e-5 relative on every element of a sum with cancellation, so a fp32 result is checked element
by element against the float64 oracle *and* against what float32 evaluations of the same computation
achieve on the same inputs: over the elements with |ref| > floor * max|ref|, the relative error is no
worse than the fp32 references' by `factor` at the 50th, 99th and 99.9th percentiles and by
`max_factor` at the maximum.  Unlike a max-normalised bound, a near-zero element cannot hide behind
max|ref|.

"The fp32 references' error" is the largest of a few equally valid fp32 evaluations (oracle.py
ppo_loss_grad_fp32_band / mlp_forward_fp32_band: hidden units relabelled, rows reversed, so every
sum runs in another order), element by element: at an element where a sum cancels, one fp32
evaluation can be exact by luck, and a bound relative to one lucky draw fails an equally accurate
computation about one time in ten (profiles/r05_precision).  A plain array is one evaluation.
"""
import numpy as np

QS = (50, 99, 99.9, 100)
# elementwise outputs and pooled gradients: an fp32 result is not asked to beat ~2 ulp of relative
# error per element (a few-element sample's fp32 reference can be exact by chance); weight gradients,
# cancellation-scaled form: the split representation's own error per row term.  Bias gradients: no floor.
ULP2 = 2.0 ** -22
ULP_OUT = 2.0 ** -24  # bias gradients: half an fp32 ulp, the rounding of the stored result itself
BIAS = (1, 3, 5, 7, 9, 11)  # bias tensors of the flat layout (rlks.policy.TENSOR_NAMES order)


def _band(ref32):
    """element-wise max |.| of the fp32 evaluations' deviations is taken by rel_errors: a list of
    arrays (the band) or one array"""
    return [np.asarray(r, np.float64).ravel() for r in (ref32 if isinstance(ref32, (list, tuple)) else [ref32])]


def rel_errors(x, ref64, ref32, floor=1e-6, single=False):
    """relative errors of x and of the fp32 band (element-wise worst evaluation) over the kept
    elements; single=True also returns those of the band's first (plain) evaluation alone"""
    x, ref64 = (np.asarray(a, np.float64).ravel() for a in (x, ref64))
    band = _band(ref32)
    assert all(x.shape == ref64.shape == r.shape for r in band), (x.shape, ref64.shape, [r.shape for r in band])
    assert np.isfinite(x).all(), "non-finite output"
    keep = np.abs(ref64) > floor * np.abs(ref64).max()
    den = np.abs(ref64[keep])
    e32 = np.max([np.abs(r - ref64)[keep] for r in band], axis=0) / den
    e = np.abs(x - ref64)[keep] / den
    if single:
        return e, e32, np.abs(band[0] - ref64)[keep] / den
    return e, e32


def assert_pcts(e, e32, factor=4.0, what="", max_factor=None, floor=ULP2):
    if e.size == 0:
        return
    for q in QS:
        a, b = np.percentile(e, q), np.percentile(e32, q)
        f = max_factor if (q == 100 and max_factor is not None) else factor
        assert a <= f * b + floor, f"{what} p{q}: {a:.3e} vs fp32 {b:.3e} (worst element {int(e.argmax())})"


def close_as_fp32(x, ref64, ref32, factor=4.0, floor=1e-6, what="", max_factor=4.0):
    """element-wise relative error of x against the float64 reference no worse than the float32
    references' by `factor` at the 50th / 99th / 99.9th percentiles and the maximum (max_factor),
    allowing ~2 fp32 ulp"""
    e, e32 = rel_errors(x, ref64, ref32, floor)
    assert_pcts(e, e32, factor, what, max_factor)


def grad_close_as_fp32(g, g64, g32, offsets, shapes, factor=4.0, floor=1e-6, scale=None, tensor_factor=4.0,
                       tensor_max_factor=8.0):
    """the gradient form of test_sf16_gradient_per_element.  g32: the fp32 band (or one evaluation).

    Pooled over all parameter tensors (the floor relative to each tensor's own max): the relative
    error |g - g64| / |g64| no worse than one plain fp32 evaluation's by `factor` at p50 / p99 and
    than the fp32 band's at p99.9.

    Bias tensors, each on its own and unscaled (a bias gradient is a plain sum over the minibatch
    rows, so a coherent error shows there first: VERDICT r04 item 1): the relative error at p99
    within `tensor_factor` and at the maximum within `tensor_max_factor` of the fp32 references',
    allowing the result's own rounding to fp32 (2^-24) only for tensors of fewer than 100 elements
    (the value head's one-element bias is a lottery below that for the fp32 references as well).

    Weight tensors: every element against its own cancellation scale s (oracle.ppo_loss_grad(...,
    scale=True): the sum over the minibatch rows of the absolute per-row terms of that element):
    |g - g64| / s at p99 within `tensor_factor` and at the maximum within `tensor_max_factor` of the
    fp32 references', not asked to beat 2^-22 of it (the split representation's own error per row
    term).  Without `scale` the weight tensors take the bias tensors' unscaled form."""
    band = _band(g32)
    es, e32s, e1s = [], [], []
    for i, shp in enumerate(shapes):
        o, n = offsets[i], int(np.prod(shp))
        e, e32, e1 = rel_errors(g[o:o + n], g64[o:o + n], [r[o:o + n] for r in band], floor, single=True)
        es.append(e)
        e32s.append(e32)
        e1s.append(e1)
        if scale is not None and i not in BIAS:
            s = np.asarray(scale[o:o + n], np.float64)
            keep = s > 0
            ref = np.asarray(g64[o:o + n], np.float64)[keep]
            es_ = np.abs(np.asarray(g[o:o + n], np.float64)[keep] - ref) / s[keep]
            e32_ = np.max([np.abs(r[o:o + n][keep] - ref) for r in band], axis=0) / s[keep]
            fl, kind = ULP2, " (scaled)"
        else:  # floor, only for a tensor of < 100 elements (the value head's one-element bias): the
            # result's own rounding to fp32, half an ulp, which no fp32 output can beat there
            es_, e32_, fl, kind = e, e32, (ULP_OUT if n < 100 else 0.0), ""
        if es_.size:
            assert es_.max() <= tensor_max_factor * e32_.max() + fl, \
                f"tensor {i} max: {es_.max():.3e} vs fp32 {e32_.max():.3e}{kind}"
            if es_.size >= 100 or i in BIAS:
                a, b = np.percentile(es_, 99), np.percentile(e32_, 99)
                assert a <= tensor_factor * b + fl, f"tensor {i} p99: {a:.3e} vs fp32 {b:.3e}{kind}"
    # pooled: p50 / p99 against the single plain fp32 evaluation (over ~10^5 elements its percentiles
    # are not luck: ADVICE r05), p99.9 against the band
    e, e32, e1 = np.concatenate(es), np.concatenate(e32s), np.concatenate(e1s)
    for q in QS[:-1]:
        a, b = np.percentile(e, q), np.percentile(e1 if q < 99.9 else e32, q)
        assert a <= factor * b, f"pooled p{q}: {a:.3e} vs fp32 {b:.3e}{'' if q < 99.9 else ' (band)'}"


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
