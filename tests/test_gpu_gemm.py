"""GPU parity of the generic split-fp16 GEMM (csrc/gemm_sf16.hip, the wide-MLP path of config c5)
against float64 numpy, for every transpose combination and epilogue, on ragged sizes (M, N, K not
multiples of the 128 x 128 x 32 tiling) and on a 2048-wide layer.

Tolerance (north star: gradients within 1e-5 relative): |C - ref| <= 1e-5 * max|ref| + 1e-5 * |ref|
and ||C - ref|| <= 1e-5 ||ref||."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _gemm(a, b, *, ta, tb, epi=0, bias=None, aux=None, m, n, k, c_max=False):
    from rlks import _lib

    d = a.device
    c = torch.zeros(m, n, dtype=torch.float32, device=d)
    slots = torch.zeros(3, dtype=torch.int32, device=d)
    _lib.call("rlks_absmax", a.data_ptr(), a.shape[0], a.shape[1], a.shape[1], slots[0:].data_ptr(), None)
    _lib.call("rlks_absmax", b.data_ptr(), b.shape[0], b.shape[1], b.shape[1], slots[1:].data_ptr(), None)
    g = _lib.GemmDesc(a.data_ptr(), b.data_ptr(), c.data_ptr(), bias.data_ptr() if bias is not None else None,
                      aux.data_ptr() if aux is not None else None, m, n, k, a.shape[1], b.shape[1], n,
                      aux.shape[1] if aux is not None else 0, int(ta), int(tb), epi, 0, 0,
                      slots[0:].data_ptr(), slots[1:].data_ptr(), slots[2:].data_ptr() if c_max else None)
    _lib.call("rlks_gemm_sf16", C.byref(g), None)
    return c, slots


def _check(x, ref):
    x = np.asarray(x, np.float64)
    err = np.abs(x - ref)
    scale = np.abs(ref).max()
    assert (err <= 1e-5 * scale + 1e-5 * np.abs(ref)).all(), f"max err {err.max():.3e} vs max|ref| {scale:.3e}"
    assert np.linalg.norm(x - ref) <= 1e-5 * np.linalg.norm(ref)


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("m,n,k", [(300, 200, 70), (128, 64, 2048), (1, 257, 33)])
def test_gemm_matches_fp64(ta, tb, m, n, k):
    d = _dev()
    rng = np.random.default_rng(m * 7 + n + k)
    a = (rng.standard_normal((k, m) if ta else (m, k)) * 0.3).astype(np.float32)
    b = (rng.standard_normal((n, k) if tb else (k, n)) * 1e-4).astype(np.float32)  # small, gradient-like
    c, _ = _gemm(torch.from_numpy(a).to(d), torch.from_numpy(b).to(d), ta=ta, tb=tb, m=m, n=n, k=k)
    ref = (a.T if ta else a).astype(np.float64) @ (b.T if tb else b).astype(np.float64)
    _check(c.cpu().numpy(), ref)


def test_gemm_epilogues():
    from rlks import _lib

    d = _dev()
    rng = np.random.default_rng(5)
    m, n, k = 256, 384, 192
    a = rng.random((m, k)).astype(np.float32)
    w = (rng.standard_normal((n, k)) / np.sqrt(k)).astype(np.float32)
    bias = (rng.standard_normal(n) * 0.1).astype(np.float32)
    z = a.astype(np.float64) @ w.T.astype(np.float64)
    at, wt, bt = (torch.from_numpy(x).to(d) for x in (a, w, bias))
    c, _ = _gemm(at, wt, ta=False, tb=True, epi=_lib.RLKS_GEMM_TANH_BIAS, bias=bt, m=m, n=n, k=k)
    _check(c.cpu().numpy(), np.tanh(z + bias))
    c, _ = _gemm(at, wt, ta=False, tb=True, epi=_lib.RLKS_GEMM_BIAS, bias=bt, m=m, n=n, k=k)
    _check(c.cpu().numpy(), z + bias)
    g = np.tanh(rng.standard_normal((m, n))).astype(np.float32)
    c, slots = _gemm(at, wt, ta=False, tb=True, epi=_lib.RLKS_GEMM_DTANH, aux=torch.from_numpy(g).to(d), m=m, n=n,
                     k=k, c_max=True)
    ref = z * (1 - g.astype(np.float64) ** 2)
    _check(c.cpu().numpy(), ref)
    # the c_max slot holds max |C| (float bits)
    cm = np.array([slots[2].item()], np.int32).view(np.float32)[0]
    assert abs(cm - np.abs(c.cpu().numpy()).max()) == 0
