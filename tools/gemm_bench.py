#!/usr/bin/env python3
"""Throughput of the split-fp16 GEMM (csrc/gemm_sf16.hip) at the c5 wide-MLP shapes:
M = 16,384 minibatch rows, hidden 2,048, obs 192.  Prints fp32-equivalent TFLOP/s and the fraction
of the split-fp16 ceiling (2.5 PF dense f16 MFMA / 3 products)."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))


def main():
    import torch
    from rlks import _lib

    d = torch.device("cuda", 0)
    M, H, D = 16384, 2048, 192
    f = dict(dtype=torch.float32, device=d)
    slots = torch.zeros(4, dtype=torch.int32, device=d)
    one = torch.tensor([1.0], **f).view(torch.int32)
    cases = [  # name, A shape, B shape, ta, tb, m, n, k
        ("NT fwd  H1 W2^T", (M, H), (H, H), 0, 1, M, H, H),
        ("NN bwd  dZ2 W2", (M, H), (H, H), 0, 0, M, H, H),
        ("TN grad dZ2^T H1", (M, H), (M, H), 1, 0, H, H, M),
        ("NT fwd  X W1^T", (M, D), (H, D), 0, 1, M, H, D),
    ]
    for name, sa, sb, ta, tb, m, n, k in cases:
        a = torch.randn(*sa, **f) * 0.3
        b = torch.randn(*sb, **f) * 0.02
        c = torch.empty(m, n, **f)
        slots.zero_()
        _lib.call("rlks_absmax", a.data_ptr(), sa[0], sa[1], sa[1], slots[0:].data_ptr(), None)
        _lib.call("rlks_absmax", b.data_ptr(), sb[0], sb[1], sb[1], slots[1:].data_ptr(), None)
        g = _lib.GemmDesc(a.data_ptr(), b.data_ptr(), c.data_ptr(), None, None, m, n, k, sa[1], sb[1], n, 0, ta, tb,
                          0, 0, 0, slots[0:].data_ptr(), slots[1:].data_ptr(), None)
        for _ in range(3):
            _lib.call("rlks_gemm_sf16", C.byref(g), None)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = 20
        for _ in range(reps):
            _lib.call("rlks_gemm_sf16", C.byref(g), None)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        tf = 2.0 * m * n * k / (ms * 1e-3) / 1e12
        print(f"{name:20s} {m}x{n}x{k}: {ms * 1e3:8.1f} us  {tf:7.1f} TFLOP/s  {tf / 833.3:.2f} of sf16 peak")


if __name__ == "__main__":
    main()
