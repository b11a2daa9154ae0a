#!/usr/bin/env python3
"""Profiling driver (for rocprofv3 --kernel-trace --stats): the c5 SGD-step gradient on the
generic-width path (wide_mlp.hip) — minibatch rows x obs 192 x hidden 2,048 x 64 actions, both nets.
Prints the HIP-event average of one rlks_ppo_grad and its fp32-equivalent TFLOP/s."""
import argparse
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--hidden", type=int, default=2048)
    ap.add_argument("--actions", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from bench import flops_per_row
    from rlks import _lib
    from rlks.policy import PolicyParams

    d = torch.device("cuda", 0)
    A, H, M = a.actions, a.hidden, a.rows
    D = 3 * A
    p = PolicyParams(D, H, A, device=d, seed=1)
    p.desc.precision = _lib.RLKS_PRECISION_WIDE
    stride = _lib.lib().rlks_minibatch_stride(C.byref(p.desc))
    mb = torch.rand(M, stride, device=d)
    mb[:, D + A + 3] = torch.randint(0, A, (M,), device=d).float()
    lg, _ = p.forward(mb[:, :D].contiguous())
    mb[:, D:D + A] = lg + 0.1 * torch.randn_like(lg)
    mb[:, D + A + 2] = torch.log_softmax(mb[:, D:D + A], 1).gather(1, mb[:, D + A + 3].long()[:, None])[:, 0]
    dyn = torch.tensor([0.0, 1.0, 0.2, 1.0 / M, 0, 0, 0, 0], device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.0)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), M, C.byref(wsb))
    ws = torch.empty(wsb.value, dtype=torch.uint8, device=d)
    grad = torch.zeros(p.padded, device=d)
    s = torch.cuda.current_stream()

    def step():
        _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mb.data_ptr(), M,
                  grad.data_ptr(), None, ws.data_ptr(), ws.numel(), s.cuda_stream)

    step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.reps):
        step()
    e1.record(s)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    tf = flops_per_row("wide_grad", D, H, A) * M / (ms * 1e-3) / 1e12
    print(f"wide grad rows {M} obs {D} hidden {H} actions {A}: {ms:.3f} ms  {tf:.1f} TFLOP/s "
          f"({tf / 833.3:.3f} of the split-fp16 ceiling)  finite={bool(torch.isfinite(grad).all())}", flush=True)


if __name__ == "__main__":
    main()
