"""time the SGD-step phases (F1a, F1b, F2, whole gradient) of the library RLKS_LIB points at, on a
c4-shaped 65,536-row minibatch (HIP events, 50 reps); one line per library for A/B runs"""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))
import torch  # noqa: E402

from rlks import _lib  # noqa: E402
from rlks.policy import PolicyParams  # noqa: E402

A = int(os.environ.get("XP_A", "2"))
D, M = 3 * A, 65536
d = torch.device("cuda", 0)
p = PolicyParams(D, 256, A, device=d, seed=3)
p.desc.precision = _lib.RLKS_PRECISION_SF16
stride = _lib.lib().rlks_minibatch_stride(C.byref(p.desc))
g = torch.Generator(device=d).manual_seed(1)
mb = torch.zeros(M, stride, device=d)
mb[:, :D] = torch.rand(M, D, generator=g, device=d)
mb[:, D:D + A] = torch.randn(M, A, generator=g, device=d)
mb[:, D + A] = torch.randn(M, generator=g, device=d)
mb[:, D + A + 1] = torch.randn(M, generator=g, device=d) * 30
mb[:, D + A + 2] = -torch.rand(M, generator=g, device=d) * 2
mb[:, D + A + 3] = torch.randint(0, A, (M,), generator=g, device=d).float()
dyn = torch.tensor([0.1, 1.3, 0.2, 1.0 / M, 0, 0, 0, 0], dtype=torch.float32, device=d)
co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.0)
wsb = C.c_int64()
_lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), M, C.byref(wsb))
ws = torch.zeros(wsb.value, dtype=torch.uint8, device=d)
grad = torch.zeros(p.padded, device=d)
s = torch.cuda.current_stream()


def phase(mask):
    _lib.call("rlks_ppo_grad_phases", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mb.data_ptr(),
              M, grad.data_ptr(), None, ws.data_ptr(), ws.numel(), mask, s.cuda_stream)


def timed(fn, n=50):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


phase(_lib.RLKS_PHASE_ALL)
out = {k: timed(lambda m=m: phase(m)) for k, m in (("F1a", _lib.RLKS_PHASE_F1A), ("F1b", _lib.RLKS_PHASE_F1B),
                                                  ("F2", _lib.RLKS_PHASE_DW2), ("all", _lib.RLKS_PHASE_ALL))}
g1 = grad.clone()
phase(_lib.RLKS_PHASE_ALL)
print(f"{Path(os.environ.get('RLKS_LIB', 'librlks.so')).name:28s} A={A} " +
      " ".join(f"{k} {v:6.1f}us" for k, v in out.items()) + f"  |g| {float(g1.norm()):.6e}", flush=True)
