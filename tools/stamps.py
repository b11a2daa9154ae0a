#!/usr/bin/env python3
"""Phase timing of the split-fp16 F1a (k_sf_fwd) and F2 (k_sf_dw2) kernels from in-kernel s_memtime stamps (diagnostic build).

  make -C rl-k8s-scheduler_amd/csrc stamps
  RLKS_LIB=rl-k8s-scheduler_amd/rlks/librlks_stamps.so python tools/stamps.py

Runs a few c2-sized SGD-step gradients (65,536 rows), then prints, per net, the median over waves
of each phase's shader cycles (the stamps are taken by lane 0 of every wave after the phase), and how
the waves that share a SIMD overlap in time.  --roll: the rollout step kernel's phases."""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))


def roll():
    """phase clocks of the split-fp16 rollout step kernel (k_sf_roll), c2 shapes"""
    import torch
    from rlks import _lib
    from rlks.ppo import PPO, PPOConfig

    cfg = PPOConfig().training(train_batch_size=4096 * 128, sgd_minibatch_size=65536, num_sgd_iter=1)
    cfg.num_envs = 4096
    cfg.rollout_fragment_length = 128
    algo = PPO(config=cfg, device=torch.device("cuda", 0))
    for _ in range(3):
        algo.rollout()
    torch.cuda.synchronize()
    st = np.zeros((256, 2, 8), np.uint64)
    assert _lib.lib().rlks_dbg_roll_stamps(st.ctypes.data_as(C.c_void_p)) == 0
    s = st[:128].astype(np.int64)
    names = ["X split", "phase 1 (H1^T) + barrier", "phase 2 (Z2^T)", "phase 3 + barrier", "sample + env step"]
    for wv, who in ((0, "wave 0 (pi)"), (1, "wave 4 (vf)")):
        dt = np.diff(s[:, wv, :6], axis=1)
        print(f"{who}:")
        for i, n in enumerate(names[: 5 if wv == 0 else 4]):
            print(f"  {n:26s} median {np.median(dt[:, i]):7.0f} cyc")


def fwd_report(lib, tiles):
    """F1a (k_sf_fwd) phases per wave, and how the waves that share a SIMD overlap in time"""
    st = np.zeros((2, 8192, 8), np.uint64)
    assert lib.rlks_dbg_fa_stamps(st.ctypes.data_as(C.c_void_p)) == 0
    names = ["prologue", "Z2 k-tile 0", "Z2 k-tiles 1-7", "H2 + head", "loss + dW3 + stats", "dZ2 store"]
    t = st[:, :tiles, :7].astype(np.int64)
    hw = st[:, :tiles, 7]
    t0 = t[..., 0].min()
    for net in range(2):
        s = t[net]
        dt = np.diff(s, axis=1)
        tot = s[:, 6] - s[:, 0]
        print(f"F1a net {net}: wave lifetime median {np.median(tot):.0f} cyc (p10 {np.percentile(tot, 10):.0f}, "
              f"p90 {np.percentile(tot, 90):.0f})")
        for i, n in enumerate(names):
            print(f"  {n:20s} median {np.median(dt[:, i]):8.0f}  p90 {np.percentile(dt[:, i], 90):8.0f}")
    # SIMD identity: XCC, SE, SH, CU, SIMD fields of HW_ID (gfx9 layout)
    hwid = (hw & 0xFFFFFFFF).astype(np.int64)
    xcc = (hw >> 32).astype(np.int64) & 0xF
    simd = (hwid >> 4) & 3
    cu = (hwid >> 8) & 0xF
    sh = (hwid >> 12) & 1
    se = (hwid >> 13) & 7
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    start = t[..., 0].ravel() - t0
    end = t[..., 6].ravel() - t0
    k = key.ravel()
    print(f"distinct SIMDs {len(np.unique(k))}, kernel span {end.max():.0f} cyc")
    # per SIMD: busy span vs sum of wave lifetimes -> average waves resident
    spans, conc = [], []
    for q in np.unique(k)[:4096]:
        m = k == q
        spans.append(end[m].max() - start[m].min())
        conc.append((end[m] - start[m]).sum() / max(1, spans[-1]))
    print(f"per-SIMD span median {np.median(spans):.0f}, waves per SIMD {np.bincount(np.unique(k, return_counts=True)[1]).nonzero()[0]}, "
          f"mean resident waves {np.mean(conc):.2f}")
    order = np.argsort(start)
    print("first 12 waves (start, end, simd key):", [(int(start[i]), int(end[i]), int(k[i])) for i in order[:12]])


def f2_report(lib):
    """F2 (k_sf_dw2) per-wave phase cycles summed over its chunks (waves 0-7 of each workgroup)"""
    st = np.zeros((2, 128, 16, 6), np.uint64)
    assert lib.rlks_dbg_f2_stamps(st.ctypes.data_as(C.c_void_p)) == 0
    names = ["prologue", "MFMA issue", "production", "barrier waits", "epilogue"]
    for net in range(2):
        for ws, who in ((slice(0, 4), "waves 0-3 (H1)"), (slice(4, 8), "waves 4-7 (dZ2)")):
            s = st[net, :, ws, :5].astype(np.int64)
            tot = s.sum(-1)
            print(f"F2 net {net} {who}: wave lifetime median {np.median(tot):.0f} cyc (p90 {np.percentile(tot, 90):.0f})")
            for i, n in enumerate(names):
                print(f"  {n:16s} median {np.median(s[..., i]):8.0f}  p90 {np.percentile(s[..., i], 90):8.0f}")


def main():
    if "--roll" in sys.argv:
        return roll()

    import torch
    from rlks import _lib
    from rlks.policy import PolicyParams

    assert "stamps" in os.environ.get("RLKS_LIB", ""), "set RLKS_LIB to librlks_stamps.so"
    d = torch.device("cuda", 0)
    rows = 65536
    p = PolicyParams(6, 256, 2, device=d, seed=1)
    p.desc.precision = _lib.RLKS_PRECISION_SF16
    rng = np.random.default_rng(0)
    mb = np.zeros((rows, 12), np.float32)
    mb[:, :6] = rng.random((rows, 6))
    mb[:, 6:8] = rng.standard_normal((rows, 2))
    mb[:, 8] = rng.standard_normal(rows)
    mb[:, 9] = rng.standard_normal(rows)
    mb[:, 11] = rng.integers(0, 2, rows)
    mb[:, 10] = -0.7
    dyn = torch.tensor([0, 1, 0.2, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.0)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
    ws = torch.empty(wsb.value, dtype=torch.uint8, device=d)
    grad = torch.zeros(p.padded, device=d)
    mbt = torch.from_numpy(mb).to(d)
    for _ in range(5):
        _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
                  rows, grad.data_ptr(), None, ws.data_ptr(), ws.numel(), None)
    torch.cuda.synchronize()
    fwd_report(_lib.lib(), rows // 16)  # F1a (k_sf_fwd) phases, one wave per 16-row tile
    f2_report(_lib.lib())

if __name__ == "__main__":
    main()
