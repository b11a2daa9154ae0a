"""which 16-row tiles' dZ2 hand-off differs between two runs of the same fused-F1 gradient"""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "rl-k8s-scheduler_amd"), str(ROOT / "oracle")]
import torch  # noqa: E402
from test_gpu_learn import _minibatch, _params  # noqa: E402


def main():
    from rlks import _lib

    os.environ["RLKS_F1_FUSED"] = "1"
    d = torch.device("cuda", 0)
    A = int(os.environ.get("F1_A", "2"))
    rows = int(os.environ.get("F1_ROWS", "65536"))
    D = 3 * A
    p = _params(d, seed=rows + A, D=D, A=A)
    p.desc.precision = 1
    mb = _minibatch(rows, np.random.default_rng(rows), D=D, A=A, p=p, d=d)
    mbt = torch.from_numpy(mb).to(d)
    dyn = torch.tensor([0.3, 0.7, 0.2, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
    co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.01)
    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
    ws = torch.zeros(wsb.value, dtype=torch.uint8, device=d)
    out = (C.c_void_p * 4)()
    _lib.call("rlks_debug_sf_handoff", C.byref(p.desc), rows, ws.data_ptr(), out)
    tiles = rows // 16
    runs = []
    for r in range(int(os.environ.get("F1_RUNS", "4"))):
        g = torch.zeros(p.padded, device=d)
        _lib.call("rlks_ppo_grad_phases", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(),
                  mbt.data_ptr(), rows, g.data_ptr(), None, ws.data_ptr(), ws.numel(),
                  _lib.RLKS_PHASE_PREP | _lib.RLKS_PHASE_FWD, None)
        torch.cuda.synchronize()
        rec = []
        for net in range(2):
            dz = torch.empty(tiles * 16 * 256 * 2, dtype=torch.float16, device=d)
            ed = torch.empty(tiles, dtype=torch.int32, device=d)
            rec.append((ptr_copy(out[net], dz), ptr_copy(out[2 + net], ed)))
        runs.append(rec)
    for r in range(1, len(runs)):
        for net in range(2):
            a, b = runs[0][net][0].view(tiles, -1), runs[r][net][0].view(tiles, -1)
            bad = (a != b).any(1).nonzero().flatten().cpu().numpy()
            ea, eb = runs[0][net][1], runs[r][net][1]
            bade = (ea != eb).nonzero().flatten().cpu().numpy()
            print(f"run {r} net {net}: {len(bad)} tiles with dZ2 differing, {len(bade)} with edz differing; "
                  f"tiles {bad[:24].tolist()} groups {sorted(set((bad // 8).tolist()))[:24]}", flush=True)
            if len(bad):
                t = int(bad[0])
                x, y = a[t].float(), b[t].float()
                diff = (x != y).nonzero().flatten()
                print(f"   tile {t}: {diff.numel()} of {x.numel()} halves differ, first at {diff[:8].tolist()}; "
                      f"max |d| {float((x - y).abs().max()):.3e} max |x| {float(x.abs().max()):.3e}", flush=True)


def ptr_copy(ptr, like):
    """copy like.numel() elements from device pointer ptr into a new tensor shaped like `like`"""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    t = torch.empty_like(like)
    rc = hip.hipMemcpy(t.data_ptr(), ptr, t.numel() * t.element_size(), 3)
    assert rc == 0, rc
    return t


if __name__ == "__main__":
    main()
