"""fused F1 (k_sf_f1, RLKS_F1_FUSED=1) vs the two kernels (the default): the same arithmetic, so with the
same workgroup size the gradients must be bit-identical.  Prints per tensor the max |fused - split| at several minibatch sizes."""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "rl-k8s-scheduler_amd"), str(ROOT / "oracle")]
import torch  # noqa: E402
from test_gpu_learn import _minibatch, _params  # noqa: E402


def grad(p, mbt, rows, co, dyn, d):
    from rlks import _lib

    wsb = C.c_int64()
    _lib.call("rlks_ppo_workspace_bytes", C.byref(p.desc), rows, C.byref(wsb))
    ws = torch.full((wsb.value,), 0x7f, dtype=torch.uint8, device=d)
    g = torch.zeros(p.padded, device=d)
    st = torch.zeros(8, dtype=torch.float64, device=d)
    _lib.call("rlks_ppo_grad", C.byref(p.desc), C.byref(co), p.flat.data_ptr(), dyn.data_ptr(), mbt.data_ptr(),
              rows, g.data_ptr(), st.data_ptr(), ws.data_ptr(), ws.numel(), None)
    torch.cuda.synchronize()
    return g.cpu().numpy()


def main():
    from rlks import _lib
    from rlks.policy import TENSOR_NAMES

    d = torch.device("cuda", 0)
    bad = 0
    for A in [int(a) for a in os.environ.get('F1_AS', '2,8').split(',')]:
        for rows in [int(x) for x in os.environ.get('F1_ROWS', '16384,32768,65536').split(',')]:
            D = 3 * A
            p = _params(d, seed=rows + A, D=D, A=A)
            p.desc.precision = int(os.environ.get('F1_PREC', '1'))
            rng = np.random.default_rng(rows)
            mb = _minibatch(rows, rng, D=D, A=A, p=p, d=d)
            mbt = torch.from_numpy(mb).to(d)
            dyn = torch.tensor([0.3, 0.7, 0.2, 1.0 / rows, 0, 0, 0, 0], dtype=torch.float32, device=d)
            co = _lib.PpoCoeffs(0.3, 10.0, 1.0, 0.01)
            os.environ.pop("RLKS_F1_FUSED", None)
            gs = grad(p, mbt, rows, co, dyn, d)
            srep = float(np.abs(gs - grad(p, mbt, rows, co, dyn, d)).max())
            os.environ["RLKS_F1_FUSED"] = "1"
            gf = grad(p, mbt, rows, co, dyn, d)
            gf2 = grad(p, mbt, rows, co, dyn, d)
            out = []
            for i, (name, _, _) in enumerate(TENSOR_NAMES):
                o, n = p.offsets[i], int(np.prod(p.shapes[i]))
                a, b = gs[o:o + n], gf[o:o + n]
                dm = float(np.abs(a - b).max())
                if dm:
                    out.append(f"{name}:{dm:.2e}/{float(np.abs(a).max()):.1e}({int((a != b).sum())})")
            rep = float(np.abs(gf - gf2).max())
            bad += bool(out) or rep != 0.0
            print(f"A={A} rows={rows} fused-vs-split {'IDENTICAL' if not out else ' '.join(out)}  fused rerun maxdiff {rep:.2e} split rerun {srep:.2e}",
                  flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
