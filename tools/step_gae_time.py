"""A/B timing of the GAE scan and the 2-cloud env step on one GPU (select a library with RLKS_LIB).

Prints one JSON line: GAE ms at c2 (128 x 4,096) and c4 (128 x 131,072) shapes, and the lean
k_env_step2 at 16M lanes.  Average over back-to-back launches measured with HIP events on the
launch stream.
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))

import torch  # noqa: E402

from rlks import VecK8sMultiCloudEnv, _lib  # noqa: E402


def timed(fn, s, n=50):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    d = torch.device("cuda", 0)
    s = torch.cuda.current_stream(d)
    out = {"lib": str(_lib.LIB_PATH.name)}
    for T, N in ((128, 4096), (128, 131072)):
        r = torch.rand(T, N, device=d) * 100
        v = torch.randn(T + 1, N, device=d) * 50
        dn = (torch.rand(T, N, device=d) < 0.01).to(torch.uint8)
        adv = torch.empty(T, N, device=d)
        vt = torch.empty(T, N, device=d)
        part = torch.zeros(_lib.lib().rlks_gae_partials_count(N), 2, dtype=torch.float64, device=d)
        ms = timed(lambda: _lib.call("rlks_gae", r.data_ptr(), v.data_ptr(), dn.data_ptr(), 0.99, 1.0, T, N,
                                     adv.data_ptr(), vt.data_ptr(), part.data_ptr(), s.cuda_stream), s)
        out[f"gae_{T}x{N}_ms"] = ms
        out[f"gae_{T}x{N}_GBps"] = 17 * T * N / (ms * 1e-3) / 1e9
    big = 1 << 24
    venv = VecK8sMultiCloudEnv(big, seed=1, device=d, track_returns=False)
    venv.reset()
    acts = torch.randint(0, 2, (big,), dtype=torch.int32, device=d)
    ms = timed(lambda: _lib.call("rlks_env_step", venv.handle, acts.data_ptr(), venv.obs.data_ptr(),
                                 venv.reward.data_ptr(), None, venv.terminated.data_ptr(), None, None,
                                 venv.final_obs.data_ptr(), None, s.cuda_stream), s, n=20)
    out["env_step_16M_ms"] = ms
    out["env_step_16M_GBps"] = 49 * big / (ms * 1e-3) / 1e9
    print(json.dumps(out))


if __name__ == "__main__":
    main()
