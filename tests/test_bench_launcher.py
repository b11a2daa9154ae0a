"""bench.py's multi-rank launch, on the CPU: `python bench.py --gpus N` with no
torch.distributed launcher starts the N ranks itself (launch_ranks), the ranks rendezvous over gloo,
time with the barrier + MAX-over-ranks contract and rank 0 alone prints one JSON line.  --dry-run
replaces the PPO iteration by an empty step, so no GPU is needed; the real two-rank bench on the
GPU is tests/test_gpu_multirank.py::test_bench_launches_two_ranks."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _bench(*args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["RLKS_DIST_BACKEND"] = "gloo"
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_launcher_runs_two_ranks_and_prints_one_line():
    r = _bench("--dry-run", "--gpus", "2", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == 2 and j["steps"] == 3 and j["scaling"] == "weak"
    assert j["config"]["parallelism"] == "dp2"
    # weak: every rank owns the per-GPU c4 shard
    assert j["config"]["envs_per_gpu"] == 131072 and j["config"]["global_envs"] == 262144
    assert j["ms_per_step"] >= 1.0  # the empty step sleeps 1 ms; the max over ranks cannot be less


@pytest.mark.parametrize("n", [1, 2, 4])
def test_strong_scaling_fixes_the_whole_job(n):
    r = _bench("--dry-run", "--gpus", str(n), "--scaling", "strong", "--steps", "1", "--warmup", "0")
    assert r.returncode == 0, r.stderr
    (j,) = _json_lines(r.stdout)
    assert j["n_gpus"] == n and j["scaling"] == "strong"
    assert j["config"]["global_envs"] == 1048576 and j["config"]["global_minibatch"] == 524288
    assert j["config"]["envs_per_gpu"] == 1048576 // n


def test_world_size_must_match_gpus():
    env = {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1"}
    r = _bench("--dry-run", "--gpus", "1", env_extra=env, timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE 2 != --gpus 1" in r.stderr


def test_strong_scaling_rejects_an_uneven_split():
    r = _bench("--dry-run", "--gpus", "3", "--scaling", "strong", "--steps", "1")
    assert r.returncode != 0 and "do not split over 3 ranks" in r.stderr


def test_launcher_stops_the_others_when_a_later_rank_fails():
    """every rank is polled in every pass, so rank 1 failing while rank 0 blocks at the
    barrier ends the job promptly with rank 1's status (not at RCCL's watchdog, or never)."""
    import time

    t0 = time.monotonic()
    r = _bench("--dry-run", "--gpus", "2", "--steps", "1", "--warmup", "0", env_extra={"RLKS_DRYRUN_FAIL_RANK": "1"},
               timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert time.monotonic() - t0 < 60


def test_launcher_parent_stays_hip_free():
    """the launcher parent counts GPUs from sysfs and never initialises HIP (nor
    imports torch) before it starts the ranks."""
    code = ("import sys; sys.argv = ['bench.py']; import bench; "
            "n = bench.visible_gpus(); "
            "rc = bench.launch_ranks(2, ['--dry-run', '--gpus', '2', '--steps', '1', '--warmup', '0']); "
            "assert rc == 0, rc; "
            "assert 'torch' not in sys.modules, 'launcher parent imported torch'; "
            "print('ok', n)")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["RLKS_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def test_visible_gpus_honours_the_visible_devices_list(monkeypatch):
    sys.path.insert(0, str(ROOT))
    import bench

    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2")
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    assert bench.visible_gpus() == 3
