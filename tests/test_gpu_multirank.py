"""The data-parallel path with the real PPO class in two processes: two ranks as
fresh child processes, gloo, both on device 0 (this box has one GPU; the 8-GPU RCCL run is the
driver's).  Checked:
  - both ranks end with bit-identical parameters (every rank applies the same all-reduced gradient);
  - the two-rank run equals a single-rank run over all 2N lanes with num_lane_groups = 2 (the same
    minibatches, rlks_ppo_gather_grouped): parameters within 1e-5 of their norm and 1e-3 of the
    update's norm (fp32 summation order differs: per-rank partial sums + all-reduce vs one sum), KL
    coefficient, episode counts and episode_reward_mean (the lanes' f64 returns are the same)."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

HERE = Path(__file__).resolve().parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(out, N, T, mb, epochs, iters, world, overlap=1, extra_env=None):
    out.mkdir(parents=True, exist_ok=True)
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0", **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, str(HERE / "multirank_worker.py"), str(out), str(N),
                                       str(T), str(mb), str(epochs), str(iters), str(overlap)], env=env))
    try:
        for p in procs:
            assert p.wait(timeout=100) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return [np.load(out / f"rank{r}.npz") for r in range(world)]


def test_two_ranks_equal_one_rank_with_two_lane_groups(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rlks.ppo import PPO, PPOConfig

    N, T, mb, epochs, iters, world = 512, 128, 4096, 2, 2, 2
    ranks = _run_ranks(tmp_path, N, T, mb, epochs, iters, world)
    assert np.array_equal(ranks[0]["params"], ranks[1]["params"])
    res = [json.loads(str(z["results"])) for z in ranks]
    assert res[0] == res[1]
    # single rank over all lanes, two lane groups
    d = torch.device("cuda", 0)
    cfg = (PPOConfig().environment("K8sMultiCloudEnv").framework("torch")
           .training(train_batch_size=N * T * world, sgd_minibatch_size=mb, num_sgd_iter=epochs, lr=3e-4, gamma=0.99)
           .debugging(seed=13))
    cfg.num_envs = N * world
    cfg.rollout_fragment_length = T
    cfg.num_lane_groups = world
    algo = PPO(config=cfg, device=d)
    p0 = algo.params.flat.cpu().numpy().astype(np.float64)
    single = [algo.train() for _ in range(iters)]
    p1 = algo.params.flat.cpu().numpy().astype(np.float64)
    p2 = ranks[0]["params"].astype(np.float64)
    dn = np.linalg.norm(p2 - p1)
    print(f"||p_2rank - p_1rank|| / ||p|| = {dn / np.linalg.norm(p1):.2e}, / ||update|| = "
          f"{dn / np.linalg.norm(p1 - p0):.2e}")
    assert dn <= 1e-5 * np.linalg.norm(p1)
    assert dn <= 1e-3 * np.linalg.norm(p1 - p0)
    assert float(ranks[0]["kl_coeff"]) == float(algo.dyn[2].item())
    for a, b in zip(res[0], single):
        assert a["episodes_this_iter"] == b["episodes_this_iter"] and a["timesteps_total"] == b["timesteps_total"]
        assert a["episode_reward_mean"] == pytest.approx(b["episode_reward_mean"], rel=1e-12)
        assert a["kl"] == pytest.approx(b["info"]["learner"]["default_policy"]["learner_stats"]["kl"], rel=1e-3)


def test_overlapped_allreduce_is_bit_identical(tmp_path):
    """PPOConfig.overlap_allreduce (rlks_ppo_grad_step_part: the W2 / W3 bucket all-reduced while the
    dW1 kernel runs, then the W1 bucket) leaves the parameters, KL coefficient and results of the
    one-bucket path bit for bit, on both ranks; the profile reports both forms' exposed time"""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    N, T, mb, epochs, iters, world = 512, 64, 4096, 2, 2, 2
    # (both forms on the two F1 kernels: the overlapped form always runs them, the one-bucket form by
    # default runs the fused F1 at 2 actions, whose workgroup sums add in another order)
    split = {"RLKS_F1_SPLIT": "1"}
    on = _run_ranks(tmp_path / "on", N, T, mb, epochs, iters, world, overlap=1, extra_env=split)
    off = _run_ranks(tmp_path / "off", N, T, mb, epochs, iters, world, overlap=0, extra_env=split)
    for r in range(world):
        assert np.array_equal(on[r]["params"].view(np.int32), off[r]["params"].view(np.int32)), r
        assert float(on[r]["kl_coeff"]) == float(off[r]["kl_coeff"])
        assert json.loads(str(on[r]["results"])) == json.loads(str(off[r]["results"]))
    p_on, p_off = json.loads(str(on[0]["allreduce"])), json.loads(str(off[0]["allreduce"]))
    assert p_on["overlapped"] and not p_off["overlapped"]
    print(f"exposed all-reduce per SGD step: overlapped {p_on['allreduce_ms_per_sgd_step']:.3f} ms, "
          f"one bucket {p_off['allreduce_ms_per_sgd_step']:.3f} ms ({p_on['backend']})")


def test_bench_launches_two_ranks(tmp_path):
    """`bench.py --gpus 2` with no torch.distributed launcher: bench.py starts
    both ranks itself (gloo here: the box has one GPU, both ranks share it; RCCL is the 8-GPU node's),
    rank 0 prints one JSON line with n_gpus 2 and a finite policy, the whole job's lanes counted"""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    root = HERE.parent
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(RLKS_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--config", "c2", "--envs", "512",
                        "--rollout", "16", "--minibatch", "4096", "--epochs", "1", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-kernel-timing"], cwd=root, env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2" and j["finite"]
    assert j["config"]["global_batch"] == 2 * 512 * 16
    assert j["value"] == pytest.approx(2 * 512 * 16 * 2 / (j["ms_per_step"] * 2e-3), rel=1e-6)
    assert j["allreduce"] is not None


@pytest.mark.parametrize("overlap", [1, 0])
def test_one_rank_rccl_multirank_path_equals_one_rank(tmp_path, overlap, monkeypatch):
    """RCCL on hardware with one GPU: a one-rank RCCL process group with RLKS_DDP_FORCE=1 takes the
    multi-rank SGD step (gradient -> RCCL all-reduce -> Adam; overlap=1: the two-bucket all-reduce on
    RCCL's stream under F1b) with every collective issued, exactly the calls of the 8-GPU run.  A
    one-rank all-reduce is the identity, so the parameters equal the ordinary one-rank run's bit for bit;
    the worker's profile_allreduce reports RCCL's per-step time on this box."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from rlks.ppo import PPO, PPOConfig

    N, T, mb, epochs, iters = 1024, 64, 8192, 2, 2
    env = {"RLKS_DIST_BACKEND": "nccl", "RLKS_DDP_FORCE": "1"}
    if overlap:  # the overlapped form runs the two F1 kernels: so does the one-rank reference here
        env["RLKS_F1_SPLIT"] = "1"
        monkeypatch.setenv("RLKS_F1_SPLIT", "1")
    (z,) = _run_ranks(tmp_path, N, T, mb, epochs, iters, 1, overlap=overlap, extra_env=env)
    prof = json.loads(str(z["allreduce"]))
    assert prof is not None and prof["backend"] == "nccl" and prof["overlapped"] == bool(overlap), prof
    print("one-rank RCCL all-reduce:", json.dumps(prof))
    cfg = (PPOConfig().environment("K8sMultiCloudEnv").framework("torch")
           .training(train_batch_size=N * T, sgd_minibatch_size=mb, num_sgd_iter=epochs, lr=3e-4, gamma=0.99)
           .debugging(seed=13))
    cfg.num_envs = N
    cfg.rollout_fragment_length = T
    algo = PPO(config=cfg, device=torch.device("cuda", 0))
    assert not algo.multi
    single = [algo.train() for _ in range(iters)]
    assert np.array_equal(z["params"].view(np.uint32), algo.params.flat.cpu().numpy().view(np.uint32))
    res = json.loads(str(z["results"]))
    np.testing.assert_equal([r["episode_reward_mean"] for r in res], [r["episode_reward_mean"] for r in single])
