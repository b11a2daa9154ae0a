"""Host-side checkpoint discovery (final_evaluation.py:13-25) and the JSON-lines reporter (SURVEY.md
§5): no GPU needed."""
import json
import sys
from pathlib import Path
from types import SimpleNamespace

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))


def test_latest_checkpoint_picks_highest_number(tmp_path, monkeypatch):
    from rlks.checkpoints import checkpoint_number, find_checkpoints, latest_checkpoint

    exp = tmp_path / "FINAL_PPO_AWS_AZURE"
    for trial, nums in (("PPO_K8sMultiCloudEnv_00000", (10, 20, 80)), ("PPO_K8sMultiCloudEnv_00001", (9, 100))):
        for n in nums:
            (exp / trial / f"checkpoint_{n:06d}").mkdir(parents=True)
    (exp / "PPO_K8sMultiCloudEnv_00000" / "checkpoint_tmp").mkdir()       # no trailing number: ignored
    (exp / "PPO_K8sMultiCloudEnv_00000" / "checkpoint_000999.json").write_text("{}")  # a file: ignored
    got = latest_checkpoint(tmp_path, "FINAL_PPO_AWS_AZURE")
    assert got == exp / "PPO_K8sMultiCloudEnv_00001" / "checkpoint_000100"
    assert [checkpoint_number(p) for p in find_checkpoints(exp)] == [9, 10, 20, 80, 100]
    assert latest_checkpoint(tmp_path / "missing") is None
    monkeypatch.setenv("RLKS_RESULTS_DIR", str(tmp_path))
    assert latest_checkpoint(name="FINAL_PPO_AWS_AZURE") == got


def test_json_lines_reporter(tmp_path):
    from rlks.metrics import JsonLinesReporter, flops_per_env_step

    # 269,824 FLOP forward per sample (2 actions), ~8.37 MFLOP per env-step at 10 epochs
    fwd = flops_per_env_step(6, 256, 2, 0)
    assert fwd == 2 * (6 * 256 + 256 * 256 + 256 * 2) + 2 * (6 * 256 + 256 * 256 + 256)
    assert abs(flops_per_env_step(6, 256, 2, 10) / 8.37e6 - 1) < 0.03
    r = JsonLinesReporter(tmp_path / "m" / "metrics.jsonl")
    algo = SimpleNamespace(samples=4000, world=1, D=6, H=256, A=2, precision="sf16",
                           config=SimpleNamespace(num_sgd_iter=10))
    res = {"training_iteration": 3, "timesteps_total": 12000, "episode_reward_mean": 4765.2,
           "episode_reward_mean_this_iter": float("nan"), "episodes_this_iter": 40, "episodes_total": 120,
           "time_this_iter_s": 0.5,
           "info": {"learner": {"default_policy": {"learner_stats": {"policy_loss": -0.01, "kl": 0.002}}}}}
    for _ in range(2):
        r.report(res, algo)
    lines = (tmp_path / "m" / "metrics.jsonl").read_text().splitlines()
    assert len(lines) == 2
    rec = json.loads(lines[0])
    assert rec["training_iteration"] == 3 and rec["episode_reward_mean"] == 4765.2
    assert rec["episode_reward_mean_this_iter"] is None      # NaN is not JSON
    assert rec["env_steps_per_s"] == 8000.0 and rec["learner"]["kl"] == 0.002
    assert 0 < rec["frac_sf16_mfma_ceiling"] < 1
    quiet = JsonLinesReporter(tmp_path / "rank1.jsonl", rank=1)
    quiet.report(res, algo)
    assert not (tmp_path / "rank1.jsonl").exists()


def test_per_tensor_state_survives_a_layout_change():
    """Adam moments are checkpointed per tensor (PolicyParams.split / join): state saved
    under one flat storage order lands on the same named tensors under another"""
    import torch

    from rlks.policy import TENSOR_NAMES, PolicyParams

    p = PolicyParams(6, 256, 2, device=torch.device("cpu"))
    m = torch.arange(p.padded, dtype=torch.float32)
    sd = p.split(m)
    assert list(sd) == [n for n, _, _ in TENSOR_NAMES]
    for i, (name, _, _) in enumerate(TENSOR_NAMES):
        assert sd[name].shape == torch.Size(p.shapes[i])
        assert float(sd[name].reshape(-1)[0]) == float(p.offsets[i])
    # another storage order: the tensors in reverse, packed back to back
    q = PolicyParams(6, 256, 2, device=torch.device("cpu"))
    o, offs = 0, [0] * 12
    for i in reversed(range(12)):
        offs[i] = o
        o += int(torch.tensor(q.shapes[i]).prod())
    q.offsets = offs
    buf = torch.zeros(o)
    q.join(buf, sd)
    back = q.split(buf)
    for name in sd:
        assert torch.equal(back[name], sd[name])
    bad = dict(sd)
    bad[TENSOR_NAMES[0][0]] = torch.zeros(3)
    try:
        q.join(buf, bad)
    except ValueError:
        pass
    else:
        raise AssertionError("a shape mismatch must refuse")


def test_run_experiment_fans_out_reporters_and_restores(tmp_path):
    """a caller's reporter and the algorithm's own both receive every iteration, and the
    algorithm's own is back in place when run_experiment returns (a fake algorithm: no GPU)"""
    from rlks.checkpoints import run_experiment

    class Rec:
        def __init__(self):
            self.seen = []

        def report(self, result, algo):
            self.seen.append(result["training_iteration"])

    class FakeAlgo:
        rank = 0

        def __init__(self):
            self.iteration = 0
            self.reporter = Rec()

        def train(self):
            self.iteration += 1
            r = {"training_iteration": self.iteration}
            if self.reporter is not None:
                self.reporter.report(r, self)
            return r

        def save(self, d):
            p = Path(d) / f"checkpoint_{self.iteration:06d}"
            p.mkdir(parents=True, exist_ok=True)
            return str(p)

    class Cfg:
        env = "K8sMultiCloudEnv"

    algo = FakeAlgo()
    own, mine = algo.reporter, Rec()
    out = run_experiment(Cfg(), stop_iterations=3, checkpoint_frequency=2, num_to_keep=5, storage_path=tmp_path,
                         reporter=mine, algo=algo)
    assert own.seen == [1, 2, 3] and mine.seen == [1, 2, 3]
    assert algo.reporter is own
    assert [Path(p).name for p in out["checkpoints"]] == ["checkpoint_000002", "checkpoint_000003"]
