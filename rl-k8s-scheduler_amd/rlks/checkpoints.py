"""Checkpoint layout, discovery and the Tune-shaped checkpoint policy of the training drivers.

Reference call sites:
  * `agent.save()` once per iteration, default location under ~/ray_results
    (train_ppo.py:31, train_and_compare.py:49; RLlib Algorithm.save -> <logdir>/checkpoint_NNNNNN);
  * `tune.Tuner("PPO", run_config=air.RunConfig(stop={"training_iteration": 80},
    checkpoint_config=air.CheckpointConfig(checkpoint_frequency=10, num_to_keep=5,
    checkpoint_at_end=True), name="FINAL_PPO_AWS_AZURE"))` (train_final.py:22-35);
  * the evaluation script picks the newest `checkpoint_*[0-9]` below
    ~/ray_results/FINAL_PPO_AWS_AZURE by the number after the last "_" (final_evaluation.py:13-25).

Ray Tune itself (trial scheduling, search, remote trials) is out of scope; what the
drivers rely on is the directory layout and the checkpoint policy, restated here:
    <results root>/<experiment name>/<trial dir>/checkpoint_<iteration:06d>/
with results root = $RLKS_RESULTS_DIR or ~/ray_results, so that latest_checkpoint(), like
final_evaluation.py:16-25, finds what run_experiment() and PPO.save() write.
"""
from __future__ import annotations

import os
import re
import shutil
import time
from pathlib import Path

RESULTS_ENV = "RLKS_RESULTS_DIR"
_NUM = re.compile(r"_(\d+)$")


def results_root() -> Path:
    """~/ray_results (RLlib / Tune's default storage path), or $RLKS_RESULTS_DIR"""
    v = os.environ.get(RESULTS_ENV)
    return Path(v).expanduser() if v else Path.home() / "ray_results"


def default_logdir(env_name: str = "K8sMultiCloudEnv") -> Path:
    """RLlib's Algorithm logdir: <root>/PPO_<env>_<YYYY-MM-DD_HH-MM-SS>"""
    return results_root() / f"PPO_{env_name}_{time.strftime('%Y-%m-%d_%H-%M-%S')}"


def checkpoint_number(path) -> int:
    """the number after the last underscore (final_evaluation.py:25: int(p.name.split("_")[-1]))"""
    return int(Path(path).name.split("_")[-1])


def find_checkpoints(root) -> list[Path]:
    """every directory `checkpoint_*[0-9]` below root (recursive, as final_evaluation.py:16's
    rglob), oldest first by number"""
    root = Path(root)
    if not root.exists():
        return []
    c = [p for p in root.rglob("checkpoint_*[0-9]") if p.is_dir() and _NUM.search(p.name)]
    return sorted(c, key=lambda p: (checkpoint_number(p), str(p)))


def latest_checkpoint(root=None, name: str | None = None) -> Path | None:
    """the checkpoint with the highest number below root/name (default root: results_root());
    None when there is none (the reference prints a hint and exits, final_evaluation.py:18-22)"""
    base = Path(root) if root is not None else results_root()
    if name:
        base = base / name
    c = find_checkpoints(base)
    return max(c, key=checkpoint_number) if c else None


def run_experiment(config, *, name: str = "FINAL_PPO_AWS_AZURE", stop_iterations: int = 80,
                   checkpoint_frequency: int = 10, num_to_keep: int | None = 5, checkpoint_at_end: bool = True,
                   storage_path=None, reporter=None, algo=None, **ppo_kw) -> dict:
    """train_final.py's Tune run on one trial: train() until `stop_iterations`, save every
    `checkpoint_frequency` iterations and at the end, keep the `num_to_keep` newest checkpoints.
    Layout: <storage>/<name>/PPO_<env>_00000/checkpoint_<iteration:06d>.  Returns the last result,
    the trial directory and the kept checkpoints (oldest first).  `reporter` receives every
    iteration once; if the algorithm already has a reporter of its own (PPOConfig.metrics_json_lines /
    RLKS_METRICS_JSONL), both receive it (a fan-out).  The algorithm's previous reporter is restored
    when the run ends."""
    from .ppo import PPO

    root = Path(storage_path) if storage_path is not None else results_root()
    env = getattr(config.env, "__name__", None) or (str(config.env) if config.env else "K8sMultiCloudEnv")
    trial = root / name / f"PPO_{env}_00000"
    trial.mkdir(parents=True, exist_ok=True)
    algo = algo if algo is not None else PPO(config=config, **ppo_kw)
    prev = getattr(algo, "reporter", None)
    if reporter is not None:
        algo.reporter = reporter if prev is None else FanOut(prev, reporter)
    try:
        return _run(algo, trial, stop_iterations, checkpoint_frequency, num_to_keep, checkpoint_at_end)
    finally:
        algo.reporter = prev


class FanOut:
    """several reporters as one: each report() goes to all of them, in order"""

    def __init__(self, *reporters):
        self.reporters = reporters

    def report(self, result, algo):
        for r in self.reporters:
            r.report(result, algo)


def _run(algo, trial, stop_iterations, checkpoint_frequency, num_to_keep, checkpoint_at_end):
    kept: list[Path] = []
    result = None

    def save():
        p = Path(algo.save(trial))
        if p not in kept:
            kept.append(p)
        while num_to_keep and len(kept) > num_to_keep:
            old = kept.pop(0)
            if algo.rank == 0:
                shutil.rmtree(old, ignore_errors=True)

    while algo.iteration < stop_iterations:
        result = algo.train()
        if checkpoint_frequency and algo.iteration % checkpoint_frequency == 0:
            save()
    if checkpoint_at_end and (not kept or checkpoint_number(kept[-1]) != algo.iteration):
        save()
    return {"result": result, "trial_dir": str(trial), "checkpoints": [str(p) for p in kept], "algo": algo}
