"""JSON-lines metrics reporter for PPO.train() results (SURVEY.md §5 "Metrics / logging").

The reference prints `result['episode_reward_mean']` once per iteration (train_ppo.py:29-30,
train_and_compare.py:46-48) and Tune logs results with verbose=2 (train_final.py:32-33).  Here each
train() result can also be appended as one JSON object per line: the iteration, episode statistics,
learner stats, env-steps/s over the iteration's wall clock, and the iteration's arithmetic rate as a
fraction of the split-fp16 MFMA ceiling.  Enabled by PPOConfig.reporting(json_lines=path) or the
environment variable RLKS_METRICS_JSONL; written by rank 0 only.
"""
from __future__ import annotations

import json
import math
import os
from pathlib import Path

METRICS_ENV = "RLKS_METRICS_JSONL"
# MI355X dense f16 MFMA peak (MI355X_MICROARCH.md) / 3 f16 products per fp32-accurate FLOP
SF16_PEAK_TFLOPS = 2500.0 / 3


def flops_per_env_step(D: int, H: int, A: int, epochs: int) -> float:
    """algorithmic FLOPs per env-step of one PPO iteration: the rollout forward of
    both nets, then `epochs` x (forward + backward) of both nets per sample"""
    fwd = sum(2 * (D * H + H * H + H * An) for An in (A, 1))
    return fwd + epochs * 3 * fwd


def _clean(x):
    if isinstance(x, float) and not math.isfinite(x):
        return None
    if isinstance(x, dict):
        return {k: _clean(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_clean(v) for v in x]
    if hasattr(x, "item") and not isinstance(x, (str, bytes)):
        try:
            return _clean(x.item())
        except Exception:
            return str(x)
    return x


class JsonLinesReporter:
    """appends one JSON line per reported result (flushed, so a killed run keeps its lines)"""

    def __init__(self, path, rank: int = 0):
        self.path = Path(path)
        self.rank = rank
        if rank == 0:
            self.path.parent.mkdir(parents=True, exist_ok=True)

    @classmethod
    def from_config(cls, config, rank=0):
        p = getattr(config, "metrics_json_lines", None) or os.environ.get(METRICS_ENV)
        return cls(p, rank) if p else None

    def line(self, result: dict, algo=None) -> dict:
        learner = result.get("info", {}).get("learner", {}).get("default_policy", {}).get("learner_stats", {})
        out = {k: result.get(k) for k in ("training_iteration", "timesteps_total", "episode_reward_mean",
                                          "episode_reward_mean_this_iter", "episodes_this_iter", "episodes_total",
                                          "time_this_iter_s")}
        out["learner"] = learner
        if "evaluation" in result:
            out["evaluation"] = result["evaluation"]
        if algo is not None:
            t = result.get("time_this_iter_s") or float("nan")
            steps = algo.samples * algo.world
            out["env_steps_this_iter"] = steps
            out["env_steps_per_s"] = steps / t if t > 0 else None
            fl = flops_per_env_step(algo.D, algo.H, algo.A, int(algo.config.num_sgd_iter)) * steps / algo.world
            tf = fl / t / 1e12 if t > 0 else None
            out["tflops_per_gpu"] = tf
            out["frac_sf16_mfma_ceiling"] = tf / SF16_PEAK_TFLOPS if tf is not None else None
            out["sgd_precision"] = algo.precision
            out["n_gpus"] = algo.world
        return _clean(out)

    def report(self, result: dict, algo=None) -> dict:
        rec = self.line(result, algo)
        if self.rank == 0:
            with open(self.path, "a") as f:
                f.write(json.dumps(rec) + "\n")
        return rec
