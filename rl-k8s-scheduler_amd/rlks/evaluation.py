"""Batched evaluation harness: the reference's evaluation and baseline loops, one env lane per episode.

Reference loops restated here (all sequential over ONE env and the process-global `random` stream):
  * final_evaluation.py:39-77 — 100 greedy episodes (`compute_single_action(obs, explore=False)`),
    per-episode cost `-ep_reward`, AWS / Azure choice counts, improvement vs the 4.765 greedy
    baseline, summary text (:80-82);
  * train_and_compare.py:53-79 — the round-robin baseline (`0 if env.current_step % 2 == 0 else 1`)
    and the side-by-side RL vs baseline table;
  * k8s_multi_cloud_env.py:156-157 — the cost-only greedy scheduler `normal_scheduler_step`.

Here episode e runs on lane e of a VecK8sMultiCloudEnv in CPython-MT19937 mode, and every lane
steps in the same kernel launch.  Lane e's generator is seeded like `random.seed(seed)` and then
advanced (rlks_env_mt_discard) by the 200 random() draws each earlier episode consumes (2 per
observation: reset + 99 steps), so lane e sees exactly the cpu-load draws episode e of the
reference's sequential loop sees.  Episode returns accumulate in float64 in step order from 0.0,
as `ep_reward += reward` does, so rewards, choices and costs equal the sequential loop's bit for bit
(tests/test_gpu_eval.py checks this against the drop-in env driven step by step).
"""
from __future__ import annotations

import random
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .env import VecK8sMultiCloudEnv
from .tables import load_table

BASELINE_COST = 4.765          # final_evaluation.py:73
DRAWS_PER_OBS = 2              # _get_obs: cpu_aws, cpu_azure (k8s_multi_cloud_env.py:92-93)
CLOUD_NAMES = ("AWS", "Azure")  # action 0 / 1 (final_evaluation.py:51)


@dataclass
class EvalResult:
    rewards: np.ndarray                 # float64 [episodes], sum of step rewards
    actions: np.ndarray                 # int32 [steps, episodes]
    baseline_cost: float = BASELINE_COST
    names: tuple = CLOUD_NAMES
    extra: dict = field(default_factory=dict)

    @property
    def costs(self) -> np.ndarray:      # final_evaluation.py:60
        return -self.rewards

    @property
    def avg_cost(self) -> float:        # :62
        return float(np.mean(self.costs))

    @property
    def choices(self) -> dict:          # :40, :51
        counts = np.bincount(self.actions.reshape(-1), minlength=len(self.names))
        return {n: int(c) for n, c in zip(self.names, counts)}

    @property
    def improvement(self) -> float:     # :74
        return 100 * (self.baseline_cost - self.avg_cost) / self.baseline_cost

    def progress_lines(self, every=20):
        """the per-episode progress prints of :54-55"""
        return [f"Episode {ep:3d} → cost = ${-self.rewards[ep - 1]:6.3f}"
                for ep in range(every, len(self.rewards) + 1, every)]

    def report(self) -> str:
        """the results block of final_evaluation.py:64-77"""
        ch = self.choices
        total = sum(ch.values())
        lines = ["", "=" * 60, f"FINAL EVALUATION RESULTS ({len(self.rewards)} episodes)", "=" * 60,
                 f"Average cost per episode       : ${self.avg_cost:.4f}",
                 f"Total decisions total           : {total}"]
        for n in self.names:
            lines.append(f"Agent chose {n:<19}: {ch[n]:4d} times ({ch[n] / total:.1%})")
        lines += ["", f"Improvement vs greedy baseline (${self.baseline_cost:.3f}): {self.improvement:5.1f}% better",
                  "=" * 60]
        return "\n".join(lines)

    def summary_text(self) -> str:
        """the summary file body of :80-82"""
        ch = self.choices
        return (f"Avg cost: ${self.avg_cost:.4f} | Improvement: {self.improvement:.1f}%\n"
                f"{self.names[0]} choices: {ch[self.names[0]]} | {self.names[1]} choices: {ch[self.names[1]]}\n")


def _params_of(policy):
    """PolicyParams of a PPO algorithm or the params themselves"""
    return getattr(policy, "params", policy)


def evaluate(policy, num_episodes: int = 100, *, seed=None, table=None, device=None,
             baseline_cost: float = BASELINE_COST) -> EvalResult:
    """final_evaluation.py:39-77 batched: `policy` is a PPO algorithm / PolicyParams (greedy argmax,
    compute_single_action(obs, explore=False)), or "round_robin" / "greedy" for the baselines.

    seed: the value of the reference's `random.seed(seed)` before its first episode (its env is
    unseeded, so the process-global stream decides; None draws one from this process's `random`)."""
    import torch

    if num_episodes <= 0:
        raise ValueError("num_episodes must be positive")
    table = table if table is not None else load_table()
    if isinstance(policy, str):
        if policy not in ("round_robin", "greedy"):
            raise ValueError(f"unknown baseline policy {policy!r}")
        params = None
    else:
        params = _params_of(policy)
        if params.D != 3 * table.n_clouds or params.A != table.n_clouds:
            raise ValueError("policy shape does not match the table's clouds")
    if seed is None:
        seed = random.getrandbits(64)
    if device is None:
        device = params.flat.device if params is not None else torch.device("cuda", torch.cuda.current_device())
    E = int(num_episodes)
    T = table.n_rows - 1  # max_steps (:66): every episode is exactly 99 steps
    env = VecK8sMultiCloudEnv(E, table=table, noise="mt19937", autoreset=False, device=device)
    try:
        env.seed([int(seed)] * E)
        per_episode = DRAWS_PER_OBS * (T + 1)
        skip = torch.arange(E, dtype=torch.int64, device=env.device) * per_episode
        _lib.call("rlks_env_mt_discard", env.handle, None, _lib.ptr(skip), env.dev.stream)
        obs = env.reset()
        ep_ret = torch.zeros(E, dtype=torch.float64, device=env.device)
        actions = torch.empty(T, E, dtype=torch.int32, device=env.device)
        logits = torch.empty(E, table.n_clouds, dtype=torch.float32, device=env.device)
        values = torch.empty(E, dtype=torch.float32, device=env.device)
        for t in range(T):
            if params is not None:
                params.forward(obs, logits, values)
                a = torch.argmax(logits, dim=1).to(torch.int32)   # np.argmax: first maximum
            elif policy == "round_robin":                        # train_and_compare.py:65
                a = torch.full((E,), t % 2, dtype=torch.int32, device=env.device)
            else:                                                # normal_scheduler_step (:156-157)
                a = (obs[:, 0] > obs[:, 1]).to(torch.int32)
            actions[t] = a
            obs, r, term, _, _ = env.step(a)
            ep_ret += r                                          # ep_reward += reward, float64
        env.check_status()
        if not bool(term.all()):
            raise RuntimeError("evaluation lanes did not terminate after max_steps")
        return EvalResult(ep_ret.cpu().numpy(), actions.cpu().numpy(), baseline_cost,
                          CLOUD_NAMES if table.n_clouds == 2 else tuple(f"cluster{c}" for c in range(table.n_clouds)),
                          {"seed": int(seed)})
    finally:
        env.close()


def evaluate_lanes(params, num_episodes: int, *, table=None, nodes=None, seed=0, device=None) -> np.ndarray:
    """Greedy (explore=False) float64 returns of `num_episodes` episodes, one lane each, all lanes
    in one batched env: RLlib's evaluation workers (train_final.py:19 .evaluation(
    evaluation_interval=5, evaluation_duration=20), evaluation explore=False).  Table envs run the
    reference-exact evaluate() above; node-level envs (configs c3 / c5) run Philox lanes keyed by
    `seed` (episode e = lane e)."""
    import torch

    table = table if table is not None else load_table()
    if nodes is None:
        return evaluate(params, num_episodes, seed=seed, table=table, device=device).rewards
    E = int(num_episodes)
    env = VecK8sMultiCloudEnv(E, table=table, seed=int(seed), noise="philox", autoreset=False, device=device,
                              nodes=nodes)
    try:
        obs = env.reset()
        ret = torch.zeros(E, dtype=torch.float64, device=env.device)
        logits = torch.empty(E, table.n_clouds, dtype=torch.float32, device=env.device)
        values = torch.empty(E, dtype=torch.float32, device=env.device)
        for _ in range(table.n_rows - 1):
            params.forward(obs, logits, values)
            obs, r, term, _, _ = env.step(torch.argmax(logits, dim=1).to(torch.int32))
            ret += r
        env.check_status()
        return ret.cpu().numpy()
    finally:
        env.close()


def round_robin_baseline(num_episodes: int = 5, **kw) -> np.ndarray:
    """train_and_compare.py:53-72: per-episode round-robin returns"""
    return evaluate("round_robin", num_episodes, **kw).rewards


def comparison_lines(rl_rewards, baseline_rewards):
    """train_and_compare.py:75-79: the side-by-side table"""
    return [f"Iteration {i + 1}: RL = {r:.2f} | Baseline = {b:.2f}"
            for i, (r, b) in enumerate(zip(rl_rewards, baseline_rewards))]
