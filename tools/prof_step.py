#!/usr/bin/env python3
"""Profiling driver: one rollout + GAE + `--sgd` SGD steps of the c2 workload (for rocprofv3)."""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "rl-k8s-scheduler_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sgd", type=int, default=8)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=1)
    a = ap.parse_args()
    import torch
    from rlks.ppo import PPO, PPOConfig

    cfg = PPOConfig().training(train_batch_size=a.envs * 128, sgd_minibatch_size=65536, num_sgd_iter=10, lr=3e-4)
    cfg.num_envs = a.envs
    cfg.rollout_fragment_length = 128
    algo = PPO(config=cfg, device=torch.device("cuda", 0))
    for _ in range(a.iters):
        algo.rollout()
        algo.advantages()
        for k in range(a.sgd):
            algo.sgd_step(k // algo.n_mb, k % algo.n_mb, algo.stats[k])
    torch.cuda.synchronize()
    print("done", algo.stats[: a.sgd, :5].cpu().numpy().sum(0))


if __name__ == "__main__":
    main()
