#!/usr/bin/env python3
"""Profiling driver (for rocprofv3): one rollout + GAE + `--sgd` SGD steps of the c2 workload, or
with `--c3 K`, K steps of the c3 node-level env (65,536 envs x 8 clusters x 256 nodes)."""
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
    ap.add_argument("--c3", type=int, default=0)
    a = ap.parse_args()
    import torch
    if a.c3:
        from rlks import VecK8sMultiCloudEnv
        from rlks.env import NodeSpec
        from rlks.tables import synthetic_table

        dev = torch.device("cuda", 0)
        spec = NodeSpec(8, 256, arrival_rate=1.0, init_occupancy=0.5)
        venv = VecK8sMultiCloudEnv(65536, table=synthetic_table(8, 100, seed=42), seed=42, nodes=spec, device=dev)
        venv.reset()
        acts = [torch.randint(0, 8, (65536,), dtype=torch.int32, device=dev) for _ in range(8)]
        for t in range(300 + a.c3):
            venv.step(acts[t % 8])
        venv.check_status()
        print("done c3", a.c3)
        return
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
