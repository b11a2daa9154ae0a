"""CPU port of one PPO iteration (torch-CPU fp32 + the C env oracle) — BENCHMARK BASELINE ONLY.

Used by bench.py's cpu_baseline leg (rank 0, N = 1) to time the same workload on the host cores:
batched env stepping with the C restatement of the reference env (oracle/rlks_oracle.c),
the RLlib-default FCNet forward/backward with torch autograd on CPU, GAE in numpy, and
torch.optim.Adam.  It is never part of the product path.
"""
from __future__ import annotations

import time

import numpy as np


def _mlp(torch, D, H, A):
    nn = torch.nn

    def net(out):
        return nn.Sequential(nn.Linear(D, H), nn.Tanh(), nn.Linear(H, H), nn.Tanh(), nn.Linear(H, out))

    return net(A), net(1)


def time_cpu_iteration(n_envs=4096, T=128, minibatch=65536, epochs=10, epochs_timed=1, threads=None, seed=0,
                       table=None, nodes=None, hidden=256, label="c2"):
    """Returns dict(value=env-steps/s, cores, sample, seconds).  Times the full rollout plus
    `epochs_timed` of the `epochs` SGD epochs, and scales the update to `epochs`.  `table` /
    `nodes` (an rlks.env.NodeSpec) select the node-level env of configs c3 / c5."""
    import torch

    import oracle

    if threads:
        torch.set_num_threads(int(threads))
    cores = torch.get_num_threads()
    from rlks.tables import load_table

    tab = table if table is not None else load_table()
    if nodes is None:
        env = oracle.OracleEnv(oracle.make_cfg(n_envs, tab.n_rows, tab.n_clouds, noise_mode=0, seed=seed, autoreset=1),
                               tab.cost, tab.latency)
    else:
        tr = nodes.arrival_trace
        env = oracle.OracleEnv(
            oracle.make_cfg(n_envs, tab.n_rows, tab.n_clouds, noise_mode=0, seed=seed, autoreset=1,
                            nodes=nodes.nodes_per_cluster, arrival_mode=0 if tr is None else 1,
                            arrival_rate=nodes.arrival_rate, depart_prob=nodes.depart_prob,
                            init_occupancy=nodes.init_occupancy, reject_penalty=nodes.reject_penalty),
            tab.cost, tab.latency, nodes.node_cpu_m, nodes.node_mem_mi, tr)
    D, A, H = 3 * tab.n_clouds, tab.n_clouds, int(hidden)
    torch.manual_seed(seed)
    pi, vf = _mlp(torch, D, H, A)
    opt = torch.optim.Adam(list(pi.parameters()) + list(vf.parameters()), lr=3e-4)
    obs = env.reset()
    t0 = time.perf_counter()
    O = np.zeros((T + 1, n_envs, D), np.float32)
    LG = np.zeros((T, n_envs, A), np.float32)
    V = np.zeros((T + 1, n_envs), np.float32)
    ACT = np.zeros((T, n_envs), np.int64)
    R = np.zeros((T, n_envs), np.float32)
    DN = np.zeros((T, n_envs), np.uint8)
    O[0] = obs
    with torch.no_grad():
        for t in range(T):
            x = torch.from_numpy(O[t])
            lg = pi(x)
            V[t] = vf(x)[:, 0].numpy()
            a = torch.distributions.Categorical(logits=lg).sample().numpy().astype(np.int32)
            LG[t], ACT[t] = lg.numpy(), a
            o, rew, term, _, _, _ = env.step(a)
            O[t + 1], R[t], DN[t] = o, rew, term
        V[T] = vf(torch.from_numpy(O[T]))[:, 0].numpy()
    adv, vt = oracle.gae(R, V, DN, 0.99, 1.0)
    adv = ((adv - adv.mean()) / max(1e-4, adv.std())).astype(np.float32)
    t_roll = time.perf_counter() - t0
    S = T * n_envs
    X = torch.from_numpy(O[:T].reshape(S, D))
    LO = torch.from_numpy(LG.reshape(S, A))
    AC = torch.from_numpy(ACT.reshape(S))
    AD = torch.from_numpy(adv.reshape(S))
    VT = torch.from_numpy(vt.astype(np.float32).reshape(S))
    LPO = torch.log_softmax(LO, 1).gather(1, AC[:, None])[:, 0]
    t1 = time.perf_counter()
    for _ in range(epochs_timed):
        perm = torch.randperm(S)
        for b in range(max(1, S // minibatch)):
            idx = perm[b * minibatch:(b + 1) * minibatch]
            lg = pi(X[idx])
            lp = torch.log_softmax(lg, 1)
            ratio = torch.exp(lp.gather(1, AC[idx][:, None])[:, 0] - LPO[idx])
            surr = torch.min(AD[idx] * ratio, AD[idx] * torch.clamp(ratio, 0.7, 1.3))
            lpo = torch.log_softmax(LO[idx], 1)
            kl = (lpo.exp() * (lpo - lp)).sum(1)
            vfl = torch.clamp((vf(X[idx])[:, 0] - VT[idx]) ** 2, 0, 10.0)
            loss = (-surr + vfl).mean() + 0.2 * kl.mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
    t_epoch = (time.perf_counter() - t1) / epochs_timed
    total = t_roll + epochs * t_epoch
    return {"value": S / total, "cores": cores, "seconds": t_roll + epochs_timed * t_epoch,
            "sample": (f"one {label} iteration ({n_envs} envs x {T} steps rollout with the C env oracle + torch-CPU fp32 "
                       f"FCNet [{H},{H}]; update timed for {epochs_timed} of {epochs} epochs of {S // minibatch} x {minibatch}-row "
                       f"minibatches and scaled): rollout {t_roll:.2f} s, epoch {t_epoch:.2f} s")}
