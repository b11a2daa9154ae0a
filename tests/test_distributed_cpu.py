"""Multi-process (gloo, world size 2, CPU) coverage of the data-parallel protocol used by rlks.ppo.

What is checked, with the CPU oracle standing in for the per-rank GPU kernels (tests only):
  1. lane sharding: rank r's lanes (env_offset = r*N) replay exactly the lanes [rN, (r+1)N) of a
     single-process run with 2N lanes (Philox counters keyed by the global lane id);
  2. the gradient protocol: per-rank gradients with loss scale 1/(rows*world), summed by
     all_reduce, equal the single-process gradient of the global-minibatch mean; the two-bucket
     async form of the overlapped SGD step gives the one-buffer all-reduce's bits;
  3. advantage-moment all-reduce gives the global mean / std used for standardisation.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tiny_net(rng):
    D, H, A = 6, 8, 2
    shapes = [(H, D), (H,), (H, H), (H,), (A, H), (A,), (H, D), (H,), (H, H), (H,), (1, H), (1,)]
    off, o = [], 0
    for s in shapes:
        off.append(o)
        o += int(np.prod(s))
    return D, H, A, off, rng.standard_normal(o) * 0.5


def _minibatch(rng, rows, D, A):
    mb = np.zeros((rows, D + A + 4))
    mb[:, :D] = rng.random((rows, D))
    mb[:, D:D + A] = rng.standard_normal((rows, A))
    mb[:, D + A] = rng.standard_normal(rows)
    mb[:, D + A + 1] = rng.standard_normal(rows)
    act = rng.integers(0, A, rows)
    mb[:, D + A + 3] = act
    lo = mb[:, D:D + A]
    mb[:, D + A + 2] = (lo - np.log(np.exp(lo).sum(1, keepdims=True)))[np.arange(rows), act]
    return mb


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "rl-k8s-scheduler_amd"), str(root / "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from rlks import distributed as ddp
        from rlks.tables import load_table

        assert ddp.rank_world() == (rank, world)
        tab = load_table()
        N = 64
        lo, hi = ddp.lane_range(N, rank)
        env = oracle.OracleEnv(oracle.make_cfg(N, tab.n_rows, tab.n_clouds, noise_mode=0, seed=5, autoreset=1,
                                               env_offset=lo), tab.cost, tab.latency)
        obs = [env.reset()]
        rng = np.random.default_rng(9)
        acts = rng.integers(0, 2, (150, N * world)).astype(np.int32)
        rew = []
        for t in range(150):
            o, r, _, _, _, _ = env.step(acts[t, lo:hi])
            obs.append(o.copy())
            rew.append(r.copy())
        # gradient protocol on this rank's half of a global minibatch
        rng = np.random.default_rng(3)
        D, H, A, off, flat = _tiny_net(rng)
        rows = 64
        mb = _minibatch(rng, rows * world, D, A)
        mine = mb[rank * rows:(rank + 1) * rows]
        g, _ = oracle.ppo_loss_grad(flat, off, D, H, A, mine, count=1.0 / ddp.loss_scale(rows, world))
        gt = torch.from_numpy(g.copy())
        # the overlapped form (PPO.sgd_step, rlks_ppo_grad_step_part): the W2 / W3 bucket of each net,
        # then the W1 bucket, as async in-place all-reduces on views of one flat fp32 buffer
        g32 = torch.from_numpy(g.astype(np.float32))
        b32 = g32.clone()
        o = off + [g32.numel()]
        h = ddp.allreduce_sum_async([b32[o[2]:o[6]], b32[o[8]:o[12]]])
        h += ddp.allreduce_sum_async([b32[o[0]:o[2]], b32[o[6]:o[8]]])
        for w in h:
            w.wait()
        ddp.allreduce_sum_(g32)
        assert torch.equal(b32.view(torch.int32), g32.view(torch.int32))
        ddp.allreduce_sum_(gt)
        # advantage moments
        adv = rng.standard_normal(1000 * world)[rank * 1000:(rank + 1) * 1000]
        mom = torch.tensor([adv.sum(), (adv ** 2).sum(), float(adv.size)], dtype=torch.float64)
        ddp.allreduce_sum_(mom)
        q.put((rank, np.stack(obs), np.stack(rew), gt.numpy(), mom.numpy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_protocol_matches_single_process():
    import oracle
    from rlks.tables import load_table

    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, obs, rew, g, mom = q.get(timeout=240)
        res[r] = (obs, rew, g, mom)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # 1. sharded lanes == the corresponding lanes of one 2N-lane process
    tab = load_table()
    N = 64
    env = oracle.OracleEnv(oracle.make_cfg(N * world, tab.n_rows, tab.n_clouds, noise_mode=0, seed=5, autoreset=1),
                           tab.cost, tab.latency)
    obs = [env.reset()]
    rng = np.random.default_rng(9)
    acts = rng.integers(0, 2, (150, N * world)).astype(np.int32)
    rew = []
    for t in range(150):
        o, r, _, _, _, _ = env.step(acts[t])
        obs.append(o.copy())
        rew.append(r.copy())
    obs, rew = np.stack(obs), np.stack(rew)
    for r in range(world):
        np.testing.assert_array_equal(res[r][0], obs[:, r * N:(r + 1) * N])
        np.testing.assert_array_equal(res[r][1], rew[:, r * N:(r + 1) * N])
    # 2. all-reduced gradient == single-process gradient of the global-minibatch mean
    rng = np.random.default_rng(3)
    D, H, A, off, flat = _tiny_net(rng)
    mb = _minibatch(rng, 64 * world, D, A)
    g_ref, _ = oracle.ppo_loss_grad(flat, off, D, H, A, mb)
    for r in range(world):
        np.testing.assert_allclose(res[r][2], g_ref, rtol=1e-10, atol=1e-12)
    # 3. moments
    adv = rng.standard_normal(1000 * world)
    for r in range(world):
        np.testing.assert_allclose(res[r][3], [adv.sum(), (adv ** 2).sum(), adv.size], rtol=1e-12)
