"""GPU parity of the node-level env extension (clusters x nodes, Poisson / bursty pod
arrivals, first-fit placement, integer resource accounting) against the C oracle: observations,
f64 rewards, terminations, every node's free millicores / MiB, the per-cluster aggregates and the
placement counters must be bit-identical."""
import ctypes as C_

import numpy as np
import pytest

import oracle
from parity import close_as_fp32, gae_fp32_serial, grad_close_as_fp32, logp_of

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _pair(n, C, nodes, *, seed=4, rate=2.0, trace=None, depart=0.05, occ=0.5, penalty=0.0):
    from rlks import VecK8sMultiCloudEnv
    from rlks.env import NodeSpec
    from rlks.tables import synthetic_table

    tab = synthetic_table(C, 100, seed=7)
    spec = NodeSpec(C, nodes, arrival_rate=rate, arrival_trace=trace, depart_prob=depart, init_occupancy=occ,
                    reject_penalty=penalty)
    venv = VecK8sMultiCloudEnv(n, table=tab, seed=seed, nodes=spec, env_offset=3, device=_dev())
    ora = oracle.OracleEnv(oracle.make_cfg(n, 100, C, noise_mode=0, seed=seed, autoreset=1, env_offset=3, nodes=nodes,
                                           arrival_mode=1 if trace is not None else 0, arrival_rate=rate,
                                           depart_prob=spec.depart_prob, init_occupancy=occ, reject_penalty=penalty),
                           tab.cost, tab.latency, spec.node_cpu_m, spec.node_mem_mi, trace)
    return venv, ora


def _compare_state(venv, ora):
    fc, fm, used = (x.cpu().numpy() for x in venv.node_state())
    efc, efm, eused = ora.node_state()
    np.testing.assert_array_equal(fc, efc)
    np.testing.assert_array_equal(fm, efm)
    np.testing.assert_array_equal(used, eused)


@pytest.mark.parametrize("mode", ["poisson", "bursty"])
def test_nodes_match_oracle(mode):
    from rlks.env import bursty_trace

    n, C, nodes, steps = 512, 8, 64, 230
    trace = bursty_trace() if mode == "bursty" else None
    venv, ora = _pair(n, C, nodes, trace=trace, penalty=0.25 if mode == "bursty" else 0.0,
                      depart=0.3 if mode == "bursty" else 0.05)
    venv.counters(enable=1)
    _compare_state(venv, ora)  # creation-time occupancy (episode 0)
    np.testing.assert_array_equal(venv.reset().cpu().numpy().view(np.uint32), ora.reset().view(np.uint32))
    _compare_state(venv, ora)
    rng = np.random.default_rng(1)
    for t in range(steps):
        a = rng.integers(0, C, n).astype(np.int32)
        obs, rew, term, _, info = venv.step(torch.from_numpy(a).to(venv.device))
        eo, er, et, es, _, _ = ora.step(a)
        np.testing.assert_array_equal(obs.cpu().numpy().view(np.uint32), eo.view(np.uint32))
        np.testing.assert_array_equal(rew.cpu().numpy().view(np.uint64), er.view(np.uint64))
        np.testing.assert_array_equal(term.cpu().numpy(), et)
        if t % 23 == 0 or t == steps - 1:
            _compare_state(venv, ora)
    venv.check_status()
    got = venv.counters().cpu().numpy()
    exp = ora.counters()
    # the oracle also counted the creation/reset-free steps; both count only env steps
    np.testing.assert_array_equal(got, exp)
    assert exp[1] > 0 and exp[3] > 0


def test_nodes_full_c3_size():
    """BASELINE configs[2]: 65,536 envs x 8 clusters x 256 nodes — 20 steps bit-exact vs the oracle,
    then 200 more steps checked for the size-independent invariants of the integer state"""
    n, C, nodes = 65536, 8, 256
    venv, ora = _pair(n, C, nodes, rate=1.0, depart="stationary")
    venv.reset()
    ora.reset()
    rng = np.random.default_rng(2)
    for t in range(20):
        a = rng.integers(0, C, n).astype(np.int32)
        obs, rew, term, _, _ = venv.step(torch.from_numpy(a).to(venv.device))
        eo, er, et, _, _, _ = ora.step(a)
        if t % 5 == 4:
            np.testing.assert_array_equal(obs.cpu().numpy().view(np.uint32), eo.view(np.uint32))
            np.testing.assert_array_equal(rew.cpu().numpy().view(np.uint64), er.view(np.uint64))
    _compare_state(venv, ora)
    del ora
    cap_cpu = torch.from_numpy(venv.nodes.node_cpu_m).to(venv.device)
    cap_mem = torch.from_numpy(venv.nodes.node_mem_mi).to(venv.device)
    for t in range(200):
        a = torch.randint(0, C, (n,), dtype=torch.int32, device=venv.device)
        obs, _, _, _, _ = venv.step(a)
    venv.check_status()
    fc, fm, used = venv.node_state()
    assert bool((fc >= 0).all()) and bool((fm >= 0).all())
    assert bool((fc <= cap_cpu[None, :, None]).all()) and bool((fm <= cap_mem[None, :, None]).all())
    pods_c = (cap_cpu[None, :, None] - fc) // 100
    pods_m = (cap_mem[None, :, None] - fm) // 64
    assert torch.equal(pods_c, pods_m)
    assert torch.equal(used, (cap_cpu[None, :, None] - fc).sum(-1).to(torch.int32))
    util = used.float() / (nodes * cap_cpu[None, :]).float()
    assert torch.equal(obs[:, 2 * C:], util)


# ----------------------------------------------------------------------------- PPO on node envs
@pytest.mark.parametrize("C,nodes,H,N,T,mb,precision", [
    (8, 64, 256, 2048, 24, 8192, "auto"),    # c3 shape (obs 24, 8 actions), split-fp16 rollout forward
    (8, 64, 256, 1024, 16, 4096, "fp32"),    # same env, fp32-MFMA rollout forward
    (16, 32, 384, 512, 12, 2048, "auto"),    # generic-width path (hidden 384, obs 48, 16 actions)
])
def test_ppo_on_node_envs(C, nodes, H, N, T, mb, precision):
    """PPO rollout over node-level envs (rlks_rollout_ws: forward -> sample -> node step per step):
    transitions replayed bit-exactly by the C oracle fed the rollout's actions, logits / values
    vs the fp64 oracle, logp consistent, GAE, one SGD gradient, then two train() iterations"""
    from rlks import _lib
    from rlks.env import NodeSpec
    from rlks.ppo import PPO, PPOConfig
    from rlks.tables import synthetic_table

    d = _dev()
    tab = synthetic_table(C, 100, seed=7)
    spec = NodeSpec(C, nodes, arrival_rate=2.0, depart_prob=0.05, init_occupancy=0.5, reject_penalty=0.1)
    cfg = (PPOConfig().framework("torch")
           .training(train_batch_size=N * T, sgd_minibatch_size=mb, num_sgd_iter=2, lr=3e-4, gamma=0.99,
                     sgd_precision=precision, model={"fcnet_hiddens": [H, H]})
           .debugging(seed=5))
    cfg.num_envs, cfg.table, cfg.nodes = N, tab, spec
    algo = PPO(config=cfg, device=d)
    assert algo.T == T and algo.D == 3 * C and algo.A == C
    assert algo.precision == ("wide" if H != 256 else ("fp32" if precision == "fp32" else "sf16"))
    algo.rollout(explore=True)
    b = {k: v.cpu().numpy() for k, v in algo.buf.items()}
    assert b["actions"].min() >= 0 and b["actions"].max() < C and len(np.unique(b["actions"])) == C
    ora = oracle.OracleEnv(oracle.make_cfg(N, 100, C, noise_mode=0, seed=5, autoreset=1, nodes=nodes, arrival_rate=2.0,
                                           depart_prob=0.05, init_occupancy=0.5, reject_penalty=0.1),
                           tab.cost, tab.latency, spec.node_cpu_m, spec.node_mem_mi, None)
    np.testing.assert_array_equal(ora.reset().view(np.uint32), b["obs"][0].view(np.uint32))
    for t in range(T):
        o, r, term, _, _, _ = ora.step(b["actions"][t])
        np.testing.assert_array_equal(o.view(np.uint32), b["obs"][t + 1].view(np.uint32))
        np.testing.assert_array_equal(r.astype(np.float32).view(np.uint32), b["rewards"][t].view(np.uint32))
        np.testing.assert_array_equal(term, b["dones"][t])
    close_as_fp32(b["logp"], logp_of(b["logits"], b["actions"]), logp_of(b["logits"], b["actions"], np.float32),
                  what="logp")
    flat = algo.params.flat.cpu().numpy()
    for t in (0, T // 2, T):
        el, ev = oracle.mlp_forward(flat, algo.params.offsets, 3 * C, H, C, b["obs"][t])
        fl, fv = oracle.mlp_forward_fp32_band(flat, algo.params.offsets, 3 * C, H, C, b["obs"][t])
        close_as_fp32(b["values"][t], ev, fv, what=f"values[{t}]")
        if t < T:
            close_as_fp32(b["logits"][t], el, fl, what=f"logits[{t}]")
    algo.advantages()
    ea, evt = oracle.gae(b["rewards"], b["values"], b["dones"], 0.99, 1.0)
    fa, fvt = gae_fp32_serial(b["rewards"], b["values"], b["dones"], 0.99, 1.0)
    close_as_fp32(algo.buf["adv"].cpu().numpy(), ea, fa, what="adv")
    close_as_fp32(algo.buf["vtarg"].cpu().numpy(), evt, fvt, what="vtarg")
    _lib.call("rlks_ppo_gather", C_.byref(algo.params.desc), C_.byref(algo.bufs), 3, 0, 0, algo.mb,
              algo.dyn.data_ptr(), algo.mbuf.data_ptr(), None)
    mbh = algo.mbuf.cpu().numpy()
    dyn = algo.dyn.cpu().numpy()
    _lib.call("rlks_ppo_grad", C_.byref(algo.params.desc), C_.byref(algo.coeffs), algo.params.flat.data_ptr(),
              algo.dyn.data_ptr(), algo.mbuf.data_ptr(), algo.mb, algo.grad.data_ptr(), None, algo.ws.data_ptr(),
              algo.ws.numel(), None)
    kw = dict(kl_coeff=float(dyn[2]), adv_mean=float(dyn[0]), adv_inv_std=float(dyn[1]))
    eg, est = oracle.ppo_loss_grad(flat, algo.params.offsets, 3 * C, H, C, mbh, **kw, scale=True)
    eg32 = oracle.ppo_loss_grad_fp32_band(flat, algo.params.offsets, 3 * C, H, C, mbh, **kw)
    g = algo.grad.cpu().numpy()
    assert np.linalg.norm(g - eg) <= 1e-5 * np.linalg.norm(eg)
    grad_close_as_fp32(g, eg, eg32, algo.params.offsets, algo.params.shapes, scale=est["scale"])
    for _ in range(2):
        r = algo.train()
        assert np.isfinite(r["info"]["learner"]["default_policy"]["learner_stats"]["policy_loss"])
    assert bool(torch.isfinite(algo.params.flat).all())


@pytest.mark.parametrize("C,N,T", [(4, 1000, 32), (2, 77, 256), (8, 2056, 32)])  # N T % 256 == 0 (sf16)
def test_node_rollout_ragged_lanes(C, N, T):
    """node_rollout's split-fp16 forward (k_sf_fwd16, 16-row tiles of 128-row workgroups) with a
    lane count that is not a multiple of 16 / 128: logits and values of every lane, the last
    partial tile included, per element against fp64 / fp32 references; transitions bit-exact"""
    from rlks.env import NodeSpec
    from rlks.ppo import PPO, PPOConfig
    from rlks.tables import synthetic_table

    d = _dev()
    tab = synthetic_table(C, 100, seed=3)
    spec = NodeSpec(C, 16, arrival_rate=1.0, depart_prob=0.05, init_occupancy=0.5)
    cfg = (PPOConfig().framework("torch")
           .training(train_batch_size=N * T, sgd_minibatch_size=N * T, num_sgd_iter=1, lr=3e-4)
           .debugging(seed=11))
    cfg.num_envs, cfg.table, cfg.nodes = N, tab, spec
    cfg.rollout_fragment_length = T
    algo = PPO(config=cfg, device=d)
    assert algo.precision == "sf16" and algo.A == C
    algo.rollout(explore=True)
    b = {k: v.cpu().numpy() for k, v in algo.buf.items()}
    ora = oracle.OracleEnv(oracle.make_cfg(N, 100, C, noise_mode=0, seed=11, autoreset=1, nodes=16, arrival_rate=1.0,
                                           depart_prob=0.05, init_occupancy=0.5),
                           tab.cost, tab.latency, spec.node_cpu_m, spec.node_mem_mi, None)
    np.testing.assert_array_equal(ora.reset().view(np.uint32), b["obs"][0].view(np.uint32))
    for t in range(T):
        o, r, term, _, _, _ = ora.step(b["actions"][t])
        np.testing.assert_array_equal(o.view(np.uint32), b["obs"][t + 1].view(np.uint32))
    flat = algo.params.flat.cpu().numpy()
    for t in (0, 1, T):
        el, ev = oracle.mlp_forward(flat, algo.params.offsets, 3 * C, 256, C, b["obs"][t])
        fl, fv = oracle.mlp_forward_fp32_band(flat, algo.params.offsets, 3 * C, 256, C, b["obs"][t])
        close_as_fp32(b["values"][t], ev, fv, what=f"values[{t}]")
        if t < T:
            close_as_fp32(b["logits"][t], el, fl, what=f"logits[{t}]")


def test_node_rollout_full_c3_size():
    """BASELINE configs[2] through the agent: PPO.rollout over 65,536 envs x 8 clusters x 256 nodes
    (bench.py's c3 env: Poisson(1) arrivals, stationary departures), T = 4 steps of node_rollout
    (forward of both nets -> Categorical sample -> node step).  Every transition replays bit-exactly
    in the C oracle fed the rollout's actions (obs, f32 rewards, dones, and every node's free cpu /
    mem at the end); every sampled action equals the Philox inverse-CDF draw recomputed on the CPU
    from the stored logits (up to draws within 4 float32 ulp of a CDF boundary, bounded at 1e-4);
    logits / values / logp per element against fp64 and fp32 references (tests/parity.py)"""
    from bench import env_setup
    from rlks.ppo import PPO, PPOConfig

    d = _dev()
    N, T, seed = 65536, 4, 42
    tab, spec = env_setup("c3")
    cfg = (PPOConfig().framework("torch")
           .training(train_batch_size=N * T, sgd_minibatch_size=65536, num_sgd_iter=1, lr=3e-4, gamma=0.99)
           .debugging(seed=seed))
    cfg.num_envs, cfg.table, cfg.nodes = N, tab, spec
    cfg.rollout_fragment_length = T
    algo = PPO(config=cfg, device=d)
    assert algo.T == T and algo.D == 24 and algo.A == 8 and algo.precision == "sf16"
    algo.rollout(explore=True)
    b = {k: v.cpu().numpy() for k, v in algo.buf.items()}
    ora = oracle.OracleEnv(oracle.make_cfg(N, tab.n_rows, 8, noise_mode=0, seed=seed, autoreset=1, nodes=256,
                                           arrival_rate=spec.arrival_rate, depart_prob=spec.depart_prob,
                                           init_occupancy=spec.init_occupancy, reject_penalty=spec.reject_penalty),
                           tab.cost, tab.latency, spec.node_cpu_m, spec.node_mem_mi, None)
    np.testing.assert_array_equal(ora.reset().view(np.uint32), b["obs"][0].view(np.uint32))
    gids = np.arange(N)
    amb = 0
    for t in range(T):
        st, ep = ora.lane_counters()
        act, margin = oracle.sample_actions(b["logits"][t], gids, ep, st, seed)
        near = margin < 4.0
        amb += int(near.sum())
        bad = (act != b["actions"][t]) & ~near
        assert not bad.any(), f"t={t}: {int(bad.sum())} sampled actions differ from the Philox inverse CDF"
        o, r, term, _, _, _ = ora.step(b["actions"][t])
        np.testing.assert_array_equal(o.view(np.uint32), b["obs"][t + 1].view(np.uint32))
        np.testing.assert_array_equal(r.astype(np.float32).view(np.uint32), b["rewards"][t].view(np.uint32))
        np.testing.assert_array_equal(term, b["dones"][t])
    assert amb <= 1e-4 * N * T, amb
    assert len(np.unique(b["actions"])) == 8
    _compare_state(algo.env, ora)
    close_as_fp32(b["logp"], logp_of(b["logits"], b["actions"]), logp_of(b["logits"], b["actions"], np.float32),
                  what="logp")
    flat = algo.params.flat.cpu().numpy()
    rows = slice(0, 16384)   # a quarter of the lanes: the fp64 / fp32 CPU forwards stay in seconds
    for t in (0, T):
        el, ev = oracle.mlp_forward(flat, algo.params.offsets, 24, 256, 8, b["obs"][t][rows])
        fl, fv = oracle.mlp_forward_fp32_band(flat, algo.params.offsets, 24, 256, 8, b["obs"][t][rows])
        close_as_fp32(b["values"][t][rows], ev, fv, what=f"values[{t}]")
        if t < T:
            close_as_fp32(b["logits"][t][rows], el, fl, what=f"logits[{t}]")


def test_node_rollout_two_streams_equal_one_stream(monkeypatch):
    """node_rollout can run its lanes in two halves on two streams (one half's node
    step beside the other half's forward; RLKS_NODE_TWO_STREAMS=1, measured no faster at c3).  With a lane count whose halves are ragged (12,000 lanes:
    5,888 + 6,112) the rollout buffers and the env state equal the single-stream order's bit for bit,
    and both replay in the C oracle"""
    from rlks.env import NodeSpec
    from rlks.ppo import PPO, PPOConfig
    from rlks.tables import synthetic_table

    d = _dev()
    N, T, C = 12000, 16, 8
    tab = synthetic_table(C, 100, seed=5)
    spec = NodeSpec(C, 64, arrival_rate=1.5, depart_prob=0.03, init_occupancy=0.5)
    out = []
    for one in (True, False):
        if one:
            monkeypatch.delenv("RLKS_NODE_TWO_STREAMS", raising=False)
        else:
            monkeypatch.setenv("RLKS_NODE_TWO_STREAMS", "1")
        cfg = (PPOConfig().framework("torch")
               .training(train_batch_size=N * T, sgd_minibatch_size=N * T // 4, num_sgd_iter=1, lr=3e-4)
               .debugging(seed=21))
        cfg.num_envs, cfg.table, cfg.nodes = N, tab, spec
        cfg.rollout_fragment_length = T
        algo = PPO(config=cfg, device=d)
        algo.rollout(explore=True)
        algo.rollout(explore=True)  # the second one starts from the carried observations
        torch.cuda.synchronize()
        out.append(({k: v.cpu().numpy() for k, v in algo.buf.items()}, algo.env.save_state().cpu().numpy()))
    (b1, s1), (b2, s2) = out
    for k in b1:
        np.testing.assert_array_equal(b1[k].view(np.uint8), b2[k].view(np.uint8), err_msg=k)
    # the snapshot's segments (rlks_env_save_state order, 256-byte aligned)
    al = lambda b: (b + 255) // 256 * 256  # noqa: E731
    segs = [("step", 4 * N), ("episode", 4 * N), ("ep_ret", 8 * N), ("ret_sum", 8 * N), ("ep_cnt", 4 * N),
            ("free", 8 * C * 64 * N), ("chunk", 2 * C * 8 * N), ("used_cpu", 4 * C * N)]
    o = 0
    for name, nb in segs:
        a, b = s1[o:o + nb], s2[o:o + nb]
        bad = np.nonzero(a != b)[0]
        assert bad.size == 0, f"{name}: {bad.size} bytes differ, first at byte {bad[:8].tolist()}"
        o += al(nb)
    assert o == s1.size
