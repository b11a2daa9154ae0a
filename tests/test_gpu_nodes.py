"""GPU parity of the node-level env extension (clusters x nodes, Poisson / bursty pod
arrivals, first-fit placement, integer resource accounting) against the C oracle: observations,
f64 rewards, terminations, every node's free millicores / MiB, the per-cluster aggregates and the
placement counters must be bit-identical."""
import numpy as np
import pytest

import oracle

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
