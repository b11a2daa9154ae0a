"""CPU tests of the node-level env extension in the oracle: invariants of the
integer cluster state, first-fit placement and the reduction to the reference at zero nodes."""
import numpy as np
import pytest

import oracle


def _tables(C, T=100, seed=1):
    from rlks.tables import synthetic_table

    t = synthetic_table(C, T, seed=seed)
    return t.cost, t.latency


def _caps(C):
    # t3.micro-like (2 vCPU / 1 GiB) and Standard_B2s-like (2 vCPU / 4 GiB) node types alternate
    return np.full(C, 2000, np.int32), np.array([1024 if c % 2 == 0 else 4096 for c in range(C)], np.int32)


def _check_invariants(env, cap_cpu, cap_mem, req=(100, 64)):
    fc, fm, used = env.node_state()
    assert (fc >= 0).all() and (fm >= 0).all()
    assert (fc <= cap_cpu[None, :, None]).all() and (fm <= cap_mem[None, :, None]).all()
    pods_c = (cap_cpu[None, :, None] - fc) // req[0]
    pods_m = (cap_mem[None, :, None] - fm) // req[1]
    np.testing.assert_array_equal(pods_c, pods_m)                 # homogeneous pods
    np.testing.assert_array_equal(used, (cap_cpu[None, :, None] - fc).sum(-1))  # aggregate = sum of nodes
    return fc, used


@pytest.mark.parametrize("mode", [0, 1])
def test_node_state_invariants_and_obs(mode):
    C, N, n = 8, 32, 64
    cost, lat = _tables(C)
    cc, cm = _caps(C)
    trace = np.concatenate([np.linspace(0.0, 3.0, 20), np.full(80, 1.5)]) if mode else None
    env = oracle.OracleEnv(oracle.make_cfg(n, 100, C, noise_mode=0, seed=3, autoreset=1, nodes=N, arrival_mode=mode,
                                           arrival_rate=2.0, depart_prob=0.1, init_occupancy=0.5),
                           cost, lat, cc, cm, trace)
    obs = env.reset()
    assert obs.shape == (n, 3 * C)
    rng = np.random.default_rng(0)
    for t in range(250):
        a = rng.integers(0, C, n).astype(np.int32)
        obs, rew, term, step, _, st = env.step(a)
        assert st[0] == 0 and st[1] == 0
        fc, used = _check_invariants(env, cc, cm)
        util = used.astype(np.float32) / (N * cc[None, :]).astype(np.float32)
        np.testing.assert_array_equal(obs[:, 2 * C:], util)
        row = np.where(term.astype(bool), 0, step)  # auto-reset lanes show their new episode's row 0
        np.testing.assert_array_equal(obs[:, :C], cost[row].astype(np.float32))
    scanned, placed, rejected, departed, written, reads = env.counters()
    assert placed > 0 and scanned >= placed and departed > 0 and written > 0 and reads > 0


def test_first_fit_places_on_lowest_fitting_node():
    """one lane, no departures: every arrival lands on the lowest node with room"""
    C, N = 2, 8
    cost, lat = _tables(C)
    cc, cm = np.array([300, 300], np.int32), np.array([4096, 4096], np.int32)  # 3 pods per node
    env = oracle.OracleEnv(oracle.make_cfg(1, 100, C, noise_mode=0, seed=1, nodes=N, arrival_rate=1.5,
                                           depart_prob=0.0, init_occupancy=0.0), cost, lat, cc, cm)
    env.reset()
    prev = env.node_state()[0][0, 0].copy()
    for t in range(40):
        env.step(np.array([0], np.int32))
        fc = env.node_state()[0][0, 0]
        pods = (300 - fc) // 100
        # first-fit with identical pods fills nodes in order: a non-increasing occupancy profile
        assert (np.diff(pods) <= 0).all()
        changed = np.nonzero(fc != prev)[0]
        if changed.size:
            assert (prev[: changed.min()] < 100).all()  # every lower node was already full
        prev = fc.copy()
    _, placed, rejected, _, _, _ = env.counters()
    assert placed == min(placed + rejected, 3 * N) and rejected >= 0


def test_zero_nodes_is_the_reference_env(golden_cost_lat, traces):
    """nodes_per_cluster = 0 keeps the reference behaviour (the node fields are inert)"""
    cost, lat = golden_cost_lat
    env = oracle.OracleEnv(oracle.make_cfg(1, 100, 2, noise_mode=1, nodes=0, depart_prob=0.9, arrival_rate=5.0,
                                           reject_penalty=3.0), cost, lat)
    env.seed(0, 42)
    obs = env.reset()
    seq = [obs[0].copy()]
    while True:
        a = 0 if env.lane_step(0) % 2 == 0 else 1
        obs, _, term, _, _, _ = env.step([a])
        seq.append(obs[0].copy())
        if term[0]:
            break
    np.testing.assert_array_equal(np.stack(seq).view(np.uint32), traces["s42_rr_obs"].view(np.uint32))


def test_reject_penalty_applies():
    C, N = 2, 8
    cost, lat = _tables(C)
    cc, cm = np.array([100, 100], np.int32), np.array([64, 64], np.int32)  # one pod per node
    base = oracle.OracleEnv(oracle.make_cfg(16, 100, C, noise_mode=0, seed=2, nodes=N, arrival_rate=3.0,
                                            depart_prob=0.0, init_occupancy=1.0), cost, lat, cc, cm)
    pen = oracle.OracleEnv(oracle.make_cfg(16, 100, C, noise_mode=0, seed=2, nodes=N, arrival_rate=3.0,
                                           depart_prob=0.0, init_occupancy=1.0, reject_penalty=0.5), cost, lat, cc, cm)
    base.reset(); pen.reset()
    a = np.zeros(16, np.int32)
    tot = 0
    for _ in range(20):
        _, r0, _, _, _, _ = base.step(a)
        _, r1, _, _, _, _ = pen.step(a)
        assert (r1 <= r0).all()
        tot += (r0 - r1).sum()
    assert tot == 0.5 * pen.counters()[2]


def test_departure_skip_table():
    """the departure-skip table is the geometric survival (1 - p)^j to 2^-32, non-increasing, capped
    at 2^32 - 1, and ends at pmax or where it reaches 0"""
    for p, pmax in ((0.0, 50), (1.1e-4, 10240), (0.02, 65536), (0.3, 500), (0.5, 100), (1.0, 10)):
        s = oracle.skip32(pmax, p).astype(np.int64)
        j = np.arange(len(s))
        ref = np.minimum(np.round((1.0 - p) ** j * 2.0**32), 2**32 - 1)
        assert s[0] == 2**32 - 1 and (np.diff(s) <= 0).all() and (s > 0).all()
        assert np.abs(s - ref).max() <= 2, p
        if len(s) < pmax + 1:
            assert np.round((1.0 - p) ** len(s) * 2.0**32) == 0, p


def test_departure_skip_estimate_bound():
    """the device decides u < S[x] without the table where u is more than 2^16 from the fp32 estimate
    exp2(x * log2(1 - p)) 2^32 (env.hip:u_below_S): that estimate, computed in fp32 as the device does,
    stays within 2^12 of the table for every entry (16x inside the margin, for the device exp2's ulps)"""
    for p in (1e-6, 1e-5, 1.085e-4, 1e-3, 5e-3, 0.02, 0.05, 0.1, 0.3, 0.5, 0.9, 0.99):
        s = oracle.skip32(20000, p).astype(np.float64)
        x = np.arange(len(s), dtype=np.float32)
        lg1p = np.float32(np.log1p(-np.float32(p))) * np.float32(1.4426950408889634)
        est = np.exp2((x * np.float32(lg1p)).astype(np.float32)).astype(np.float32) * np.float32(2.0**32)
        assert np.abs(est.astype(np.float64) - s).max() <= 2.0**12, p
        # a table cut short where it reaches 0 (entries past it read as 0; a full table covers every
        # pod count the clusters can hold): the estimate there is as close to 0
        if len(s) < 20001:
            tail = np.float32(np.exp2(np.float32(len(s)) * lg1p)) * np.float32(2.0**32)
            assert tail <= 2.0**12, p


@pytest.mark.parametrize("p", [0.0, 1e-3, 0.05, 1.0])
def test_departures_are_geometric_per_pod(p):
    """no arrivals: each step every pod leaves with probability p (mean over many nodes)"""
    C, N, n = 2, 64, 256
    cost, lat = _tables(C)
    cc, cm = np.array([2000, 2000], np.int32), np.array([4096, 4096], np.int32)
    env = oracle.OracleEnv(oracle.make_cfg(n, 100, C, noise_mode=0, seed=9, nodes=N, arrival_rate=0.0,
                                           depart_prob=p, init_occupancy=1.0), cost, lat, cc, cm)
    env.reset()
    pods0 = ((2000 - env.node_state()[0]) // 100).sum()
    a = np.zeros(n, np.int32)
    env.step(a)
    pods1 = ((2000 - env.node_state()[0]) // 100).sum()
    left = pods0 - pods1
    assert env.counters()[3] == left
    if p in (0.0, 1.0):
        assert left == p * pods0
    else:
        sd = np.sqrt(pods0 * p * (1 - p))
        assert abs(left - p * pods0) < 5 * sd
