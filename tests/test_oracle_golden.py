"""Pin the CPU oracle against the golden vectors generated from the reference env itself
(tools/make_goldens.py).  CPU only."""
import json

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

POLICIES = ["all0", "all1", "rr", "greedy", "rand"]
SEEDS = [0, 7, 42]


def test_mt19937_matches_cpython_streams(mt_draws):
    seeds = [int(s) for s in mt_draws["seeds"]]
    for i, s in enumerate(seeds):
        got = oracle.mt_random(s, 1500)
        np.testing.assert_array_equal(got.view(np.uint64), mt_draws[f"s{i}"].view(np.uint64))


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    assert list(oracle.philox([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(oracle.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2)) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(oracle.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0])) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def _policy(pol, t, step, obs, rand):
    if pol == "all0":
        return 0
    if pol == "all1":
        return 1
    if pol == "rr":
        return 0 if step % 2 == 0 else 1
    if pol == "greedy":
        return 0 if obs[0] <= obs[1] else 1
    return int(rand[t])


def replay_oracle(cost, lat, seed, pol, rand):
    env = oracle.OracleEnv(oracle.make_cfg(1, 100, 2, noise_mode=1), cost, lat)
    env.seed(0, seed)
    obs = env.reset()
    out = {"obs": [obs[0].copy()], "reward": [], "done": [], "step": [], "action": []}
    t = 0
    while True:
        a = _policy(pol, t, env.lane_step(0), obs[0], rand)
        obs, rew, term, step, _, status = env.step([a])
        assert status[0] == 0 and status[1] == 0
        out["obs"].append(obs[0].copy())
        out["reward"].append(rew[0])
        out["done"].append(term[0])
        out["step"].append(step[0])
        out["action"].append(a)
        t += 1
        if term[0]:
            break
    _, _, _, step, _, status = env.step([0])
    return {k: np.array(v) for k, v in out.items()}, status, step[0], env.lane_step(0)


@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("pol", POLICIES)
def test_oracle_replays_reference_traces(golden_cost_lat, traces, traces_meta, seed, pol):
    cost, lat = golden_cost_lat
    got, status, _, cs_after = replay_oracle(cost, lat, seed, pol, traces["rand_actions"])
    key = f"s{seed}_{pol}"
    np.testing.assert_array_equal(got["obs"].view(np.uint32), traces[key + "_obs"].view(np.uint32))
    np.testing.assert_array_equal(got["reward"].view(np.uint64), traces[key + "_reward"].view(np.uint64))
    np.testing.assert_array_equal(got["done"], traces[key + "_done"])
    np.testing.assert_array_equal(got["step"], traces[key + "_step"])
    np.testing.assert_array_equal(got["action"], traces[key + "_action"])
    # stepping past the last row: reference IndexError after current_step was incremented
    ie = traces_meta["index_error"][f"{seed}_{pol}"]
    assert ie["raised"] and status[1] == 1 and cs_after == ie["current_step_after"]


def test_oracle_episode_returns(golden_cost_lat, traces, traces_meta):
    cost, lat = golden_cost_lat
    for pol in POLICIES:
        got, _, _, _ = replay_oracle(cost, lat, 42, pol, traces["rand_actions"])
        acc = 0.0
        for r in got["reward"]:
            acc += float(r)
        assert acc == traces_meta["returns"][pol]
    assert traces_meta["returns"]["rr"] == 4765.215199784463


def test_unseeded_reset_continues_stream(golden_cost_lat, traces):
    cost, lat = golden_cost_lat
    env = oracle.OracleEnv(oracle.make_cfg(1, 100, 2, noise_mode=1), cost, lat)
    env.seed(0, 42)
    obs = env.reset()
    seq = [obs[0].copy()]
    for ep in range(2):
        if ep == 1:
            obs = env.reset()
            seq.append(obs[0].copy())
        while True:
            a = 0 if env.lane_step(0) % 2 == 0 else 1
            obs, _, term, _, _, _ = env.step([a])
            seq.append(obs[0].copy())
            if term[0]:
                break
    np.testing.assert_array_equal(np.stack(seq).view(np.uint32), traces["cont_s42_rr_obs"].view(np.uint32))


def test_autoreset_matches_step_then_reset(golden_cost_lat):
    """vector-env auto-reset consumes the terminal obs draws, then the reset draws (reference order)"""
    cost, lat = golden_cost_lat
    a = oracle.OracleEnv(oracle.make_cfg(1, 100, 2, noise_mode=1, autoreset=1), cost, lat)
    b = oracle.OracleEnv(oracle.make_cfg(1, 100, 2, noise_mode=1, autoreset=0), cost, lat)
    a.seed(0, 3); b.seed(0, 3)
    a.reset(); b.reset()
    for t in range(250):
        oa, ra, ta, _, fa, _ = a.step([t % 2])
        ob, rb, tb, _, _, _ = b.step([t % 2])
        assert ra[0] == rb[0] and ta[0] == tb[0]
        if tb[0]:
            np.testing.assert_array_equal(fa, ob)
            ob = b.reset()
        np.testing.assert_array_equal(oa, ob)


def test_gae_oracle_matches_lfilter_goldens():
    g = np.load(GOLDEN / "gae.npz")
    for ci in range(3):
        gamma, lam = g[f"c{ci}_params"]
        adv, vt = oracle.gae(g[f"c{ci}_r"], g[f"c{ci}_v"], g[f"c{ci}_d"], gamma, lam)
        np.testing.assert_allclose(adv, g[f"c{ci}_adv"], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(vt, g[f"c{ci}_vt"], rtol=1e-12, atol=1e-12)


def test_action_validity_matches_reference():
    from rlks.spaces import Discrete

    validity = json.loads((GOLDEN / "action_validity.json").read_text())
    cases = {
        "int0": 0, "int1": 1, "int2": 2, "int_neg1": -1, "bool_true": True, "bool_false": False,
        "np_int64_1": np.int64(1), "np_int32_0": np.int32(0), "np_uint8_1": np.uint8(1),
        "np_0d_int_1": np.array(1), "np_0d_int_2": np.array(2), "np_1d_int": np.array([1]),
        "float_1": 1.0, "np_float32_0": np.float32(0), "str_1": "1", "none": None,
        "np_int64_big": np.int64(2**40),
    }
    d = Discrete(2)
    for name, a in cases.items():
        assert d.contains(a) == validity[name], name


def test_packaged_table_is_reference_bits(golden_table):
    from rlks.tables import PACKAGED, load_table

    t = load_table(None) if not (GOLDEN / "..").joinpath("data").exists() else None
    z = np.load(PACKAGED)
    np.testing.assert_array_equal(z["table"].view(np.uint64), golden_table.view(np.uint64))
    if t is not None:
        np.testing.assert_array_equal(t.cost.view(np.uint64), golden_table[:, [1, 2]].view(np.uint64))
