"""GPU parity of the env kernel (K1) and RNGs (K2) against the reference goldens and the oracle."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def test_philox_device_known_answers():
    from rlks import _lib

    d = _dev()
    ctr = torch.tensor([[0, 0, 0, 0], [-1, -1, -1, -1], [0x243F6A88, 0x85A308D3 - 2**32, 0x13198A2E, 0x03707344]],
                       dtype=torch.int32, device=d)
    outs = []
    for key in ([0, 0], [-1, -1], [0xA4093822 - 2**32, 0x299F31D0]):
        k = torch.tensor(key, dtype=torch.int32, device=d)
        o = torch.zeros(3, 4, dtype=torch.int32, device=d)
        _lib.call("rlks_philox4x32_10", ctr.data_ptr(), k.data_ptr(), o.data_ptr(), 3, None)
        outs.append(o.cpu().numpy().view(np.uint32))
    assert list(outs[0][0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert list(outs[1][1]) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(outs[2][2]) == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]
    # and random counters vs the C oracle
    rng = np.random.default_rng(1)
    c = rng.integers(0, 2**32, (257, 4), dtype=np.uint64).astype(np.uint32)
    k = np.array([123456789, 987654321], np.uint32)
    ct = torch.from_numpy(c.view(np.int32)).to(d)
    kt = torch.from_numpy(k.view(np.int32)).to(d)
    o = torch.zeros(257, 4, dtype=torch.int32, device=d)
    _lib.call("rlks_philox4x32_10", ct.data_ptr(), kt.data_ptr(), o.data_ptr(), 257, None)
    got = o.cpu().numpy().view(np.uint32)
    for i in range(0, 257, 16):
        assert list(got[i]) == list(oracle.philox(c[i], k))


def test_mt19937_device_matches_cpython(mt_draws):
    from rlks import _lib
    from rlks.env import seed_key_words

    d = _dev()
    seeds = [int(s) for s in mt_draws["seeds"]]
    for i, s in enumerate(seeds):
        w = np.array(seed_key_words(s), np.uint32)
        kt = torch.from_numpy(w.view(np.int32)).to(d)
        out = torch.zeros(1500, dtype=torch.float64, device=d)
        _lib.call("rlks_mt_random", kt.data_ptr(), len(w), out.data_ptr(), 1500, None)
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint64), mt_draws[f"s{i}"].view(np.uint64))


POLICIES = ["all0", "all1", "rr", "greedy", "rand"]


@pytest.mark.parametrize("stream", ["instance", "global"])
@pytest.mark.parametrize("seed", [0, 7, 42])
@pytest.mark.parametrize("pol", POLICIES)
def test_dropin_env_replays_reference(traces, traces_meta, seed, pol, stream):
    """K8sMultiCloudEnv (GPU lane, MT19937 noise) reproduces the reference env bit for bit, with a
    private noise generator and on the process-global `random` stream"""
    from rlks import K8sMultiCloudEnv

    _dev()
    env = K8sMultiCloudEnv(noise_stream=stream)
    assert env.max_steps == 99
    obs, info = env.reset(seed=seed)
    assert info == {} and obs.dtype == np.float32 and obs.shape == (6,)
    key = f"s{seed}_{pol}"
    obs_l, rew_l, done_l, step_l, cloud_l = [obs], [], [], [], []
    rand = traces["rand_actions"]
    t, done = 0, False
    while not done:
        if pol == "all0":
            a = 0
        elif pol == "all1":
            a = 1
        elif pol == "rr":
            a = 0 if env.current_step % 2 == 0 else 1
        elif pol == "greedy":
            a = env.normal_scheduler_step(obs)
        else:
            a = int(rand[t])
        obs, r, done, trunc, info = env.step(a)
        assert trunc is False and isinstance(r, float) and isinstance(done, bool)
        obs_l.append(obs)
        rew_l.append(r)
        done_l.append(done)
        step_l.append(info["step"])
        cloud_l.append(0 if info["chosen_cloud"] == "aws" else 1)
        t += 1
    np.testing.assert_array_equal(np.stack(obs_l).view(np.uint32), traces[key + "_obs"].view(np.uint32))
    np.testing.assert_array_equal(np.array(rew_l).view(np.uint64), traces[key + "_reward"].view(np.uint64))
    np.testing.assert_array_equal(np.array(done_l, np.uint8), traces[key + "_done"])
    np.testing.assert_array_equal(np.array(step_l), traces[key + "_step"])
    np.testing.assert_array_equal(np.array(cloud_l), traces[key + "_cloud"])
    acc = 0.0
    for r in rew_l:
        acc += r
    assert acc == traces_meta["returns"][pol]
    with pytest.raises(IndexError):
        env.step(0)
    assert env.current_step == traces_meta["index_error"][f"{seed}_{pol}"]["current_step_after"]


def test_dropin_invalid_actions_and_continuation(traces):
    from rlks import K8sMultiCloudEnv

    _dev()
    env = K8sMultiCloudEnv()
    env.reset(seed=0)
    for bad in (2, -1, 1.0, "1", None, np.array([1]), np.float32(0)):
        with pytest.raises(AssertionError, match="Invalid action"):
            env.step(bad)
    assert env.current_step == 0
    for good in (True, np.int64(1), np.array(0), np.uint8(1)):
        env.step(good)
    assert env.current_step == 4
    # reset(seed=42), an episode, reset() without seed continues the MT stream
    obs, _ = env.reset(seed=42)
    seq = [obs]
    for ep in range(2):
        if ep == 1:
            obs, _ = env.reset()
            seq.append(obs)
        done = False
        while not done:
            obs, _, done, _, _ = env.step(0 if env.current_step % 2 == 0 else 1)
            seq.append(obs)
    np.testing.assert_array_equal(np.stack(seq).view(np.uint32), traces["cont_s42_rr_obs"].view(np.uint32))


@pytest.mark.parametrize("noise,n,steps", [("philox", 1000, 260), ("mt19937", 96, 400), ("philox", 131072, 120)])
def test_vec_env_matches_oracle(golden_cost_lat, noise, n, steps):
    """batched lanes with auto-reset, bit-exact vs the C oracle (last case: c4's per-GPU lane count)"""
    from rlks import VecK8sMultiCloudEnv
    from rlks.tables import load_table

    d = _dev()
    cost, lat = golden_cost_lat
    table = load_table()
    venv = VecK8sMultiCloudEnv(n, table=table, seed=1234, noise=noise, env_offset=17, device=d)
    ora = oracle.OracleEnv(oracle.make_cfg(n, 100, 2, noise_mode=1 if noise == "mt19937" else 0, seed=1234,
                                           autoreset=1, env_offset=17), cost, lat)
    got = venv.reset().cpu().numpy()
    exp = ora.reset()
    np.testing.assert_array_equal(got.view(np.uint32), exp.view(np.uint32))
    rng = np.random.default_rng(5)
    for t in range(steps):
        a = rng.integers(0, 2, n).astype(np.int32)
        obs, rew, term, trunc, info = venv.step(torch.from_numpy(a).to(d))
        eo, er, et, es, ef, st = ora.step(a)
        if t % 7 == 0 or t == steps - 1 or n <= 1000:
            np.testing.assert_array_equal(obs.cpu().numpy().view(np.uint32), eo.view(np.uint32))
            np.testing.assert_array_equal(rew.cpu().numpy().view(np.uint64), er.view(np.uint64))
            np.testing.assert_array_equal(term.cpu().numpy(), et)
            np.testing.assert_array_equal(info["step"].cpu().numpy(), es)
            tm = et.astype(bool)
            np.testing.assert_array_equal(info["final_observation"].cpu().numpy()[tm].view(np.uint32),
                                          ef[tm].view(np.uint32))
    venv.check_status()


def test_lean_step_contract_matches_oracle(golden_cost_lat):
    """the plain gymnasium step (k_env_step2 through the ABI with trusted actions, no truncated /
    step / status outputs, no episode-return bookkeeping) is bit-exact vs the C oracle, including
    final observations of auto-reset lanes, and leaves the episode accumulators empty"""
    from rlks import VecK8sMultiCloudEnv, _lib

    d = _dev()
    cost, lat = golden_cost_lat
    n, steps = 4099, 230  # a ragged last workgroup; two auto-resets per lane
    venv = VecK8sMultiCloudEnv(n, seed=77, env_offset=5, device=d, track_returns=False)
    ora = oracle.OracleEnv(oracle.make_cfg(n, 100, 2, noise_mode=0, seed=77, autoreset=1, env_offset=5), cost, lat)
    np.testing.assert_array_equal(venv.reset().cpu().numpy().view(np.uint32), ora.reset().view(np.uint32))
    rng = np.random.default_rng(11)
    stream = torch.cuda.current_stream(d).cuda_stream
    for _ in range(steps):
        a = rng.integers(0, 2, n).astype(np.int32)
        acts = torch.from_numpy(a).to(d)
        _lib.call("rlks_env_step", venv.handle, acts.data_ptr(), venv.obs.data_ptr(), venv.reward.data_ptr(), None,
                  venv.terminated.data_ptr(), None, None, venv.final_obs.data_ptr(), None, stream)
        eo, er, et, es, ef, st = ora.step(a)
        np.testing.assert_array_equal(venv.obs.cpu().numpy().view(np.uint32), eo.view(np.uint32))
        np.testing.assert_array_equal(venv.reward.cpu().numpy().view(np.uint64), er.view(np.uint64))
        np.testing.assert_array_equal(venv.terminated.cpu().numpy(), et)
        tm = et.astype(bool)
        np.testing.assert_array_equal(venv.final_obs.cpu().numpy()[tm].view(np.uint32), ef[tm].view(np.uint32))
    steps_now, eps_now = venv.lane_state()
    assert int(eps_now.min()) == int(eps_now.max()) and bool((steps_now == steps - 2 * 99).all())
    s = venv.episode_stats(clear=True).cpu().numpy()
    assert s[0] == 0.0 and s[1] == 0.0


def test_vec_env_invalid_action_steps_nothing():
    from rlks import VecK8sMultiCloudEnv

    d = _dev()
    venv = VecK8sMultiCloudEnv(300, seed=3, device=d)
    venv.reset()
    a = torch.zeros(300, dtype=torch.int32, device=d)
    venv.step(a)
    before = venv.lane_state()[0].clone()
    a[77] = 2
    venv.step(a)
    with pytest.raises(AssertionError):
        venv.check_status()
    assert torch.equal(venv.lane_state()[0], before)


def test_vec_env_no_autoreset_overrun():
    from rlks import VecK8sMultiCloudEnv

    d = _dev()
    venv = VecK8sMultiCloudEnv(64, seed=3, autoreset=False, device=d)
    venv.reset()
    a = torch.ones(64, dtype=torch.int32, device=d)
    for _ in range(99):
        _, _, term, _, _ = venv.step(a)
    venv.check_status()
    assert bool(term.all())
    venv.step(a)
    with pytest.raises(IndexError):
        venv.check_status()


def test_episode_stats_match_returns():
    from rlks import VecK8sMultiCloudEnv

    d = _dev()
    venv = VecK8sMultiCloudEnv(128, seed=9, device=d)
    venv.reset()
    venv.episode_stats(clear=True)
    a = torch.zeros(128, dtype=torch.int32, device=d)
    tot = torch.zeros(128, dtype=torch.float64, device=d)
    for _ in range(99):
        _, r, _, _, _ = venv.step(a)
        tot += r
    s = venv.episode_stats(clear=True).cpu().numpy()
    assert s[1] == 128
    assert abs(s[0] / 128 - 4912.769165045401) < 1e-9


def test_global_stream_replays_interleaved_reference_envs():
    """noise_stream="global": two drop-in envs and the caller's own random.random() draws share the
    process-global stream in call order, as the reference's random.uniform does
    (k8s_multi_cloud_env.py:87, :109-111): tests/golden/global_stream.npz (tools/make_goldens.py,
    two reference envs interleaved after one random.seed, a mid-episode reset(seed) of one of them)
    replayed bit for bit"""
    import random

    from rlks import K8sMultiCloudEnv

    _dev()
    from conftest import GOLDEN

    g = np.load(GOLDEN / "global_stream.npz")
    random.seed(int(g["seed"]))
    np.random.seed(int(g["seed"]))
    envs = [K8sMultiCloudEnv(env_config={"noise_stream": "global"}), K8sMultiCloudEnv(noise_stream="global")]
    for i in range(len(g["kind"])):
        kind, e, arg = int(g["kind"][i]), int(g["env"][i]), int(g["arg"][i])
        if kind == 3:
            assert random.random() == g["draw"][i], i
            continue
        if kind == 2:
            obs, r, done, _, _ = envs[e].step(arg)
            assert np.float64(r).view(np.uint64) == g["reward"][i].view(np.uint64), i
            assert done == bool(g["done"][i]), i
        else:
            obs, _ = envs[e].reset(seed=arg if kind == 1 else None)
        np.testing.assert_array_equal(obs.view(np.uint32), g["obs"][i].view(np.uint32), err_msg=f"event {i}")
