#!/usr/bin/env python3
"""Generate the golden parity fixtures under tests/golden/ from the REFERENCE env.

Runs ONLY in the build container (needs /root/reference); never on the GPU box.
The fixtures are data (inputs + expected outputs); no reference source is copied.

How the reference is imported: `gymnasium` and `kubernetes` are not
installed here, so two minimal stub modules are injected into `sys.modules` and
`/root/reference/rl_scheduler/env/k8s_multi_cloud_env.py` is loaded unmodified via
importlib under a private module name. The env then reads its own CSV through its
own DATA_PATH (k8s_multi_cloud_env.py:22-27).

The gymnasium stub reproduces `spaces.Discrete.contains` (gymnasium semantics: python
int incl. bool, or a 0-d numpy integer; 0 <= x < n), which is what
`K8sMultiCloudEnv.step` asserts on (k8s_multi_cloud_env.py:116).

Outputs (all small):
  table.npz           float64 [100,7] table exactly as pandas parsed it (+ column names)
  mt_draws.npz        Python `random.random()` streams after `random.seed(s)` (compat RNG pin)
  traces.npz          per (seed, policy) replay traces: obs f32, reward f64, done, step, cloud
  traces_meta.json    keys of traces.npz, returns per policy, IndexError behaviour
  action_validity.json  which action values the reference accepts / rejects
  gae.npz             GAE goldens from scipy.signal.lfilter (RLlib discount_cumsum form)
  global_stream.npz   two envs + caller draws interleaved on the process-global `random` stream
                      (--only-global-stream regenerates just this file)
"""
from __future__ import annotations

import importlib.util
import json
import random
import sys
import types
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parents[1] / "tests" / "golden"


# ----------------------------------------------------------------------------- stubs
def _install_stubs() -> None:
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")

    class Env:
        def __init__(self, *a, **k):
            pass

        def reset(self, *, seed=None, options=None):
            return None

    class Discrete:
        def __init__(self, n, start=0):
            self.n = int(n)
            self.start = int(start)
            self._rng = np.random.default_rng(0)

        def contains(self, x) -> bool:  # gymnasium.spaces.Discrete.contains semantics
            if isinstance(x, int):
                as_int64 = np.int64(x)
            elif isinstance(x, (np.generic, np.ndarray)) and (
                np.issubdtype(x.dtype, np.integer) and x.shape == ()
            ):
                as_int64 = np.int64(x)
            else:
                return False
            return bool(self.start <= as_int64 < self.start + self.n)

        def sample(self):
            return int(self.start + self._rng.integers(self.n))

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    spaces.Discrete = Discrete
    spaces.Box = Box
    gym.Env = Env
    gym.spaces = spaces
    sys.modules["gymnasium"] = gym
    sys.modules["gymnasium.spaces"] = spaces

    k8s = types.ModuleType("kubernetes")
    k8s.client = types.SimpleNamespace()
    k8s.config = types.SimpleNamespace()
    sys.modules["kubernetes"] = k8s


def _load_reference_env():
    _install_stubs()
    path = REF / "rl_scheduler" / "env" / "k8s_multi_cloud_env.py"
    spec = importlib.util.spec_from_file_location("_ref_k8s_env", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


# ----------------------------------------------------------------------------- policies
def _policy(name, env, obs, t, rand_actions):
    if name == "all0":
        return 0
    if name == "all1":
        return 1
    if name == "rr":  # train_and_compare.py:65
        return 0 if env.current_step % 2 == 0 else 1
    if name == "greedy":  # k8s_multi_cloud_env.py:156-157
        return env.normal_scheduler_step(obs)
    if name == "rand":
        return int(rand_actions[t])
    raise KeyError(name)


POLICIES = ["all0", "all1", "rr", "greedy", "rand"]
SEEDS = [0, 7, 42]


# event codes of global_stream.npz
EV_RESET, EV_RESET_SEED, EV_STEP, EV_DRAW = 0, 1, 2, 3


def global_stream_golden(Env) -> None:
    """Two reference envs in one process sharing the process-global `random` stream
    (k8s_multi_cloud_env.py:87 draws the cpu noise from it, :109-111 reseeds it): after one
    random.seed(s), env 0 and env 1 are reset and stepped interleaved, the caller draws
    random.random() in between, one env is reset with a seed mid-episode (reseeding the stream the
    other is drawing from), and both run past an episode end.  Recorded per event: kind, env,
    argument, obs f32, reward f64, done, the caller's draw."""
    ev = []  # (kind, env, arg)
    rng = np.random.default_rng(2024)
    ev += [(EV_RESET, 0, 0), (EV_RESET, 1, 0)]
    steps = [0, 0]
    for t in range(230):
        e = int(rng.integers(0, 2))
        if steps[e] == 99:  # terminated: the next call would raise IndexError (:91)
            ev.append((EV_RESET, e, 0))
            steps[e] = 0
            continue
        ev.append((EV_STEP, e, int(rng.integers(0, 2))))
        steps[e] += 1
        if t % 7 == 3:
            ev.append((EV_DRAW, -1, 0))
        if t == 120:
            ev.append((EV_RESET_SEED, e, 99))
            steps[e] = 0
    out = {k: [] for k in ("kind", "env", "arg", "obs", "reward", "done", "draw")}
    random.seed(31337)
    np.random.seed(31337)
    envs = [Env(), Env()]
    for kind, e, arg in ev:
        obs, rew, done, draw = np.zeros(6, np.float32), 0.0, False, 0.0
        if kind == EV_RESET:
            obs, _ = envs[e].reset()
        elif kind == EV_RESET_SEED:
            obs, _ = envs[e].reset(seed=arg)
        elif kind == EV_STEP:
            obs, rew, done, _, _ = envs[e].step(arg)
        else:
            draw = random.random()
        for k, v in (("kind", kind), ("env", e), ("arg", arg), ("obs", obs), ("reward", rew), ("done", done),
                     ("draw", draw)):
            out[k].append(v)
    np.savez(OUT / "global_stream.npz", seed=np.array(31337), kind=np.array(out["kind"], np.int32),
             env=np.array(out["env"], np.int32), arg=np.array(out["arg"], np.int32),
             obs=np.array(out["obs"], np.float32), reward=np.array(out["reward"], np.float64),
             done=np.array(out["done"], np.uint8), draw=np.array(out["draw"], np.float64))


def main() -> None:
    OUT.mkdir(parents=True, exist_ok=True)
    mod = _load_reference_env()
    Env = mod.K8sMultiCloudEnv
    if "--only-global-stream" in sys.argv:
        global_stream_golden(Env)
        return

    # ---- table bits (pandas default parser; SURVEY §7.3: not correctly rounded)
    env = Env()
    cols = list(env.static_df.columns)
    table = env.static_df.to_numpy(dtype=np.float64)
    np.savez(OUT / "table.npz", table=table)
    assert env.max_steps == len(table) - 1 == 99

    # ---- MT19937 compat streams (Python random.seed(int) -> init_by_array)
    mt_seeds = [0, 1, 7, 42, 123, -5, 2**32 + 7, 2**64 + 3, 12345678901234567890]
    draws = {}
    for s in mt_seeds:
        random.seed(s)
        draws[f"s{len(draws)}"] = np.array([random.random() for _ in range(1500)], dtype=np.float64)
    np.savez(OUT / "mt_draws.npz", seeds=np.array([str(s) for s in mt_seeds]), **draws)

    # ---- replay traces
    rand_actions = np.random.default_rng(123).integers(0, 2, size=99).astype(np.int32)
    traces = {}
    returns = {}
    index_error = {}
    for seed in SEEDS:
        for pol in POLICIES:
            env = Env()
            obs, info0 = env.reset(seed=seed)
            assert info0 == {}
            obs_l = [np.asarray(obs, dtype=np.float32)]
            rew, done_l, step_l, cloud_l, act_l = [], [], [], [], []
            t = 0
            done = False
            while not done:
                a = _policy(pol, env, obs, t, rand_actions)
                obs, r, done, trunc, info = env.step(a)
                assert trunc is False and isinstance(r, float) and isinstance(done, bool)
                obs_l.append(np.asarray(obs, dtype=np.float32))
                rew.append(r)
                done_l.append(done)
                step_l.append(info["step"])
                cloud_l.append(0 if info["chosen_cloud"] == "aws" else 1)
                act_l.append(int(a))
                t += 1
            # stepping past the terminal step raises IndexError (iloc[100]) after incrementing
            try:
                env.step(0)
                raised = False
            except IndexError:
                raised = True
            index_error[f"{seed}_{pol}"] = {"raised": raised, "current_step_after": env.current_step}
            key = f"s{seed}_{pol}"
            traces[key + "_obs"] = np.stack(obs_l)
            traces[key + "_reward"] = np.array(rew, dtype=np.float64)
            traces[key + "_done"] = np.array(done_l, dtype=np.uint8)
            traces[key + "_step"] = np.array(step_l, dtype=np.int32)
            traces[key + "_cloud"] = np.array(cloud_l, dtype=np.int32)
            traces[key + "_action"] = np.array(act_l, dtype=np.int32)
            returns.setdefault(pol, float(np.sum(np.array(rew, dtype=np.float64))))
            # python-order float sum (matches `total_reward += reward`)
            acc = 0.0
            for r in rew:
                acc += r
            returns[pol] = acc

    # unseeded reset continues the global MT stream: reset(seed=42), one rr episode,
    # then reset() with no seed and a second rr episode.
    env = Env()
    obs, _ = env.reset(seed=42)
    cont = [np.asarray(obs, np.float32)]
    for ep in range(2):
        if ep == 1:
            obs, _ = env.reset()
            cont.append(np.asarray(obs, np.float32))
        done = False
        while not done:
            a = 0 if env.current_step % 2 == 0 else 1
            obs, r, done, _, _ = env.step(a)
            cont.append(np.asarray(obs, np.float32))
    traces["cont_s42_rr_obs"] = np.stack(cont)
    traces["rand_actions"] = rand_actions
    np.savez(OUT / "traces.npz", **traces)

    per_step_max = float(np.maximum(
        100 * (0.6 * table[:99, 1] + 0.4 * table[:99, 3]),
        100 * (0.6 * table[:99, 2] + 0.4 * table[:99, 4])).sum())
    meta = {
        "columns": cols,
        "seeds": SEEDS,
        "policies": POLICIES,
        "returns": returns,
        "index_error": index_error,
        "max_steps": 99,
        "per_step_max_return": per_step_max,
        "generated_by": "tools/make_goldens.py (reference env stub-imported in the build container)",
    }
    (OUT / "traces_meta.json").write_text(json.dumps(meta, indent=1, sort_keys=True))

    # ---- action validity (gymnasium Discrete(2).contains via the env's assert)
    cases = {
        "int0": 0, "int1": 1, "int2": 2, "int_neg1": -1, "bool_true": True, "bool_false": False,
        "np_int64_1": np.int64(1), "np_int32_0": np.int32(0), "np_uint8_1": np.uint8(1),
        "np_0d_int_1": np.array(1), "np_0d_int_2": np.array(2), "np_1d_int": np.array([1]),
        "float_1": 1.0, "np_float32_0": np.float32(0), "str_1": "1", "none": None,
        "np_int64_big": np.int64(2**40),
    }
    validity = {}
    for name, a in cases.items():
        env = Env()
        env.reset(seed=0)
        try:
            env.step(a)
            validity[name] = True
        except AssertionError as e:
            validity[name] = False
            assert str(e).startswith("Invalid action")
    (OUT / "action_validity.json").write_text(json.dumps(validity, indent=1, sort_keys=True))

    # ---- GAE goldens (RLlib compute_advantages restated: discount_cumsum via lfilter)
    from scipy.signal import lfilter

    rng = np.random.default_rng(7)
    gae = {}
    for ci, (T, N, gamma, lam) in enumerate([(128, 16, 0.99, 1.0), (64, 8, 0.995, 0.95), (17, 5, 0.9, 0.0)]):
        r = rng.standard_normal((T, N)).astype(np.float32)
        v = rng.standard_normal((T + 1, N)).astype(np.float32)
        d = (rng.random((T, N)) < 0.05).astype(np.uint8)
        adv = np.zeros((T, N), np.float64)
        for n in range(N):
            # split each env column into fragments at terminal steps
            start = 0
            for t in range(T):
                if d[t, n] or t == T - 1:
                    end = t + 1
                    last_r = 0.0 if d[t, n] else float(v[T, n])
                    vp = np.concatenate([v[start:end, n].astype(np.float64), [last_r]])
                    delta = r[start:end, n].astype(np.float64) + gamma * vp[1:] - vp[:-1]
                    adv[start:end, n] = lfilter([1], [1, -gamma * lam], delta[::-1], axis=0)[::-1]
                    start = end
        gae[f"c{ci}_r"] = r
        gae[f"c{ci}_v"] = v
        gae[f"c{ci}_d"] = d
        gae[f"c{ci}_adv"] = adv
        gae[f"c{ci}_vt"] = adv + v[:T].astype(np.float64)
        gae[f"c{ci}_params"] = np.array([gamma, lam], np.float64)
    np.savez(OUT / "gae.npz", **gae)
    global_stream_golden(Env)
    print("wrote", sorted(p.name for p in OUT.iterdir()))
    print("returns", returns)


if __name__ == "__main__":
    main()
