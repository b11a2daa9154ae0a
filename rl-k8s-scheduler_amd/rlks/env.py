"""Drop-in environments backed by the HIP env kernel (librlks.so).

`K8sMultiCloudEnv` keeps the reference's surface (k8s_multi_cloud_env.py:36-157):
    K8sMultiCloudEnv(env_config=None, fast_mode=True)
    reset(seed=None, options=None) -> (np.float32[6], {})
    step(action) -> (np.float32[6], float reward, bool done, False, {"chosen_cloud", "step"})
    attributes action_space, observation_space, max_steps, current_step, static_df;
    normal_scheduler_step(obs); render(); close()
    errors: AssertionError("Invalid action ...") (:116), IndexError past the table (:91 via :144),
            FileNotFoundError for a missing table (:56-64)
and runs on one GPU lane.  Its utilisation noise is CPython's MT19937 (noise="mt19937"), so with a
seeded reset the observations are bit-identical to the reference.  The reference draws that noise
from the process-global `random` stream (:87) and reseeds it in reset (:109-111):
  noise_stream="global" (or env_config={"noise_stream": "global"}) reproduces exactly that: the
    lane's MT19937 state is loaded from random.getstate() before every reset / step and written
    back with random.setstate() after it, so all envs of the process and the caller's own random
    draws share one stream in call order (tests/golden/global_stream.npz);
  noise_stream="instance" (the default) gives each env a private generator: no host round trip of
    the 2.5 KB state per step; an env never seeded takes its seed from `random`.  Both reseed
    `random` and `np.random` in reset(seed) as the reference does.

`VecK8sMultiCloudEnv` is the batched form over device tensors (one lane per env, auto-reset,
Philox noise by default) used by the rollout engine.
"""
from __future__ import annotations

import json
import random
from pathlib import Path

import numpy as np

from . import _lib
from .spaces import Box, Discrete
from .tables import load_table

try:  # subclass gymnasium.Env when it is installed (RLlib registers gymnasium envs)
    import gymnasium as _gym

    _EnvBase = _gym.Env
except Exception:  # pragma: no cover - gymnasium absent in this image
    _EnvBase = object

CLOUD_NAMES = ("aws", "azure")


def _torch():
    import torch

    return torch


def _device(device):
    torch = _torch()
    if not torch.cuda.is_available():
        raise _lib.RlksError("librlks needs a HIP device (MI355X); none is visible")
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device(device)


def seed_key_words(seed: int) -> list:
    """32-bit little-endian words of abs(seed), as CPython random_seed() builds init_by_array's key"""
    n = abs(int(seed))
    words = []
    while n:
        words.append(n & 0xFFFFFFFF)
        n >>= 32
    return words or [0]


def make_cfg(n_envs, table, *, noise="philox", seed=0, autoreset=True, env_offset=0, max_steps=None,
             nodes=None, track_returns=True):
    """rlks_env_cfg for `n_envs` lanes over `table`; `nodes` (a NodeSpec) enables the node-level
    extension; track_returns=False drops the per-lane episode-return bookkeeping
    (episode_stats / episode_log stay empty) and leaves the plain gymnasium step"""
    cfg = _lib.EnvCfg()
    cfg.n_envs = int(n_envs)
    cfg.n_rows = table.n_rows
    cfg.n_clouds = table.n_clouds
    cfg.max_steps = int(max_steps if max_steps is not None else table.n_rows - 1)  # :66
    cfg.noise_mode = _lib.RLKS_NOISE_MT19937 if noise == "mt19937" else _lib.RLKS_NOISE_PHILOX
    cfg.autoreset = int(bool(autoreset))
    cfg.env_offset = int(env_offset)
    cfg.skip_returns = 0 if track_returns else 1
    cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    cfg.cpu_lo, cfg.cpu_hi = 0.1, 0.8          # random.uniform(0.1, 0.8) (:87)
    cfg.w_cost, cfg.w_lat, cfg.scale = 0.6, 0.4, 100.0  # 100 * (0.6*cost + 0.4*latency) (:122)
    if nodes is not None:
        cfg.nodes_per_cluster = nodes.nodes_per_cluster
        cfg.pod_cpu_m, cfg.pod_mem_mi = nodes.pod_cpu_m, nodes.pod_mem_mi
        cfg.arrival_mode = 1 if nodes.arrival_trace is not None else 0
        cfg.arrival_rate, cfg.depart_prob = nodes.arrival_rate, nodes.depart_prob
        cfg.init_occupancy, cfg.reject_penalty = nodes.init_occupancy, nodes.reject_penalty
    return cfg


class NodeSpec:
    """Node-level cluster model (builder-defined, the reference has no node state).

    Defaults follow the reference manifests: pod request 100m / 64Mi (simple-service.yaml:25-28);
    node types t3.micro-like (2 vCPU / 1 GiB) and Standard_B2s-like (2 vCPU / 4 GiB)
    (aws-/azure-cluster-config.yaml:12) alternating over the clusters.  Each step every running pod
    leaves with probability `depart_prob` (geometric lifetimes), then
    Poisson(`arrival_rate`) pods (or `arrival_trace[t]`) arrive at the chosen cluster.
    depart_prob="stationary" balances the two at the initial mean occupancy
    (arrival_rate / expected initial pods per env), so a cluster neither drains nor fills.
    """

    def __init__(self, n_clouds, nodes_per_cluster=256, *, node_cpu_m=None, node_mem_mi=None, pod_cpu_m=100,
                 pod_mem_mi=64, arrival_rate=1.0, arrival_trace=None, depart_prob="stationary", init_occupancy=0.5,
                 reject_penalty=0.0):
        self.n_clouds = int(n_clouds)
        self.nodes_per_cluster = int(nodes_per_cluster)
        self.node_cpu_m = np.ascontiguousarray(node_cpu_m if node_cpu_m is not None else [2000] * self.n_clouds,
                                               np.int32)
        self.node_mem_mi = np.ascontiguousarray(
            node_mem_mi if node_mem_mi is not None else [1024 if c % 2 == 0 else 4096 for c in range(self.n_clouds)],
            np.int32)
        self.pod_cpu_m, self.pod_mem_mi = int(pod_cpu_m), int(pod_mem_mi)
        self.arrival_rate = float(arrival_rate)
        self.arrival_trace = None if arrival_trace is None else np.ascontiguousarray(arrival_trace, np.float64)
        self.init_occupancy = float(init_occupancy)
        self.reject_penalty = float(reject_penalty)
        self.depart_prob = self.stationary_depart_prob() if depart_prob == "stationary" else float(depart_prob)

    def to_dict(self) -> dict:
        """JSON-able fields (checkpoints): from_dict(to_dict()) rebuilds the same spec"""
        return {"n_clouds": self.n_clouds, "nodes_per_cluster": self.nodes_per_cluster,
                "node_cpu_m": self.node_cpu_m.tolist(), "node_mem_mi": self.node_mem_mi.tolist(),
                "pod_cpu_m": self.pod_cpu_m, "pod_mem_mi": self.pod_mem_mi, "arrival_rate": self.arrival_rate,
                "arrival_trace": None if self.arrival_trace is None else self.arrival_trace.tolist(),
                "depart_prob": self.depart_prob, "init_occupancy": self.init_occupancy,
                "reject_penalty": self.reject_penalty}

    @classmethod
    def from_dict(cls, d: dict) -> "NodeSpec":
        return cls(**d)

    def max_pods(self):
        """pods a node of each cluster can hold"""
        return np.minimum(self.node_cpu_m // self.pod_cpu_m, self.node_mem_mi // self.pod_mem_mi)

    def expected_initial_pods(self):
        """mean pods per env after a reset: node pods ~ U{0..floor(init_occupancy * max_pods)}"""
        mp = self.max_pods()
        init_max = np.minimum(mp, np.floor(self.init_occupancy * mp))
        return float(self.nodes_per_cluster * (init_max / 2.0).sum())

    def stationary_depart_prob(self):
        rate = float(np.mean(self.arrival_trace)) if self.arrival_trace is not None else self.arrival_rate
        pods = self.expected_initial_pods()
        return min(1.0, rate / pods) if pods > 0 else 0.0


MMPP_PATH = Path(__file__).resolve().parent / "data" / "locust_mmpp.json"


def locust_mmpp() -> dict:
    """The Markov-modulated Poisson arrival model fitted to the reference's Locust runs
    (data/local_{aws,azure}_load_stats_history.csv) by tools/fit_locust_mmpp.py: modulating state
    = Locust user count, ML transition matrix, per-state request rate (req/s), plateau dispersion."""
    return json.loads(MMPP_PATH.read_text())


def bursty_trace(n=100, base=1.0, cloud="pooled", model=None):
    """Per-step Poisson rates of BASELINE configs[4]'s Locust-style arrivals (arrival_mode 1):
    lambda[t] = base * E[rate(state_t)] / rate(plateau), state_t the fitted MMPP's user-count state
    t steps (Locust seconds) after a reset, plateau = the chain's absorbing top state.  The fit is
    the observed 5 users/s spawn ramp 0 -> 20 then 20 users (per-state 0, 5, 7, 9, 9.9 req/s
    pooled), a deterministic chain, so the expectation is the chain's single realisation; the
    plateau's dispersion index 0.47-0.51 leaves no hidden burst state to fit (fit_locust_mmpp.py)."""
    m = model if model is not None else locust_mmpp()
    states = [int(s) for s in m["states"]]
    P = np.asarray(m["transitions"], np.float64)
    r = np.array([m["rate"][cloud][str(s)] for s in states], np.float64)
    pi = np.zeros(len(states))
    pi[states.index(int(m["initial_state"]))] = 1.0
    lam = np.empty(n, np.float64)
    for t in range(n):
        lam[t] = pi @ r
        pi = pi @ P
    top = r[int(np.argmax(states))]
    return base * lam / top


class DeviceEnv:
    """Owner of one rlks_env handle (HBM lane state + staged tables)."""

    def __init__(self, cfg: _lib.EnvCfg, table, device=None, nodes: NodeSpec | None = None):
        import ctypes as C

        self.torch = _torch()
        self.device = _device(device)
        self.cfg = cfg
        self.table = table
        self.nodes = nodes
        with self.torch.cuda.device(self.device):
            h = C.c_void_p()
            if nodes is None:
                _lib.call("rlks_env_create", C.byref(cfg), table.cost.ctypes.data, table.latency.ctypes.data,
                          C.byref(h))
            else:
                tr = nodes.arrival_trace
                _lib.call("rlks_env_create_ext", C.byref(cfg), table.cost.ctypes.data, table.latency.ctypes.data,
                          nodes.node_cpu_m.ctypes.data, nodes.node_mem_mi.ctypes.data,
                          None if tr is None else tr.ctypes.data, 0 if tr is None else len(tr), C.byref(h))
        self.handle = h
        self.n = cfg.n_envs
        self.obs_dim = 3 * cfg.n_clouds

    @property
    def stream(self):
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def state_bytes(self) -> int:
        import ctypes as C

        n = C.c_int64()
        _lib.call("rlks_env_state_bytes", self.handle, C.byref(n))
        return int(n.value)

    def save_state(self):
        """device uint8 snapshot of every per-lane state (rlks_env_save_state)"""
        buf = self.torch.empty(self.state_bytes(), dtype=self.torch.uint8, device=self.device)
        _lib.call("rlks_env_save_state", self.handle, _lib.ptr(buf), self.stream)
        return buf

    def load_state(self, buf):
        buf = self.torch.as_tensor(buf).to(device=self.device, dtype=self.torch.uint8).contiguous()
        if buf.numel() != self.state_bytes():
            raise ValueError(f"env state snapshot has {buf.numel()} bytes, this env needs {self.state_bytes()}")
        _lib.call("rlks_env_load_state", self.handle, _lib.ptr(buf), self.stream)

    def node_state(self):
        """(free_cpu [N, C, nodes], free_mem [N, C, nodes], used_cpu [N, C]) int32 device tensors of a
        node-level env (rlks_env_node_state)"""
        torch = self.torch
        if self.nodes is None:
            raise ValueError("node_state: this env has no node-level state")
        n, C_, k = self.n, self.cfg.n_clouds, self.nodes.nodes_per_cluster
        fc = torch.empty(n, C_, k, dtype=torch.int32, device=self.device)
        fm = torch.empty(n, C_, k, dtype=torch.int32, device=self.device)
        used = torch.empty(n, C_, dtype=torch.int32, device=self.device)
        _lib.call("rlks_env_node_state", self.handle, _lib.ptr(fc), _lib.ptr(fm), _lib.ptr(used), self.stream)
        return fc, fm, used

    def episode_log(self, clear=True):
        """(returns f64 [k], keys i64 [k], total count) of the episodes completed since the last
        clear, k = min(total, RLKS_EPLOG_CAP), in completion order (sorted by episode, lane)"""
        torch = self.torch
        ret = torch.zeros(_lib.RLKS_EPLOG_CAP, dtype=torch.float64, device=self.device)
        key = torch.zeros(_lib.RLKS_EPLOG_CAP, dtype=torch.int64, device=self.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=self.device)
        _lib.call("rlks_env_episode_log", self.handle, _lib.ptr(ret), _lib.ptr(key), _lib.ptr(cnt), int(clear),
                  self.stream)
        n = int(cnt.item()) & 0xFFFFFFFF
        k = min(n, _lib.RLKS_EPLOG_CAP)
        r, kk = ret[:k].cpu().numpy(), key[:k].cpu().numpy()
        order = np.argsort(kk, kind="stable")
        return r[order], kk[order], n

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            _lib.lib().rlks_env_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class K8sMultiCloudEnv(_EnvBase):
    """Single-env drop-in for rl_scheduler.env.k8s_multi_cloud_env.K8sMultiCloudEnv."""

    metadata = {"render_modes": []}

    def __init__(self, env_config=None, fast_mode=True, *, data_path=None, device=None, noise="mt19937",
                 noise_stream=None):
        # env_config is accepted as in the reference (:46), which ignores it; here it may carry
        # "noise_stream" (module docstring)
        if noise_stream is None:
            noise_stream = (env_config or {}).get("noise_stream", "instance") if isinstance(env_config, dict) else "instance"
        if noise_stream not in ("instance", "global"):
            raise ValueError(f"noise_stream must be 'instance' or 'global', got {noise_stream!r}")
        if noise_stream == "global" and noise != "mt19937":
            raise ValueError("noise_stream='global' needs the MT19937 noise mode")
        self.noise_stream = noise_stream
        self.fast_mode = fast_mode  # slow mode's kubernetes dry-run is out of scope
        self.action_space = Discrete(2)  # 0 = AWS, 1 = Azure (:51)
        self.observation_space = Box(low=0.0, high=1.0, shape=(6,), dtype=np.float32)  # (:52)
        self._table = load_table(data_path)
        self.static_df = self._table.dataframe()
        self.max_steps = self._table.n_rows - 1  # (:66)
        self.current_step = 0
        torch = _torch()
        # the global stream must not be advanced here (the reference constructor draws nothing); its
        # state is loaded into the lane before every reset / step
        seed0 = random.getrandbits(64) if noise_stream == "instance" else 0
        self._dev = DeviceEnv(make_cfg(1, self._table, noise=noise, seed=seed0, autoreset=False), self._table, device)
        d = self._dev.device
        self._act = torch.zeros(1, dtype=torch.int32, device=d)
        self._obs = torch.zeros(1, 6, dtype=torch.float32, device=d)
        self._rew = torch.zeros(1, dtype=torch.float64, device=d)
        self._term = torch.zeros(1, dtype=torch.uint8, device=d)
        self._step = torch.zeros(1, dtype=torch.int32, device=d)
        self._status = torch.zeros(2, dtype=torch.int32, device=d)
        self._keys = torch.zeros(1, 8, dtype=torch.int32, device=d)
        self._keylen = torch.zeros(1, dtype=torch.int32, device=d)
        self._mtw = torch.zeros(625, dtype=torch.int32, device=d)  # global stream: the lane's MT19937 state
        self._seeded = False

    # ------------------------------------------------------------------ gymnasium surface
    def reset(self, seed=None, options=None):
        if seed is not None:
            random.seed(seed)       # process-global side effects of the reference (:109-111)
            np.random.seed(seed)
        if self.noise_stream == "global":
            self._push_global()
        elif seed is not None:
            self._seed_lane(seed)
        elif not self._seeded:
            self._seed_lane(random.getrandbits(64))
        s = self._dev.stream
        _lib.call("rlks_env_reset", self._dev.handle, None, _lib.ptr(self._obs), s)
        if self.noise_stream == "global":
            self._pull_global()
        self.current_step = 0
        obs = self._obs.cpu().numpy()[0].copy()
        return obs, {}

    def _push_global(self):
        """the process-global `random` state -> this env's lane (CPython getstate layout: 624 words
        and the position, rlks_env_mt_words)"""
        import torch

        words = np.array(random.getstate()[1], dtype=np.uint32)
        self._mtw.copy_(torch.from_numpy(words.view(np.int32)))
        _lib.call("rlks_env_mt_words", self._dev.handle, 0, _lib.ptr(self._mtw), 1, self._dev.stream)

    def _pull_global(self):
        """the lane's state after its draws -> the process-global `random` (gauss_next kept)"""
        _lib.call("rlks_env_mt_words", self._dev.handle, 0, _lib.ptr(self._mtw), 0, self._dev.stream)
        words = self._mtw.cpu().numpy().view(np.uint32)
        version, _, gauss = random.getstate()
        random.setstate((version, tuple(int(x) for x in words), gauss))

    def _seed_lane(self, seed):
        import torch

        words = seed_key_words(seed)
        if len(words) > self._keys.shape[1]:
            self._keys = torch.zeros(1, len(words), dtype=torch.int32, device=self._dev.device)
        key = np.zeros(self._keys.shape[1], dtype=np.uint32)
        key[: len(words)] = words
        self._keys.copy_(torch.from_numpy(key.view(np.int32))[None])
        self._keylen.fill_(len(words))
        _lib.call("rlks_env_seed", self._dev.handle, None, _lib.ptr(self._keys), _lib.ptr(self._keylen),
                  self._keys.shape[1], self._dev.stream)
        self._seeded = True

    def step(self, action):
        assert self.action_space.contains(action), f"Invalid action {action}"
        a = int(action)
        self._act.fill_(a)
        if self.noise_stream == "global":
            self._push_global()
        _lib.call("rlks_env_step", self._dev.handle, _lib.ptr(self._act), _lib.ptr(self._obs), _lib.ptr(self._rew),
                  None, _lib.ptr(self._term), None, _lib.ptr(self._step), None, _lib.ptr(self._status),
                  self._dev.stream)
        if self.noise_stream == "global":
            self._pull_global()
        status = self._status.cpu().numpy()
        self.current_step = int(self._step.item())
        if status[1]:
            raise IndexError("single positional indexer is out-of-bounds")
        reward = float(self._rew.item())
        done = bool(self._term.item())
        obs = self._obs.cpu().numpy()[0].copy()
        info = {"chosen_cloud": "aws" if a == 0 else "azure", "step": self.current_step}
        return obs, reward, done, False, info

    def render(self):
        pass

    def close(self):
        pass

    def normal_scheduler_step(self, obs):
        """cost-only greedy baseline (:156-157)"""
        return 0 if obs[0] <= obs[1] else 1


class VecK8sMultiCloudEnv:
    """Batched env over device tensors: one lane per env, all lanes stepped by one kernel launch.

    reset(seed=None) -> obs [N, 3C] float32 (device)
    step(actions int32 [N]) -> (obs, reward f64 [N], terminated u8 [N], truncated u8 [N], info)
    info = {"step": int32 [N], "final_observation": [N, 3C] (rows valid where terminated)}
    With autoreset (default) a terminated lane returns the first observation of its next episode.
    """

    def __init__(self, num_envs, *, table=None, seed=0, noise="philox", autoreset=True, env_offset=0,
                 device=None, data_path=None, nodes: NodeSpec | None = None, track_returns=True):
        torch = _torch()
        self.table = table if table is not None else load_table(data_path)
        self.nodes = nodes
        self.num_envs = int(num_envs)
        self.n_clouds = self.table.n_clouds
        self.obs_dim = 3 * self.n_clouds
        self.action_space = Discrete(self.n_clouds)
        self.observation_space = Box(0.0, 1.0, (self.obs_dim,), np.float32)
        self.max_steps = self.table.n_rows - 1
        self.cfg = make_cfg(num_envs, self.table, noise=noise, seed=seed, autoreset=autoreset, env_offset=env_offset,
                            nodes=nodes, track_returns=track_returns)
        self.dev = DeviceEnv(self.cfg, self.table, device, nodes)
        d = self.dev.device
        self.device = d
        N = self.num_envs
        self._status = torch.zeros(2, dtype=torch.int32, device=d)
        self.obs = torch.zeros(N, self.obs_dim, dtype=torch.float32, device=d)
        self.reward = torch.zeros(N, dtype=torch.float64, device=d)
        self.terminated = torch.zeros(N, dtype=torch.uint8, device=d)
        self.truncated = torch.zeros(N, dtype=torch.uint8, device=d)  # TimeLimit(100) never fires: stays 0
        self.steps = torch.zeros(N, dtype=torch.int32, device=d)
        self.final_obs = torch.zeros(N, self.obs_dim, dtype=torch.float32, device=d)
        self._stats = torch.zeros(2, dtype=torch.float64, device=d)

    @property
    def handle(self):
        return self.dev.handle

    def seed(self, seeds, mask=None):
        """per-lane random.seed(seeds[i]) (MT19937 noise mode only)"""
        torch = _torch()
        words = [seed_key_words(s) for s in seeds]
        width = max(len(w) for w in words)
        key = np.zeros((self.num_envs, width), np.uint32)
        for i, w in enumerate(words):
            key[i, : len(w)] = w
        keys = torch.from_numpy(key.view(np.int32)).to(self.device)
        klen = torch.tensor([len(w) for w in words], dtype=torch.int32, device=self.device)
        m = None if mask is None else torch.as_tensor(mask, dtype=torch.uint8, device=self.device)
        _lib.call("rlks_env_seed", self.handle, _lib.ptr(m), _lib.ptr(keys), _lib.ptr(klen), width, self.dev.stream)

    def reset(self, seed=None, mask=None):
        torch = _torch()
        if seed is not None and self.cfg.noise_mode == _lib.RLKS_NOISE_MT19937:
            self.seed([int(seed) + i for i in range(self.num_envs)])
        m = None if mask is None else torch.as_tensor(mask, dtype=torch.uint8, device=self.device)
        _lib.call("rlks_env_reset", self.handle, _lib.ptr(m), _lib.ptr(self.obs), self.dev.stream)
        return self.obs

    def step(self, actions):
        torch = _torch()
        a = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
        _lib.call("rlks_env_step", self.handle, _lib.ptr(a), _lib.ptr(self.obs), _lib.ptr(self.reward), None,
                  _lib.ptr(self.terminated), None, _lib.ptr(self.steps),
                  _lib.ptr(self.final_obs), _lib.ptr(self._status), self.dev.stream)
        return self.obs, self.reward, self.terminated, self.truncated, {"step": self.steps,
                                                                         "final_observation": self.final_obs,
                                                                         "status": self._status}

    def check_status(self):
        """raise the reference's exceptions for the last step (synchronises)"""
        st = self._status.cpu().numpy()
        if st[0]:
            raise AssertionError(f"Invalid action in {int(st[0])} lane(s)")
        if st[1]:
            raise IndexError("single positional indexer is out-of-bounds")

    def episode_stats(self, clear=True):
        """(sum of completed-episode returns, count) since the last clear"""
        _lib.call("rlks_env_episode_stats", self.handle, _lib.ptr(self._stats), int(clear), self.dev.stream)
        return self._stats

    def lane_state(self):
        torch = _torch()
        st = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
        ep = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
        _lib.call("rlks_env_lane_state", self.handle, _lib.ptr(st), _lib.ptr(ep), self.dev.stream)
        return st, ep

    def node_state(self):
        """(free_cpu [N, C, nodes], free_mem [N, C, nodes], used_cpu [N, C]) int32 device tensors"""
        return self.dev.node_state()

    def counters(self, enable=-1):
        """[node checks, pods placed, pods rejected, pods departed, node write-backs, node reads] since
        counting was enabled (enable=1 resets)"""
        torch = _torch()
        out = torch.zeros(6, dtype=torch.int64, device=self.device)
        _lib.call("rlks_env_counters", self.handle, int(enable), _lib.ptr(out), self.dev.stream)
        return out

    def close(self):
        self.dev.close()
