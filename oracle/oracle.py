"""CPU oracle for the rlks hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker (or the timed CPU baseline).  The product path never calls it.

Contents and what pins each piece:
  OracleEnv / philox / mt_random   C restatement in oracle/rlks_oracle.c of the reference env
        (k8s_multi_cloud_env.py:84-144), pinned by tests/golden/ (traces generated from the
        reference env itself by tools/make_goldens.py; see tests/test_oracle_golden.py).
  gae                              RLlib compute_advantages (use_gae=True) as a reverse
        recurrence, pinned by tests/golden/gae.npz (scipy.signal.lfilter discount_cumsum form).
  ppo_loss_grad / adam             restatement of RLlib's PPO torch loss (ppo_torch_policy.loss)
        and torch.optim.Adam in float64 autograd.  RLlib is third-party and not installed, and
        the reference repo holds no PPO vectors: PARITY UNPINNED against RLlib.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "librlks_oracle.so"
_lib = None


class EnvCfg(C.Structure):  # mirror of rlks_env_cfg (include/rlks_types.h)
    _fields_ = [
        ("n_envs", C.c_int32), ("n_rows", C.c_int32), ("n_clouds", C.c_int32), ("max_steps", C.c_int32),
        ("noise_mode", C.c_int32), ("autoreset", C.c_int32), ("env_offset", C.c_int32), ("reserved0", C.c_int32),
        ("seed", C.c_uint64), ("cpu_lo", C.c_double), ("cpu_hi", C.c_double), ("w_cost", C.c_double),
        ("w_lat", C.c_double), ("scale", C.c_double),
        ("nodes_per_cluster", C.c_int32), ("pod_cpu_m", C.c_int32), ("pod_mem_mi", C.c_int32),
        ("arrival_mode", C.c_int32), ("arrival_rate", C.c_double), ("depart_prob", C.c_double),
        ("init_occupancy", C.c_double), ("reject_penalty", C.c_double),
    ]


def build() -> Path:
    if not LIB.exists():
        subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        h = C.CDLL(str(build()))
        u32p, dp = C.POINTER(C.c_uint32), C.POINTER(C.c_double)
        h.ro_philox4x32_10.argtypes = [u32p, u32p, u32p]
        h.ro_u53.argtypes = [C.c_uint32, C.c_uint32]
        h.ro_u53.restype = C.c_double
        h.ro_mt_seed.argtypes = [u32p, u32p, C.c_int]
        h.ro_mt_random.argtypes = [u32p]
        h.ro_mt_random.restype = C.c_double
        h.ro_env_create.argtypes = [C.POINTER(EnvCfg), dp, dp]
        h.ro_env_create.restype = C.c_void_p
        h.ro_env_destroy.argtypes = [C.c_void_p]
        h.ro_env_seed_lane.argtypes = [C.c_void_p, C.c_int, u32p, C.c_int]
        h.ro_env_reset.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        h.ro_env_step.argtypes = [C.c_void_p] + [C.c_void_p] * 7
        h.ro_env_enable_nodes.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        h.ro_env_node_state.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        h.ro_env_counters.argtypes = [C.c_void_p, C.c_void_p]
        h.ro_binom_cdf32.argtypes = [C.c_int, C.c_double, C.c_void_p]
        h.ro_env_lane_step.argtypes = [C.c_void_p, C.c_int]
        h.ro_env_lane_episode.argtypes = [C.c_void_p, C.c_int]
        _lib = h
    return _lib


def _u32(a):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return a, a.ctypes.data_as(C.POINTER(C.c_uint32))


def philox(ctr, key):
    """Philox4x32-10 of ctr [4] under key [2] -> uint32 [4]"""
    c, cp = _u32(ctr)
    k, kp = _u32(key)
    o, op = _u32(np.zeros(4))
    lib().ro_philox4x32_10(cp, kp, op)
    return o.copy()


def seed_words(seed: int):
    n = abs(int(seed))
    w = []
    while n:
        w.append(n & 0xFFFFFFFF)
        n >>= 32
    return w or [0]


def mt_random(seed: int, n: int) -> np.ndarray:
    """n values of CPython random.random() after random.seed(seed), via the C restatement"""
    st, sp = _u32(np.zeros(625))
    k, kp = _u32(seed_words(seed))
    lib().ro_mt_seed(sp, kp, len(k))
    return np.array([lib().ro_mt_random(sp) for _ in range(n)], dtype=np.float64)


def make_cfg(n_envs, n_rows, n_clouds, *, noise_mode=1, seed=0, autoreset=0, env_offset=0, max_steps=None,
             nodes=0, pod_cpu_m=100, pod_mem_mi=64, arrival_mode=0, arrival_rate=1.0, depart_prob=0.02,
             init_occupancy=0.5, reject_penalty=0.0):
    cfg = EnvCfg()
    cfg.n_envs, cfg.n_rows, cfg.n_clouds = n_envs, n_rows, n_clouds
    cfg.max_steps = n_rows - 1 if max_steps is None else max_steps
    cfg.noise_mode, cfg.autoreset, cfg.env_offset, cfg.seed = noise_mode, autoreset, env_offset, seed
    cfg.cpu_lo, cfg.cpu_hi, cfg.w_cost, cfg.w_lat, cfg.scale = 0.1, 0.8, 0.6, 0.4, 100.0
    cfg.nodes_per_cluster, cfg.pod_cpu_m, cfg.pod_mem_mi = nodes, pod_cpu_m, pod_mem_mi
    cfg.arrival_mode, cfg.arrival_rate, cfg.depart_prob = arrival_mode, arrival_rate, depart_prob
    cfg.init_occupancy, cfg.reject_penalty = init_occupancy, reject_penalty
    return cfg


class OracleEnv:
    """Batched CPU env with the same semantics as librlks' env kernel."""

    def __init__(self, cfg: EnvCfg, cost: np.ndarray, lat: np.ndarray, cap_cpu=None, cap_mem=None, trace=None):
        self.cfg = cfg
        self.cost = np.ascontiguousarray(cost, dtype=np.float64)
        self.lat = np.ascontiguousarray(lat, dtype=np.float64)
        dp = C.POINTER(C.c_double)
        self.h = lib().ro_env_create(C.byref(cfg), self.cost.ctypes.data_as(dp), self.lat.ctypes.data_as(dp))
        self.n, self.D = cfg.n_envs, 3 * cfg.n_clouds
        if cfg.nodes_per_cluster > 0:
            cc = np.ascontiguousarray(cap_cpu, np.int32)
            cm = np.ascontiguousarray(cap_mem, np.int32)
            tr = np.ascontiguousarray(trace if trace is not None else [cfg.arrival_rate], np.float64)
            rc = lib().ro_env_enable_nodes(self.h, cc.ctypes.data, cm.ctypes.data, tr.ctypes.data, len(tr))
            assert rc == 0

    def node_state(self):
        C_, N = self.cfg.n_clouds, self.cfg.nodes_per_cluster
        fc = np.zeros((self.n, C_, N), np.int32)
        fm = np.zeros((self.n, C_, N), np.int32)
        used = np.zeros((self.n, C_), np.int32)
        lib().ro_env_node_state(self.h, fc.ctypes.data, fm.ctypes.data, used.ctypes.data)
        return fc, fm, used

    def counters(self):
        """[node checks, pods placed, pods rejected, pods departed, nodes written]"""
        c = np.zeros(5, np.int64)
        lib().ro_env_counters(self.h, c.ctypes.data)
        return c

    def seed(self, lane, seed):
        k, kp = _u32(seed_words(seed))
        lib().ro_env_seed_lane(self.h, lane, kp, len(k))

    def reset(self, mask=None):
        obs = np.zeros((self.n, self.D), np.float32)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        lib().ro_env_reset(self.h, None if m is None else m.ctypes.data, obs.ctypes.data)
        return obs

    def step(self, actions, obs=None):
        a = np.ascontiguousarray(actions, np.int32)
        obs = np.zeros((self.n, self.D), np.float32) if obs is None else obs
        rew = np.zeros(self.n, np.float64)
        term = np.zeros(self.n, np.uint8)
        step = np.zeros(self.n, np.int32)
        final = np.zeros((self.n, self.D), np.float32)
        status = np.zeros(2, np.int32)
        lib().ro_env_step(self.h, a.ctypes.data, obs.ctypes.data, rew.ctypes.data, term.ctypes.data,
                          step.ctypes.data, final.ctypes.data, status.ctypes.data)
        return obs, rew, term, step, final, status

    def lane_step(self, i):
        return lib().ro_env_lane_step(self.h, i)

    def __del__(self):
        try:
            lib().ro_env_destroy(self.h)
        except Exception:
            pass


# ----------------------------------------------------------------------------- GAE
def gae(r, v, d, gamma, lam):
    """RLlib compute_advantages over a time-major [T][N] rollout with auto-reset lanes.
    v is [T+1][N] (row T = bootstrap).  float64."""
    r = np.asarray(r, np.float64)
    v = np.asarray(v, np.float64)
    nd = 1.0 - np.asarray(d, np.float64)
    T = r.shape[0]
    adv = np.zeros_like(r)
    a = np.zeros(r.shape[1])
    for t in range(T - 1, -1, -1):
        delta = r[t] + gamma * v[t + 1] * nd[t] - v[t]
        a = delta + gamma * lam * nd[t] * a
        adv[t] = a
    return adv, adv + v[:T]


# ----------------------------------------------------------------------------- PPO loss (torch fp64)
def _net(torch, flat, off, D, H, A, net):
    base = 6 * net
    An = A if net == 0 else 1
    shapes = [(H, D), (H,), (H, H), (H,), (An, H), (An,)]
    ts = []
    for j, shp in enumerate(shapes):
        n = int(np.prod(shp))
        o = off[base + j]
        ts.append(flat[o: o + n].view(shp))
    return ts


def mlp_forward(flat, off, D, H, A, obs):
    """RLlib FCNet forward (tanh, separate value net) in float64: (logits, value)"""
    import torch

    x = torch.as_tensor(np.asarray(obs, np.float64))
    f = torch.as_tensor(np.asarray(flat, np.float64))
    out = []
    for net in (0, 1):
        w1, b1, w2, b2, w3, b3 = _net(torch, f, off, D, H, A, net)
        h1 = torch.tanh(x @ w1.T + b1)
        h2 = torch.tanh(h1 @ w2.T + b2)
        out.append(h2 @ w3.T + b3)
    return out[0].numpy(), out[1][:, 0].numpy()


def ppo_loss_grad(flat, off, D, H, A, mb, *, clip_param=0.3, vf_clip_param=10.0, vf_loss_coeff=1.0,
                  entropy_coeff=0.0, kl_coeff=0.2, adv_mean=0.0, adv_inv_std=1.0, count=None):
    """Gradient of RLlib's PPO torch loss w.r.t. the flat parameters, float64 autograd.

    mb: packed minibatch records [rows][stride] = [obs D | logits_old A | adv | vtarg | logp_old | action]
    Returns (grad (same length as flat), stats dict of per-row sums).
    """
    import torch

    rec = torch.as_tensor(np.asarray(mb, np.float64))
    rows = rec.shape[0]
    count = rows if count is None else count
    f = torch.tensor(np.asarray(flat, np.float64), requires_grad=True)
    x = rec[:, :D]
    lo = rec[:, D: D + A]
    adv = (rec[:, D + A] - adv_mean) * adv_inv_std
    vt = rec[:, D + A + 1]
    logp_old = rec[:, D + A + 2]
    act = rec[:, D + A + 3].long()
    outs = []
    for net in (0, 1):
        w1, b1, w2, b2, w3, b3 = _net(torch, f, off, D, H, A, net)
        h1 = torch.tanh(x @ w1.T + b1)
        h2 = torch.tanh(h1 @ w2.T + b2)
        outs.append(h2 @ w3.T + b3)
    logits, value = outs[0], outs[1][:, 0]
    logp_all = torch.log_softmax(logits, dim=1)
    logp = logp_all.gather(1, act[:, None])[:, 0]
    ratio = torch.exp(logp - logp_old)
    surr = torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip_param, 1 + clip_param))
    lpo = torch.log_softmax(lo, dim=1)
    kl = (lpo.exp() * (lpo - logp_all)).sum(1)
    ent = -(logp_all.exp() * logp_all).sum(1)
    vf = torch.clamp((value - vt) ** 2, 0, vf_clip_param)
    total = (-surr + vf_loss_coeff * vf - entropy_coeff * ent).sum() / count + kl_coeff * kl.sum() / count
    total.backward()
    stats = {"policy_loss": float((-surr).sum()), "vf_loss": float(vf.sum()), "kl": float(kl.sum()),
             "entropy": float(ent.sum()), "rows": rows}
    return f.grad.numpy(), stats


def adam(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch.optim.Adam single-tensor step (float32 semantics), returns new (p, m, v)"""
    import torch

    pt = torch.tensor(np.asarray(p, np.float32))
    mt = torch.tensor(np.asarray(m, np.float32))
    vt = torch.tensor(np.asarray(v, np.float32))
    gt = torch.tensor(np.asarray(g, np.float32))
    mt.lerp_(gt, 1 - beta1)
    vt.mul_(beta2).addcmul_(gt, gt, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (vt.sqrt() / (bc2 ** 0.5)).add_(eps)
    pt.addcdiv_(mt, denom, value=-(lr / bc1))
    return pt.numpy(), mt.numpy(), vt.numpy()


def binom_cdf32(maxp, p):
    """[maxp+1][maxp+1] Binomial(n, p) CDF table in units of 2^-32 (departure draws)"""
    out = np.zeros((maxp + 1, maxp + 1), np.uint32)
    lib().ro_binom_cdf32(int(maxp), float(p), out.ctypes.data)
    return out
