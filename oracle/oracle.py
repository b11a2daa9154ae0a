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
        ("noise_mode", C.c_int32), ("autoreset", C.c_int32), ("env_offset", C.c_int32), ("skip_returns", C.c_int32),
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
        h.ro_skip32.argtypes = [C.c_int, C.c_double, C.c_void_p]
        h.ro_skip32.restype = C.c_int
        h.ro_env_lane_step.argtypes = [C.c_void_p, C.c_int]
        h.ro_env_lane_episode.argtypes = [C.c_void_p, C.c_int]
        h.ro_env_lane_counters.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        h.ro_philox_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
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


def philox_batch(ctr, key):
    """Philox4x32-10 of counters ctr [n][4] under key [2] -> uint32 [n][4]"""
    c = np.ascontiguousarray(ctr, np.uint32).reshape(-1, 4)
    k = np.ascontiguousarray(key, np.uint32)
    out = np.zeros_like(c)
    lib().ro_philox_batch(c.ctypes.data, k.ctypes.data, out.ctypes.data, c.shape[0])
    return out


def u53(a, b):
    """vectorised ro_u53 (exact in float64)"""
    return ((a >> 5).astype(np.float64) * 67108864.0 + (b >> 6).astype(np.float64)) * (1.0 / 9007199254740992.0)


PURPOSE_ACTION = 2  # include/rlks_types.h RLKS_PURPOSE_ACTION


def sample_actions(logits, gids, episodes, steps, seed):
    """TorchCategorical draws as the rollout kernels make them (rollout_sf16.hip k_sf_roll,
    env.hip k_sample_step): u = f32(u53(Philox(ctr = {global lane, episode, step, ACTION << 16},
    key = seed)) words 0, 1) * sum_a exp(l_a - max), action = first a with u < cumsum(exp(l - max))
    (all float32, sums in index order).  logits [n][A] float32.
    Returns (actions int32 [n], margin [n]: |u - nearest cumulative boundary| in units of
    float32 ulp(boundary) — draws within a couple of ulp may differ by exp() rounding)."""
    lg = np.asarray(logits, np.float32)
    n, A = lg.shape
    mx = lg.max(1, keepdims=True)
    ex = np.exp(lg - mx).astype(np.float32)
    se = np.zeros(n, np.float32)
    for a in range(A):
        se = (se + ex[:, a]).astype(np.float32)
    ctr = np.zeros((n, 4), np.uint32)
    ctr[:, 0] = np.asarray(gids, np.uint32)
    ctr[:, 1] = np.asarray(episodes, np.uint32)
    ctr[:, 2] = np.asarray(steps, np.uint32)
    ctr[:, 3] = PURPOSE_ACTION << 16
    x = philox_batch(ctr, [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF])
    u = (u53(x[:, 0], x[:, 1]).astype(np.float32) * se).astype(np.float32)
    act = np.full(n, A - 1, np.int32)
    found = np.zeros(n, bool)
    c = np.zeros(n, np.float32)
    margin = np.full(n, np.inf)
    for a in range(A):
        c = (c + ex[:, a]).astype(np.float32)
        hit = (~found) & (u < c)
        act[hit] = a
        found |= hit
        if a < A - 1:
            margin = np.minimum(margin, np.abs(u.astype(np.float64) - c) / np.spacing(np.maximum(c, 1e-30)))
    return act, margin


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
        """[node checks, pods placed, pods rejected, pods departed, node write-backs, node reads]"""
        c = np.zeros(6, np.int64)
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

    def lane_episode(self, i):
        return lib().ro_env_lane_episode(self.h, i)

    def lane_counters(self):
        """(step [n], episode [n]) int32 of every lane"""
        st = np.zeros(self.n, np.int32)
        ep = np.zeros(self.n, np.int32)
        lib().ro_env_lane_counters(self.h, st.ctypes.data, ep.ctypes.data)
        return st, ep

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


def mlp_forward(flat, off, D, H, A, obs, dtype=np.float64):
    """RLlib FCNet forward (tanh, separate value net) in float64: (logits, value)
    (dtype=np.float32: torch fp32 on the CPU, the precision baseline of the per-element tests)"""
    import torch

    x = torch.as_tensor(np.asarray(obs, dtype))
    f = torch.as_tensor(np.asarray(flat, dtype))
    out = []
    for net in (0, 1):
        w1, b1, w2, b2, w3, b3 = _net(torch, f, off, D, H, A, net)
        h1 = torch.tanh(x @ w1.T + b1)
        h2 = torch.tanh(h1 @ w2.T + b2)
        out.append(h2 @ w3.T + b3)
    return out[0].numpy(), out[1][:, 0].numpy()


def ppo_loss_grad(flat, off, D, H, A, mb, *, clip_param=0.3, vf_clip_param=10.0, vf_loss_coeff=1.0,
                  entropy_coeff=0.0, kl_coeff=0.2, adv_mean=0.0, adv_inv_std=1.0, count=None, dtype=np.float64,
                  scale=False):
    """Gradient of RLlib's PPO torch loss w.r.t. the flat parameters, float64 autograd
    (dtype=np.float32: the same in torch fp32 on the CPU, the precision baseline of the tests).

    mb: packed minibatch records [rows][stride] = [obs D | logits_old A | adv | vtarg | logp_old | action]
    Returns (grad (same length as flat), stats dict of per-row sums); scale=True adds stats["scale"]:
    per parameter, the sum over rows of the absolute per-row terms of its gradient (|dZ|^T |input|
    for a weight, sum |dZ| for a bias): the magnitude a summation error is proportional to, i.e.
    each element's own cancellation scale (test infrastructure: tests/parity.py).
    """
    import torch

    rec = torch.as_tensor(np.asarray(mb, dtype))
    rows = rec.shape[0]
    count = rows if count is None else count
    f = torch.tensor(np.asarray(flat, dtype), requires_grad=True)
    x = rec[:, :D]
    lo = rec[:, D: D + A]
    adv = (rec[:, D + A] - adv_mean) * adv_inv_std
    vt = rec[:, D + A + 1]
    logp_old = rec[:, D + A + 2]
    act = rec[:, D + A + 3].long()
    outs, acts = [], []
    for net in (0, 1):
        w1, b1, w2, b2, w3, b3 = _net(torch, f, off, D, H, A, net)
        z1 = x @ w1.T + b1
        h1 = torch.tanh(z1)
        z2 = h1 @ w2.T + b2
        h2 = torch.tanh(z2)
        out = h2 @ w3.T + b3
        for z in (z1, z2, out):
            z.retain_grad()
        outs.append(out)
        acts.append((z1, h1, z2, h2, out))
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
    stats = {"policy_loss": float((-surr).sum().detach()), "vf_loss": float(vf.sum().detach()),
             "kl": float(kl.sum().detach()), "entropy": float(ent.sum().detach()), "rows": rows}
    if scale:
        sc = np.zeros(len(flat))
        for net, (z1, h1, z2, h2, out) in enumerate(acts):
            terms = []
            for dz, inp in ((z1.grad, x), (z2.grad, h1), (out.grad, h2)):
                adz = dz.abs().double()
                terms += [adz.T @ inp.detach().abs().double(), adz.sum(0)]
            for j, t in enumerate(terms):
                o = off[6 * net + j]
                v = t.numpy().ravel()
                sc[o:o + v.size] = v
        stats["scale"] = sc
    return f.grad.numpy(), stats


# ----------------------------------------------------------------------------- fp32 error band
# A float32 evaluation's error at one element is one draw of its rounding: at an element where a sum
# cancels, a single evaluation can be exact by luck.  The tests compare against the largest error of a
# few EQUALLY VALID fp32 evaluations of the same function: the hidden units of each layer relabelled
# (the same network; every dot product summed in another order) and the minibatch rows reversed (the
# loss is a mean over rows), each result mapped back to the original labels.  Evaluation 0 is the plain
# one.  Test infrastructure (tests/parity.py).
def _hidden_perms(H, n):
    rng = np.random.default_rng(20251)
    return [(np.arange(H), np.arange(H))] + [(rng.permutation(H), rng.permutation(H)) for _ in range(n - 1)]


def _relabel(flat, off, D, H, A, p1, p2, inverse=False):
    """flat parameters (or a gradient of them) with hidden units p1 (layer 1) / p2 (layer 2) of both
    nets relabelled: new unit i = old unit p[i]; inverse=True maps back"""
    out = np.array(flat, copy=True)
    for net in (0, 1):
        An = A if net == 0 else 1
        shapes = [(H, D), (H,), (H, H), (H,), (An, H), (An,)]
        t = [np.asarray(flat[off[6 * net + j]: off[6 * net + j] + int(np.prod(shp))]).reshape(shp)
             for j, shp in enumerate(shapes)]
        if not inverse:
            new = [t[0][p1], t[1][p1], t[2][np.ix_(p2, p1)], t[3][p2], t[4][:, p2], t[5]]
        else:
            new = [np.empty_like(x) for x in t]
            new[0][p1] = t[0]
            new[1][p1] = t[1]
            new[2][np.ix_(p2, p1)] = t[2]
            new[3][p2] = t[3]
            new[4][:, p2] = t[4]
            new[5] = t[5]
        for j, x in enumerate(new):
            out[off[6 * net + j]: off[6 * net + j] + x.size] = x.ravel()
    return out


def ppo_loss_grad_fp32_band(flat, off, D, H, A, mb, n=3, **kw):
    """n float32 gradients of the same loss (see above): [plain, relabelled, relabelled + rows reversed]"""
    out = []
    for i, (p1, p2) in enumerate(_hidden_perms(H, n)):
        f = _relabel(np.asarray(flat, np.float64), off, D, H, A, p1, p2)
        rows = np.asarray(mb)[::-1] if i == 2 else mb
        g, _ = ppo_loss_grad(f.astype(np.float32), off, D, H, A, np.ascontiguousarray(rows), dtype=np.float32, **kw)
        out.append(_relabel(np.asarray(g, np.float64), off, D, H, A, p1, p2, inverse=True))
    return out


def mlp_forward_fp32_band(flat, off, D, H, A, obs, n=3):
    """n float32 forwards of the same network, hidden units relabelled (see above):
    ([logits, ...], [values, ...])"""
    ls, vs = [], []
    for p1, p2 in _hidden_perms(H, n):
        f = _relabel(np.asarray(flat, np.float64), off, D, H, A, p1, p2).astype(np.float32)
        lg, v = mlp_forward(f, off, D, H, A, obs, dtype=np.float32)
        ls.append(lg)
        vs.append(v)
    return ls, vs


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


def adam64(p, g, m, v, step, lr, beta1=0.9, beta2=0.999, eps=1e-8):
    """the same Adam step in float64 (numpy), the whole-iteration reference"""
    m = m + (1 - beta1) * (g - m)
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    return p - (lr / bc1) * (m / (np.sqrt(v) / np.sqrt(bc2) + eps)), m, v


# ----------------------------------------------------------------------------- minibatch order
_M32 = np.uint64(0xFFFFFFFF)


def _mix32(x):
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & _M32
    x ^= x >> np.uint64(16)
    return x


def perm_keys(seed: int, epoch: int, S: int):
    """(half, mask, round keys) of the per-epoch Feistel bijection (csrc/ppo.hip make_perm)"""
    bits = 2
    while (1 << bits) < S:
        bits += 1
    bits += bits & 1
    half = bits // 2
    m64 = (1 << 64) - 1
    z = (seed ^ ((0x9E3779B97F4A7C15 * (epoch + 1)) & m64)) & m64
    keys = []
    for _ in range(4):  # splitmix64
        z = (z + 0x9E3779B97F4A7C15) & m64
        x = z
        x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m64
        x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m64
        keys.append((x ^ (x >> 31)) & 0xFFFFFFFF)
    return half, (1 << half) - 1, keys


def epoch_permutation(seed: int, epoch: int, S: int) -> np.ndarray:
    """sample index (t * N + n) of every minibatch row position of epoch `epoch`: a balanced
    4-round Feistel network on [0, 2^(2 half)) cycle-walked into [0, S) — restates
    csrc/ppo.hip perm_apply / k_gather (rows b*mb .. (b+1)*mb of the result form minibatch b)"""
    half, mask, keys = perm_keys(seed, epoch, S)
    x = np.arange(S, dtype=np.uint64)
    out = np.empty(S, np.uint64)
    todo = np.arange(S)
    cur = x.copy()
    sh, mk = np.uint64(half), np.uint64(mask)
    while todo.size:
        L, R = cur >> sh, cur & mk
        for r in range(4):
            nl = R
            R = (L ^ _mix32(R ^ np.uint64(keys[r]))) & mk
            L = nl
        cur = (L << sh) | R
        done = cur < np.uint64(S)
        out[todo[done]] = cur[done]
        todo, cur = todo[~done], cur[~done]
    return out.astype(np.int64)


GROUP_KEY = 0x632BE59BD9B4E019  # csrc/ppo.hip rlks_ppo_gather_grouped: per-group seed offset


def minibatch_indices(seed: int, epoch: int, T: int, N: int, mb: int, groups: int = 1, group0: int = 0):
    """[n_mb][mb] sample indices (t * N + n) of epoch `epoch`'s minibatches as
    rlks_ppo_gather_grouped lays them out: lane block k (global id group0 + k) has its own Feistel
    permutation of its T * (N / groups) samples and fills rows [k mb/g, (k+1) mb/g) of every
    minibatch."""
    Ng, mbg = N // groups, mb // groups
    Sg = T * Ng
    n_mb = Sg // mbg
    out = np.empty((n_mb, mb), np.int64)
    for k in range(groups):
        s = (seed + GROUP_KEY * (group0 + k)) & ((1 << 64) - 1)
        p = epoch_permutation(s, epoch, Sg)[: n_mb * mbg].reshape(n_mb, mbg)
        out[:, k * mbg:(k + 1) * mbg] = (p // Ng) * N + k * Ng + (p % Ng)
    return out


def ppo_iteration(flat, off, D, H, A, buf, *, perm_seed, epochs, mb, lr, gamma=0.99, lam=1.0, kl_coeff=0.2,
                  kl_target=0.01, adam_m=None, adam_v=None, adam_step=0, clip_param=0.3, vf_clip_param=10.0,
                  vf_loss_coeff=1.0, entropy_coeff=0.0, groups=1):
    """One PPO learner update in float64 over a recorded rollout (RLlib old-stack semantics as in
    rlks.ppo: GAE, standardisation, `epochs` x (samples // mb) minibatches in the per-epoch Feistel
    order, loss gradient by autograd, Adam, mean-KL coefficient update).  `buf` holds the rollout
    arrays obs [T+1][N][D], logits [T][N][A], values [T+1][N], actions, logp, rewards, dones [T][N].
    Returns (params, adam_m, adam_v, new kl_coeff, per-step stats)."""
    T, N = buf["rewards"].shape
    S = T * N
    adv, vt = gae(buf["rewards"], buf["values"], buf["dones"], gamma, lam)
    a = adv.reshape(-1)
    mean, inv_std = a.mean(), 1.0 / max(1e-4, a.std())
    rec = np.concatenate([buf["obs"][:T].reshape(S, D), buf["logits"].reshape(S, A), a[:, None],
                          vt.reshape(S, 1), buf["logp"].reshape(S, 1), buf["actions"].reshape(S, 1)], axis=1)
    p = np.asarray(flat, np.float64).copy()
    m = np.zeros_like(p) if adam_m is None else np.asarray(adam_m, np.float64).copy()
    v = np.zeros_like(p) if adam_v is None else np.asarray(adam_v, np.float64).copy()
    step = adam_step
    stats = []
    for ep in range(epochs):
        order = minibatch_indices(perm_seed, ep, T, N, mb, groups)
        for b in range(order.shape[0]):
            rows = rec[order[b]]
            g, st = ppo_loss_grad(p, off, D, H, A, rows, clip_param=clip_param, vf_clip_param=vf_clip_param,
                                  vf_loss_coeff=vf_loss_coeff, entropy_coeff=entropy_coeff, kl_coeff=kl_coeff,
                                  adv_mean=mean, adv_inv_std=inv_std)
            step += 1
            p, m, v = adam64(p, g, m, v, step, lr)
            stats.append(st)
    kl = np.mean([s["kl"] / s["rows"] for s in stats])
    if kl > 2.0 * kl_target:
        kl_coeff *= 1.5
    elif kl < 0.5 * kl_target:
        kl_coeff *= 0.5
    return p, m, v, kl_coeff, stats


def skip32(pmax, p):
    """departure-skip survival table round((1 - p)^j 2^32), j < min(pmax, last nonzero) + 1
    """
    n = lib().ro_skip32(int(pmax), float(p), None)
    out = np.zeros(max(n, 1), np.uint32)
    lib().ro_skip32(int(pmax), float(p), out.ctypes.data)
    return out[:n]
