"""PPO agent with RLlib's surface, running the whole hot path on the GPU.

Reference call sites:
  PPOConfig().environment(K8sMultiCloudEnv).framework("torch").rollouts(num_rollout_workers=1)
      .training(train_batch_size=4000, sgd_minibatch_size=256, num_sgd_iter=10, lr=3e-4, gamma=0.99)
                                                                         (train_ppo.py:9-21)
  agent = PPO(config=config); result = agent.train(); result["episode_reward_mean"];
  agent.save()                                                           (train_ppo.py:23-31)
  PPO.from_checkpoint(path); compute_single_action(obs[, explore=False]) (eval_ppo.py:17-27,
                                                                          final_evaluation.py:32-48)
RLlib itself is absent in this image, so the semantics restated here (GAE, advantage
standardisation, clipped surrogate + KL + clipped value loss, Adam, KL adaptation) are pinned by
the torch-CPU oracle under oracle/, not by RLlib: parity unpinned.

One PPO iteration on one GPU (all launches on torch's current stream, no host sync inside):
  rollout   rlks_rollout: T x (policy forward -> sample -> env step), bootstrap V(s_T)
  advantages rlks_gae -> rlks_adv_stats -> [all-reduce] -> rlks_adv_finalize
  update    num_sgd_iter x minibatches x (rlks_ppo_gather -> rlks_ppo_grad -> [all-reduce] ->
            rlks_adam_step); then rlks_kl_update from the mean KL over all SGD steps.  Single rank:
            rlks_ppo_sgd_step_next per minibatch (gradient + Adam, and the next minibatch's gather
            inside the same reduce launch); ranks: rlks_ppo_grad_step_next -> all-reduce ->
            rlks_ppo_adam_apply
Multi-GPU (torch.distributed, backend "nccl" = RCCL): each rank owns a contiguous block of lanes
(env_offset = rank * lanes), the flat gradient and the few scalar sums are all-reduced.
"""
from __future__ import annotations

import collections
import copy
import ctypes as C
import json
import math
import time
from pathlib import Path

import numpy as np

from . import _lib
from . import distributed as ddp
from .env import DeviceEnv, make_cfg
from .policy import PolicyParams
from .tables import load_table


class PPOConfig:
    """RLlib-style builder.  Defaults are RLlib's old-API-stack PPOConfig defaults."""

    def __init__(self):
        self.env = None
        self.env_config = {}
        self.framework_str = "torch"
        self.num_rollout_workers = 0
        self.num_envs_per_worker = 1
        self.rollout_fragment_length = "auto"
        self.train_batch_size = 4000
        self.sgd_minibatch_size = 128
        self.num_sgd_iter = 30
        self.lr = 5e-5
        self.gamma = 0.99
        self.lambda_ = 1.0
        self.clip_param = 0.3
        self.vf_clip_param = 10.0
        self.vf_loss_coeff = 1.0
        self.entropy_coeff = 0.0
        self.kl_coeff = 0.2
        self.kl_target = 0.01
        self.grad_clip = None
        self.model = {"fcnet_hiddens": [256, 256], "fcnet_activation": "tanh", "vf_share_layers": False}
        self.num_gpus = 0
        self.seed = None
        self.explore = True
        self.evaluation_interval = None
        self.evaluation_duration = 10
        self.metrics_num_episodes_for_smoothing = 100
        # rlks.metrics.JsonLinesReporter: append every train() result to this file as one JSON line
        # (also: $RLKS_METRICS_JSONL)
        self.metrics_json_lines = None
        # save() with no directory: this run's logdir under rlks.checkpoints.results_root()
        # (~/ray_results/PPO_<env>_<time>, RLlib's Algorithm.logdir)
        self.logdir = None
        # save() includes the lanes' env state: None = yes for table envs (~30 B per lane), no for
        # node-level envs (C x nodes x 8 B per lane: ~1 GB at c3, written on every save())
        self.checkpoint_env_state = None
        # minibatches are drawn per block of lanes (rlks_ppo_gather_grouped): None = one block per
        # rank.  A single-rank run with num_lane_groups = W trains exactly like W ranks (the rollout
        # picks its forward kernel from the job's lane count, rlks_rollout_bufs.global_lanes).
        self.num_lane_groups = None
        # more than one rank, split-fp16 step: True = all-reduce the W2 / W3 gradient bucket while the
        # dW1 kernel runs (rlks_ppo_grad_step_part), False = the whole gradient after it in one bucket.
        # Measured with a one-rank RCCL group at c4 (profiles/r06_rccl): one bucket costs 14 µs a step
        # over the one-rank step, two buckets 57 µs (a second all-reduce, a second reduce launch, and
        # RCCL's kernel on the CUs beside F1b) -- more than an 8-GPU all-reduce of 544 KB is expected
        # to expose, so one bucket is the default
        self.overlap_allreduce = False
        # rlks-specific knobs
        self.num_envs = None          # lanes per GPU (default: workers x envs per worker)
        self.noise = "philox"         # env utilisation noise: "philox" or "mt19937"
        self.data_path = None
        self.table = None
        self.nodes = None             # rlks.env.NodeSpec: node-level envs (configs c3 / c5)
        self.adam_betas = (0.9, 0.999)
        self.adam_eps = 1e-8
        # SGD-step matrix arithmetic (include/rlks_types.h RLKS_PRECISION_*): "sf16" = split-fp16
        # MFMA (fp32-accurate, 16x the fp32 matrix rate; minibatch rows per rank % 256 == 0),
        # "fp32" = fp32 MFMA; "auto" = sf16 where the minibatch allows it.  Policies the fused
        # kernels do not cover (hidden != 256, obs > 31, actions not 2 / 4 / 8) always run the
        # generic-width split-fp16 path ("wide").  "f16": the split-fp16 kernels with one product
        # (fp16 operands, fp32 accumulation) -- a throughput mode below the reference's fp32, never
        # chosen by "auto"
        self.sgd_precision = "auto"

    # ---- builder methods (names as in RLlib)
    def environment(self, env=None, env_config=None, **kw):
        if env is not None:
            self.env = env
        if env_config is not None:
            self.env_config = dict(env_config)
        return self

    def framework(self, framework="torch", **kw):
        if framework not in ("torch",):
            raise ValueError(f"only the torch framework is supported, got {framework!r}")
        self.framework_str = framework
        return self

    def rollouts(self, num_rollout_workers=None, num_envs_per_worker=None, rollout_fragment_length=None, **kw):
        if num_rollout_workers is not None:
            self.num_rollout_workers = int(num_rollout_workers)
        if num_envs_per_worker is not None:
            self.num_envs_per_worker = int(num_envs_per_worker)
        if rollout_fragment_length is not None:
            self.rollout_fragment_length = rollout_fragment_length
        for k, v in kw.items():
            setattr(self, k, v)
        return self

    env_runners = rollouts

    def training(self, **kw):
        alias = {"lambda": "lambda_"}
        for k, v in kw.items():
            k = alias.get(k, k)
            if k == "model":
                self.model = {**self.model, **v}
            else:
                setattr(self, k, v)
        return self

    def resources(self, num_gpus=None, **kw):
        if num_gpus is not None:
            self.num_gpus = num_gpus
        return self

    def evaluation(self, evaluation_interval=None, evaluation_duration=None, **kw):
        if evaluation_interval is not None:
            self.evaluation_interval = evaluation_interval
        if evaluation_duration is not None:
            self.evaluation_duration = evaluation_duration
        return self

    def reporting(self, metrics_num_episodes_for_smoothing=None, json_lines=None, **kw):
        if json_lines is not None:
            self.metrics_json_lines = str(json_lines)
        if metrics_num_episodes_for_smoothing is not None:
            w = int(metrics_num_episodes_for_smoothing)
            # the window is filled from the device episode log, which keeps RLKS_EPLOG_CAP episodes
            # per rank and iteration (rlks_env_episode_log)
            if not 1 <= w <= _lib.RLKS_EPLOG_CAP:
                raise ValueError(f"metrics_num_episodes_for_smoothing must be in [1, {_lib.RLKS_EPLOG_CAP}], got {w}")
            self.metrics_num_episodes_for_smoothing = w
        return self

    def debugging(self, seed=None, **kw):
        if seed is not None:
            self.seed = int(seed)
        return self

    def exploration(self, explore=None, **kw):
        if explore is not None:
            self.explore = bool(explore)
        return self

    def to_dict(self):
        """JSON-able config; the table is saved beside it by PPO.save (table.npz), the node spec
        is inlined"""
        d = {k: v for k, v in self.__dict__.items() if k not in ("env", "table", "nodes")}
        d["env"] = getattr(self.env, "__name__", str(self.env)) if self.env is not None else None
        d["lambda"] = d.pop("lambda_")
        d["nodes"] = self.nodes.to_dict() if self.nodes is not None else None
        return d

    @classmethod
    def from_dict(cls, d):
        from .env import NodeSpec

        c = cls()
        for k, v in d.items():
            if k == "lambda":
                c.lambda_ = v
            elif k == "adam_betas":
                c.adam_betas = tuple(v)
            elif k == "nodes":
                c.nodes = NodeSpec.from_dict(v) if v is not None else None
            elif k != "env" and hasattr(c, k):
                setattr(c, k, v)
        return c

    def copy(self):
        return copy.deepcopy(self)

    def build(self, **kw):
        return PPO(config=self, **kw)

    # ---- derived sizes
    def lanes(self) -> int:
        if self.num_envs:
            return int(self.num_envs)
        return max(1, self.num_rollout_workers) * max(1, self.num_envs_per_worker)

    def hidden(self) -> int:
        h = list(self.model.get("fcnet_hiddens", [256, 256]))
        if len(h) != 2 or h[0] != h[1]:
            raise ValueError(f"fcnet_hiddens must be two equal layers, got {h}")
        if self.model.get("vf_share_layers", False):
            raise ValueError("vf_share_layers=True is not supported (RLlib's PPO default is False)")
        if self.model.get("fcnet_activation", "tanh") != "tanh":
            raise ValueError("only fcnet_activation='tanh' (RLlib's default) is supported")
        return int(h[0])


class PPO:
    """One instance per GPU (rank).  train() runs one PPO iteration over all local lanes."""

    def __init__(self, config: PPOConfig | None = None, env=None, device=None, **kw):
        import torch

        self.config = cfg = (config or PPOConfig()).copy()
        if env is not None:
            cfg.env = env
        self.torch = torch
        self.rank, self.world = ddp.rank_world()
        self.multi = self.world > 1 or ddp.forced()  # the multi-rank SGD step (ddp.forced: one rank, RCCL)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        table = cfg.table if cfg.table is not None else load_table(cfg.data_path)
        self.table = table
        C_ = table.n_clouds
        if cfg.nodes is not None and cfg.nodes.n_clouds != C_:
            raise ValueError(f"NodeSpec has {cfg.nodes.n_clouds} clusters, the table {C_}")
        self.D, self.A, self.H = 3 * C_, C_, cfg.hidden()
        self.N = cfg.lanes()
        self.T = max(1, math.ceil(cfg.train_batch_size / (self.N * self.world)))
        if cfg.rollout_fragment_length not in (None, "auto"):
            self.T = int(cfg.rollout_fragment_length)
        self.samples = self.T * self.N
        if int(cfg.sgd_minibatch_size) % self.world:
            raise ValueError(f"sgd_minibatch_size {cfg.sgd_minibatch_size} is not divisible by the {self.world} ranks")
        self.mb = int(cfg.sgd_minibatch_size) // self.world  # per-rank rows of a global minibatch
        if self.mb <= 0 or self.mb % 128:
            raise ValueError(f"sgd_minibatch_size per rank must be a positive multiple of 128, got {self.mb}")
        # RLlib's torch learner (multi_gpu_train_one_step): num_batches = samples // minibatch per
        # epoch; the train batch's remainder rows (4000 mod 256 = 160 at train_ppo.py:15-16) are
        # not visited in that epoch.  Here every epoch draws a fresh permutation of all samples, so
        # each epoch leaves out a different random remainder.
        self.n_mb = self.samples // self.mb
        if self.n_mb == 0:
            raise ValueError("train batch is smaller than one minibatch")
        groups = int(cfg.num_lane_groups or self.world)
        if (groups % self.world or self.N % (groups // self.world) or self.mb % (groups // self.world)
                or groups // self.world > 64):
            # 64 = the gather's lane-group limit (ppo.hip MAX_GROUPS); shares above 8 (NEXT_GROUPS)
            # gather in a launch of their own instead of inside the gradient reduce
            raise ValueError(f"num_lane_groups {groups} must be a multiple of the {self.world} ranks and its per-rank "
                             f"share (at most 64) must divide the {self.N} lanes and the {self.mb}-row minibatch")
        self.groups = groups // self.world
        self.group0 = self.rank * self.groups
        seed = cfg.seed if cfg.seed is not None else 0
        self.seed = seed
        with torch.cuda.device(self.device):
            self.env = DeviceEnv(make_cfg(self.N, table, noise=cfg.noise, seed=seed, autoreset=True,
                                          env_offset=ddp.lane_range(self.N, self.rank)[0], nodes=cfg.nodes),
                                 table, self.device, cfg.nodes)
            self.params = PolicyParams(self.D, self.H, self.A, device=self.device, seed=seed)
            prec = cfg.sgd_precision
            if self.params.wide():
                prec = "wide"
            elif prec == "auto":
                prec = "sf16" if self.mb % 256 == 0 else "fp32"
            if prec not in ("sf16", "f16", "fp32", "wide") or (prec in ("sf16", "f16") and self.mb % 256):
                raise ValueError(f"sgd_precision {cfg.sgd_precision!r} with {self.mb} minibatch rows per rank")
            self.precision = prec
            self.params.desc.precision = {"sf16": _lib.RLKS_PRECISION_SF16, "fp32": _lib.RLKS_PRECISION_FP32,
                                          "wide": _lib.RLKS_PRECISION_WIDE, "f16": _lib.RLKS_PRECISION_F16}[prec]
            P = self.params.padded
            f32 = dict(dtype=torch.float32, device=self.device)
            self.adam_m = torch.zeros(P, **f32)
            self.adam_v = torch.zeros(P, **f32)
            self.grad = torch.zeros(P, **f32)
            self.adam_step = 0
            self.dyn = torch.zeros(_lib.RLKS_DYN_SIZE, **f32)
            self.dyn[_lib.RLKS_DYN_KL_COEFF] = float(cfg.kl_coeff)
            self.dyn[_lib.RLKS_DYN_INV_COUNT] = ddp.loss_scale(self.mb, self.world)
            T, N, D, A = self.T, self.N, self.D, self.A
            self.buf = {
                "obs": torch.zeros(T + 1, N, D, **f32), "logits": torch.zeros(T, N, A, **f32),
                "values": torch.zeros(T + 1, N, **f32), "actions": torch.zeros(T, N, dtype=torch.int32, device=self.device),
                "logp": torch.zeros(T, N, **f32), "rewards": torch.zeros(T, N, **f32),
                "dones": torch.zeros(T, N, dtype=torch.uint8, device=self.device),
                "adv": torch.zeros(T, N, **f32), "vtarg": torch.zeros(T, N, **f32),
            }
            b = self.buf
            self.bufs = _lib.RolloutBufs(b["obs"].data_ptr(), b["logits"].data_ptr(), b["values"].data_ptr(),
                                         b["actions"].data_ptr(), b["logp"].data_ptr(), b["rewards"].data_ptr(),
                                         b["dones"].data_ptr(), b["adv"].data_ptr(), b["vtarg"].data_ptr(), T, N,
                                         N * self.world)
            self.stride = _lib.lib().rlks_minibatch_stride(C.byref(self.params.desc))
            self.mbuf = torch.zeros(self.mb, self.stride, **f32)
            # one aligned record per sample (rlks_ppo_pack after GAE): a minibatch row is then one
            # random line read instead of six (2 / 4 / 8 clouds; the wide path gathers directly)
            ps = _lib.lib().rlks_packed_stride(C.byref(self.params.desc))
            self.packed = torch.empty(T * N, ps, **f32) if ps else None
            # one workspace for the SGD step and the rollout (split weights; wide: N-row activations)
            wsb, wsr = C.c_int64(), C.c_int64()
            _lib.call("rlks_ppo_workspace_bytes", C.byref(self.params.desc), self.mb, C.byref(wsb))
            _lib.call("rlks_ppo_workspace_bytes", C.byref(self.params.desc),
                      N if prec == "wide" else self.mb, C.byref(wsr))
            self.ws = torch.empty(max(wsb.value, wsr.value), dtype=torch.uint8, device=self.device)
            self.n_partials = _lib.lib().rlks_gae_partials_count(N)
            self.gae_part = torch.zeros(self.n_partials, 2, dtype=torch.float64, device=self.device)
            self.adv_sums = torch.zeros(3, dtype=torch.float64, device=self.device)
            self.stats = torch.zeros(cfg.num_sgd_iter * self.n_mb, _lib.RLKS_STAT_SIZE, dtype=torch.float64,
                                     device=self.device)
            self.kl_sc = torch.zeros(2, dtype=torch.float64, device=self.device)
            self.ep_stats = torch.zeros(2, dtype=torch.float64, device=self.device)
            self.coeffs = _lib.PpoCoeffs(cfg.clip_param, cfg.vf_clip_param, cfg.vf_loss_coeff, cfg.entropy_coeff)
            _lib.call("rlks_env_reset", self.env.handle, None, _lib.ptr(b["obs"][0]), self.stream)
            self.env.episode_log(clear=True)
        # obs[0] holds the lanes' current observations only before the first rollout; afterwards
        # they are obs[T] of the previous rollout (moved to obs[0] when the next one starts, so the
        # update can still read obs[0..T-1])
        self._carry = False
        # the previous SGD step was a fused one on the current parameters (rlks_ppo_sgd_step)
        self._fused_prev = False
        self._ep_history = collections.deque(maxlen=max(1, int(cfg.metrics_num_episodes_for_smoothing)))
        self._ar_events = None  # profile_allreduce(): (start, compute end, done) events per SGD step
        # gradient buckets of the overlapped all-reduce (include/rlks.h rlks_ppo_grad_step_part): two
        # contiguous views of the flat gradient (storage order: both nets' W1 / b1 first), W2 / b2 /
        # W3 / b3 of both nets, then W1 / b1 of both
        off = self.params.offsets
        g = self.grad
        self._buckets = ([g[off[2]:self.params.padded]], [g[off[0]:off[2]]])
        self._overlap = bool(cfg.overlap_allreduce) and self.multi and self.precision in ("sf16", "f16")
        self.sample_calls = 0   # compute_actions / compute_single_action draws so far (Philox counter)
        self.iteration = 0
        self.timesteps_total = 0
        from .metrics import JsonLinesReporter

        self.reporter = JsonLinesReporter.from_config(cfg, self.rank)
        self.episodes_total = 0

    # ------------------------------------------------------------------ internals
    @property
    def stream(self):
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def _allreduce(self, t):
        ddp.allreduce_sum_(t)

    def rollout(self, explore=True):
        s = self.stream
        b = self.buf
        if self._carry:
            b["obs"][0].copy_(b["obs"][self.T])
        self._carry = True
        # sf16: one split-fp16 launch per step computes both nets (values included) and steps the
        # env; the split weights live in the SGD workspace
        _lib.call("rlks_rollout_ws", self.env.handle, C.byref(self.params.desc), _lib.ptr(self.params.flat),
                  C.byref(self.bufs), int(explore), _lib.ptr(self.ws), self.ws.numel(), s)

    def advantages(self):
        s = self.stream
        b = self.buf
        cfg = self.config
        _lib.call("rlks_gae", _lib.ptr(b["rewards"]), _lib.ptr(b["values"]), _lib.ptr(b["dones"]), float(cfg.gamma),
                  float(cfg.lambda_), self.T, self.N, _lib.ptr(b["adv"]), _lib.ptr(b["vtarg"]),
                  _lib.ptr(self.gae_part), s)
        _lib.call("rlks_adv_stats", _lib.ptr(self.gae_part), self.n_partials, float(self.samples),
                  _lib.ptr(self.adv_sums), s)
        self._allreduce(self.adv_sums)
        _lib.call("rlks_adv_finalize", _lib.ptr(self.adv_sums), _lib.ptr(self.dyn), s)
        if self.packed is not None:
            _lib.call("rlks_ppo_pack", C.byref(self.params.desc), C.byref(self.bufs), _lib.ptr(self.packed), s)

    def perm_seed(self, iteration=None):
        """key of this iteration's minibatch permutations (resumes with the iteration counter)"""
        it = self.iteration if iteration is None else iteration
        return (self.seed * 1000003 + it) & (2**64 - 1)

    def sgd_step(self, epoch, b, stat_row, gathered=False, next_mb=None):
        """one SGD step on minibatch b of epoch `epoch`.  gathered: the previous step's launch already
        gathered it (rlks_ppo_sgd_step_next); next_mb = (epoch, b) of the following step: gather it
        inside this step's gradient-reduce launch (packed records)"""
        s = self.stream
        desc = C.byref(self.params.desc)
        beta1, beta2 = self.config.adam_betas
        if not gathered and self.packed is not None:
            _lib.call("rlks_ppo_gather_packed", desc, _lib.ptr(self.packed), self.T, self.N, self.perm_seed(), epoch,
                      self.groups, self.group0, b * self.mb, self.mb, _lib.ptr(self.mbuf), s)
        elif not gathered:
            _lib.call("rlks_ppo_gather_grouped", desc, C.byref(self.bufs), self.perm_seed(), epoch, self.groups,
                      self.group0, b * self.mb, self.mb, _lib.ptr(self.dyn), _lib.ptr(self.mbuf), s)
        self.adam_step += 1
        nxt = None
        if next_mb is not None:
            ne, nb = next_mb
            nxt = C.byref(_lib.GatherNext(_lib.ptr(self.packed), _lib.ptr(self.mbuf), self.perm_seed(), nb * self.mb,
                                          self.T, self.N, ne, self.groups, self.group0, self.mb))
        if not self.multi:  # no all-reduce between gradient and Adam: one fused launch sequence
            _lib.call("rlks_ppo_sgd_step_next", desc, C.byref(self.coeffs), _lib.ptr(self.params.flat),
                      _lib.ptr(self.dyn), _lib.ptr(self.mbuf), self.mb, _lib.ptr(self.grad), _lib.ptr(stat_row),
                      _lib.ptr(self.adam_m), _lib.ptr(self.adam_v), self.params.padded, float(self.config.lr),
                      float(beta1), float(beta2), float(self.config.adam_eps), self.adam_step, int(self._fused_prev),
                      nxt, _lib.ptr(self.ws), self.ws.numel(), s)
            self._fused_prev = True
            return
        # ranks: gradient -> all-reduce -> Adam, the Adam pass also leaving the next split's weight
        # maxima (rlks_ppo_grad_step / rlks_ppo_adam_apply: no weight-max pass per SGD step)
        ev = self._ar_events is not None  # profile_allreduce(): events on the launch stream
        cur = self.torch.cuda.current_stream(self.device)

        def event():
            e = self.torch.cuda.Event(enable_timing=True)
            e.record(cur)
            return e

        if self._overlap:
            # part 1 (F1a, F2, the W2 / W3 reduce) -> its bucket's all-reduce on the collective's stream,
            # under part 2 (F1b, the W1 reduce, the next gather) -> the W1 bucket's; Adam after both
            args = (desc, C.byref(self.coeffs), _lib.ptr(self.params.flat), _lib.ptr(self.dyn), _lib.ptr(self.mbuf),
                    self.mb, _lib.ptr(self.grad), _lib.ptr(stat_row), self.adam_step, int(self._fused_prev))
            _lib.call("rlks_ppo_grad_step_part", *args, 1, None, _lib.ptr(self.ws), self.ws.numel(), s)
            e0 = event() if ev else None
            h = ddp.allreduce_sum_async(self._buckets[0])
            _lib.call("rlks_ppo_grad_step_part", *args, 2, nxt, _lib.ptr(self.ws), self.ws.numel(), s)
            h += ddp.allreduce_sum_async(self._buckets[1])
            e1 = event() if ev else None
            for w in h:
                w.wait()
            if ev:  # (part 1 end, part 2 end, all-reduces done): exposed = the last interval
                self._ar_events.append((e0, e1, event()))
        else:
            _lib.call("rlks_ppo_grad_step_next", desc, C.byref(self.coeffs), _lib.ptr(self.params.flat),
                      _lib.ptr(self.dyn), _lib.ptr(self.mbuf), self.mb, _lib.ptr(self.grad), _lib.ptr(stat_row),
                      self.adam_step, int(self._fused_prev), nxt, _lib.ptr(self.ws), self.ws.numel(), s)
            e0 = event() if ev else None
            self._allreduce(self.grad)
            if ev:
                e1 = event()
                self._ar_events.append((e0, e0, e1))
        _lib.call("rlks_ppo_adam_apply", desc, _lib.ptr(self.params.flat), _lib.ptr(self.grad), _lib.ptr(self.adam_m),
                  _lib.ptr(self.adam_v), self.params.padded, float(self.config.lr), float(beta1), float(beta2),
                  float(self.config.adam_eps), self.adam_step, _lib.ptr(self.ws), self.ws.numel(), self.mb, s)
        self._fused_prev = True

    def update(self):
        cfg = self.config
        steps = [(epoch, b) for epoch in range(cfg.num_sgd_iter) for b in range(self.n_mb)]
        # packed records: each step's gradient-reduce launch also gathers the next minibatch
        chain = self.packed is not None
        for k, (epoch, b) in enumerate(steps):
            nxt = steps[k + 1] if chain and k + 1 < len(steps) else None
            self.sgd_step(epoch, b, self.stats[k], gathered=chain and k > 0, next_mb=nxt)
        self._allreduce(self.stats)
        st = self.stats
        # RLlib: learner stats are means over all SGD steps; kl per step = sum KL / rows
        self.kl_sc[0] = (st[:, _lib.RLKS_STAT_KL] / st[:, _lib.RLKS_STAT_ROWS]).sum()
        self.kl_sc[1] = float(st.shape[0])
        _lib.call("rlks_kl_update", _lib.ptr(self.dyn), _lib.ptr(self.kl_sc), float(cfg.kl_target), self.stream)

    def train_step_no_sync(self):
        """one PPO iteration, enqueued only (bench path)"""
        self.rollout(explore=self.config.explore)
        self.advantages()
        self.update()
        _lib.call("rlks_env_episode_stats", self.env.handle, _lib.ptr(self.ep_stats), 1, self.stream)
        self.iteration += 1
        self.timesteps_total += self.samples * self.world

    def profile_allreduce(self):
        """one PPO iteration with HIP events on the launch stream around every per-SGD-step gradient
        all-reduce (multi-rank only): where the data-parallel time goes.  Returns None
        on one rank, else the all-reduce's exposed time per SGD step (compute launches done -> all
        buckets reduced, what the step's Adam waits for; with overlap_allreduce the first bucket has
        run under the dW1 kernel), its mean / max, total and share of the iteration, and the span
        from the first bucket's start; the maximum over ranks of each."""
        if not self.multi:
            return None
        torch = self.torch
        st = torch.cuda.current_stream(self.device)
        self._ar_events = []
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(st)
        self.train_step_no_sync()
        t1.record(st)
        t1.synchronize()
        # exposed: from the end of the step's compute launches to the all-reduces' completion on the
        # launch stream (what the next step waits for); span: from the first bucket's start
        ex = [b.elapsed_time(c) for a, b, c in self._ar_events]
        sp = [a.elapsed_time(c) for a, b, c in self._ar_events]
        self._ar_events = None
        it_ms = t0.elapsed_time(t1)
        v = torch.tensor([sum(ex) / len(ex), max(ex), sum(ex), sum(sp) / len(sp), it_ms], dtype=torch.float64,
                         device=self.device)
        d = ddp.group()
        d.all_reduce(v, op=d.ReduceOp.MAX)
        mean_ms, max_ms, total_ms, span_ms, it_ms = (float(x) for x in v.cpu())
        return {"allreduce_ms_per_sgd_step": mean_ms, "allreduce_ms_max": max_ms, "sgd_steps": len(ex),
                "allreduce_span_ms_per_sgd_step": span_ms, "overlapped": self._overlap,
                "allreduce_ms_per_iteration": total_ms, "iteration_ms": it_ms,
                "allreduce_share_of_iteration": total_ms / it_ms if it_ms > 0 else None,
                "bytes_per_allreduce": int(self.grad.numel() * 4), "backend": d.get_backend()}

    # ------------------------------------------------------------------ RLlib surface
    def _episode_returns(self):
        """returns of the episodes completed this iteration in completion order (all ranks, at
        most RLKS_EPLOG_CAP per rank) and their total count"""
        torch = self.torch
        r, k, n = self.env.episode_log(clear=True)
        if self.world == 1:
            return r, n
        cap = _lib.RLKS_EPLOG_CAP
        mine = torch.zeros(2 * cap + 1, dtype=torch.float64, device=self.device)
        mine[: len(r)] = torch.from_numpy(r)
        mine[cap: cap + len(k)] = torch.from_numpy(k.astype(np.float64))  # keys < 2^53
        mine[2 * cap] = float(n)
        allv = torch.zeros(self.world, 2 * cap + 1, dtype=torch.float64, device=self.device)
        allv[self.rank] = mine
        self._allreduce(allv)
        a = allv.cpu().numpy()
        rets, keys, total = [], [], 0
        for q in range(self.world):
            nq = int(a[q, 2 * cap])
            kq = min(nq, cap)
            rets.append(a[q, :kq])
            keys.append(a[q, cap: cap + kq])
            total += nq
        rets, keys = np.concatenate(rets), np.concatenate(keys)
        return rets[np.argsort(keys, kind="stable")], total

    def _reward_mean(self, ep_sum, n_ep):
        """RLlib episode_reward_mean: the mean over this iteration's episodes, topped up with the
        most recent earlier ones to metrics_num_episodes_for_smoothing (Algorithm.
        _compile_iteration_results; RLlib third-party, parity unpinned)"""
        window = self._ep_history.maxlen
        rets, total = self._episode_returns()
        # >= window episodes: the mean of all of them, from the device sums.  Past RLKS_EPLOG_CAP the
        # log holds the first-logged episodes only, so the history kept for a later iteration with
        # fewer than `window` episodes is then approximate (such a later iteration needs lanes that
        # finish far out of step; all lanes of one rank reset together).
        if total >= window or total > len(rets):
            self._ep_history.extend(rets[-window:])
            return float(ep_sum / total) if total else float("nan")
        missing = window - total
        hist = list(self._ep_history)[-missing:] if missing > 0 else []
        vals = hist + list(rets)
        self._ep_history.extend(rets)
        return float(np.mean(vals)) if vals else float("nan")

    def evaluate(self, episodes=None):
        """greedy evaluation (RLlib evaluation workers, explore=False): `episodes` episodes, one
        lane each (train_final.py:19 .evaluation(evaluation_interval=5, evaluation_duration=20))"""
        from .evaluation import evaluate_lanes

        n = int(episodes or self.config.evaluation_duration)
        rets = evaluate_lanes(self.params, n, table=self.table, nodes=self.config.nodes,
                              seed=(self.seed * 7919 + self.iteration) & 0xFFFFFFFF, device=self.device)
        return {"episode_reward_mean": float(np.mean(rets)), "episode_reward_min": float(np.min(rets)),
                "episode_reward_max": float(np.max(rets)), "episodes_this_iter": n,
                "episode_len_mean": float(self.table.n_rows - 1)}

    def train(self):
        t0 = time.time()
        kl_before = float(self.dyn[_lib.RLKS_DYN_KL_COEFF].item())
        self.train_step_no_sync()
        self._allreduce(self.ep_stats)
        ep = self.ep_stats.cpu().numpy()
        st = self.stats.cpu().numpy()
        rows = st[:, _lib.RLKS_STAT_ROWS]
        n_ep = int(round(ep[1]))
        self.episodes_total += n_ep
        reward_mean = self._reward_mean(ep[0], n_ep)
        learner = {
            "policy_loss": float(np.mean(st[:, _lib.RLKS_STAT_POLICY_LOSS] / rows)),
            "vf_loss": float(np.mean(st[:, _lib.RLKS_STAT_VF_LOSS] / rows)),
            "kl": float(np.mean(st[:, _lib.RLKS_STAT_KL] / rows)),
            "entropy": float(np.mean(st[:, _lib.RLKS_STAT_ENTROPY] / rows)),
            "cur_kl_coeff": kl_before,
            "cur_lr": float(self.config.lr),
        }
        result = {
            "episode_reward_mean": reward_mean,
            "episode_reward_mean_this_iter": float(ep[0] / n_ep) if n_ep else float("nan"),
            "episodes_this_iter": n_ep,
            "episodes_total": self.episodes_total,
            "training_iteration": self.iteration,
            "timesteps_total": self.timesteps_total,
            "num_env_steps_sampled": self.timesteps_total,
            "info": {"learner": {"default_policy": {"learner_stats": learner}}},
        }
        # RLlib Algorithm.step(): evaluate when (iteration) % evaluation_interval == 0, after training
        iv = self.config.evaluation_interval
        if iv and self.iteration % int(iv) == 0:
            result["evaluation"] = self.evaluate()
        result["time_this_iter_s"] = time.time() - t0
        if self.reporter is not None:
            self.reporter.report(result, self)
        return result

    # Philox counter word 0 of policy-side draws (compute_actions / compute_single_action): no env
    # lane has this id, so these draws never repeat a rollout draw under the same key (config.seed)
    SAMPLER_ID = 0xFFFFFFFF

    def _sample(self, logits, explore):
        """TorchCategorical sample (explore) or argmax of logits [n, A] on the device sampler
        (rlks_sample_categorical): row i draws Philox({SAMPLER_ID, i, call counter, ACTION},
        key = config.seed), so a run's exploring actions follow from the seed and the number of
        earlier calls (the counter is checkpointed)"""
        torch = self.torch
        n = logits.shape[0]
        logits = logits.contiguous()
        act = torch.empty(n, dtype=torch.int32, device=self.device)
        ids = None
        if explore:
            idh = np.zeros((n, 3), np.uint32)
            idh[:, 0] = self.SAMPLER_ID
            idh[:, 1] = np.arange(n, dtype=np.uint32)
            idh[:, 2] = self.sample_calls & 0xFFFFFFFF
            ids = torch.from_numpy(idh.view(np.int32)).to(self.device)
            self.sample_calls += 1
        _lib.call("rlks_sample_categorical", _lib.ptr(logits), n, logits.shape[1], _lib.ptr(ids) if ids is not None else None,
                  self.seed & 0xFFFFFFFFFFFFFFFF, int(bool(explore)), _lib.ptr(act), None, self.stream)
        return act

    def compute_actions(self, obs, explore=None):
        """batched actions for obs [n, D] (device or host); returns an int32 device tensor"""
        torch = self.torch
        explore = self.config.explore if explore is None else explore
        o = torch.as_tensor(obs, dtype=torch.float32, device=self.device).reshape(-1, self.D)
        logits, _ = self.params.forward(o)
        return self._sample(logits, explore)

    def compute_single_action(self, observation=None, state=None, *, explore=None, **kw):
        """RLlib Algorithm.compute_single_action (eval_ppo.py:27 explores by default,
        final_evaluation.py:48 passes explore=False): one observation -> int action"""
        explore = self.config.explore if explore is None else explore
        o = np.asarray(observation, dtype=np.float32).reshape(1, self.D)
        logits, _ = self.params.forward(self.torch.from_numpy(o).to(self.device))
        return int(self._sample(logits, explore).item())

    def current_obs(self):
        """the lanes' current observations [N, D] (device)"""
        return self.buf["obs"][self.T] if self._carry else self.buf["obs"][0]

    def get_state(self):
        """everything a resumed run needs: weights, Adam moments and step, KL coefficient, counters,
        the smoothing window, and (checkpoint_env_state) the lanes' env state and current obs.
        The per-epoch gather permutation is keyed by (seed, iteration), so it resumes too."""
        torch = self.torch
        steps = torch.zeros(self.N, dtype=torch.int32, device=self.device)
        eps = torch.zeros(self.N, dtype=torch.int32, device=self.device)
        _lib.call("rlks_env_lane_state", self.env.handle, _lib.ptr(steps), _lib.ptr(eps), self.stream)
        st = {
            "weights": self.params.state_dict(),
            "adam_m": self.params.split(self.adam_m), "adam_v": self.params.split(self.adam_v),
            "param_offsets": list(self.params.offsets),
            "adam_step": self.adam_step, "kl_coeff": float(self.dyn[_lib.RLKS_DYN_KL_COEFF].item()),
            "iteration": self.iteration, "timesteps_total": self.timesteps_total,
            "episodes_total": self.episodes_total, "lane_steps": steps.cpu(), "lane_episodes": eps.cpu(),
            "episode_history": [float(x) for x in self._ep_history],
            "sample_calls": self.sample_calls,
            "rank": self.rank, "world": self.world,
        }
        if self._checkpoint_env_state():
            st["env_state"] = self.env.save_state().cpu()
            st["current_obs"] = self.current_obs().detach().cpu().clone()
        return st

    def _checkpoint_env_state(self):
        v = self.config.checkpoint_env_state
        return self.config.nodes is None if v is None else bool(v)

    def save(self, checkpoint_dir=None):
        """RLlib Algorithm.save(): writes <dir>/checkpoint_<iter:06d>/ and returns its path (no dir:
        this run's logdir, ~/ray_results/PPO_<env>_<time> or $RLKS_RESULTS_DIR, where
        rlks.checkpoints.latest_checkpoint finds it as final_evaluation.py:13-25 does).
        Files: state.pt (tensors, weights_only-loadable), algorithm_state.json (config + scalars),
        table.npz (the env table's float64 bits) and, with checkpoint_env_state, env_state.bin
        (raw device snapshot, rlks_env_save_state; rank-suffixed when world > 1).  The snapshot is
        rlks_env_state_bytes per rank: ~30 B per lane for table envs, plus clusters x nodes x 8 B
        per lane for node-level envs (about 1 GB at c3's 65,536 x 8 x 256, hence off by default
        there).  Multi-rank: every rank writes its own files, rank 0 the shared ones, then all
        ranks meet at a barrier."""
        import torch

        from .checkpoints import default_logdir

        if checkpoint_dir is None and self.config.logdir is None:
            # one logdir per run (RLlib's Algorithm.logdir), so that successive save() calls land
            # side by side and rlks.checkpoints.latest_checkpoint() finds the newest
            env = getattr(self.config.env, "__name__", None) or "K8sMultiCloudEnv"
            self.config.logdir = str(default_logdir(env))
        base = Path(checkpoint_dir) if checkpoint_dir else Path(self.config.logdir)
        path = base / f"checkpoint_{self.iteration:06d}"
        path.mkdir(parents=True, exist_ok=True)
        st = self.get_state()
        sfx = f".rank{self.rank}" if self.world > 1 else ""
        tensors = {f"weights/{k}": v for k, v in st.pop("weights").items()}
        for k in ("adam_m", "adam_v"):  # per tensor, like the weights
            tensors.update({f"{k}/{name}": v for name, v in st.pop(k).items()})
        tensors.update({k: st.pop(k) for k in ("lane_steps", "lane_episodes")})
        if "current_obs" in st:
            tensors["current_obs"] = st.pop("current_obs")
        env_state = st.pop("env_state", None)
        if env_state is not None:
            env_state.numpy().tofile(path / f"env_state{sfx}.bin")
            st["env_state_bytes"] = int(env_state.numel())
        st["env_state_saved"] = env_state is not None
        torch.save(tensors, path / f"state{sfx}.pt")
        if self.rank == 0:
            self.table.save(path / "table.npz")
            meta = {"state": st, "config": self.config.to_dict()}
            (path / "algorithm_state.json").write_text(json.dumps(meta, indent=1, default=str))
        if self.world > 1:  # a restore right after save() sees every rank's files
            ddp.group().barrier()
        return str(path)

    def restore(self, checkpoint_path, reset_optimizer=False):
        """load a checkpoint written by save().  Adam moments are saved per tensor (round 5 on); an
        older checkpoint's flat moments load only when it recorded the parameter layout they were
        written in (param_offsets equal to this policy's).  A flat buffer without that record cannot
        be placed safely (the flat layout order changed in round 4) and raises ValueError, unless
        reset_optimizer=True: then the weights and counters load and the moments restart at zero
        (with a warning), as a fresh Adam would."""
        import torch

        path = Path(checkpoint_path)
        meta = json.loads((path / "algorithm_state.json").read_text())["state"]
        saved_world = int(meta.get("world", 1))
        if saved_world != self.world:
            raise ValueError(f"checkpoint {path} was written by {saved_world} rank(s); this run has {self.world} "
                             "(per-rank env lanes and files do not transfer between world sizes)")
        sfx = f".rank{self.rank}" if self.world > 1 else ""
        tensors = torch.load(path / f"state{sfx}.pt", weights_only=True)
        sd = {k[len("weights/"):]: v for k, v in tensors.items() if k.startswith("weights/")}
        w = self.params.state_dict()
        for k, v in w.items():
            if tuple(sd[k].shape) != tuple(v.shape):
                raise ValueError(f"checkpoint tensor {k} has shape {tuple(sd[k].shape)}, this policy {tuple(v.shape)}")
        self.params.load_state_dict(sd)
        self._fused_prev = False
        for k, buf in (("adam_m", self.adam_m), ("adam_v", self.adam_v)):
            per = {n[len(k) + 1:]: v for n, v in tensors.items() if n.startswith(k + "/")}
            if per:
                self.params.join(buf, per)
            elif meta.get("param_offsets") == list(self.params.offsets):
                buf.copy_(tensors[k].to(self.device))  # a flat buffer saved with this very layout
            elif reset_optimizer:
                import warnings

                warnings.warn(f"checkpoint {path}: Adam moments saved without their parameter layout; "
                              "reset_optimizer=True: they restart at zero", RuntimeWarning, stacklevel=2)
                buf.zero_()
            else:
                # an older checkpoint: raw flat moments with no record of the storage order they were
                # written in; copying them could land one tensor's moments on another silently
                raise ValueError(f"checkpoint {path}: Adam moments saved as a flat buffer without their parameter "
                                 "layout; cannot restore them safely (restore(..., reset_optimizer=True) loads the "
                                 "weights and restarts Adam)")
        self.adam_step = int(meta["adam_step"])
        self.dyn[_lib.RLKS_DYN_KL_COEFF] = float(meta["kl_coeff"])
        self.iteration = int(meta["iteration"])
        self.timesteps_total = int(meta["timesteps_total"])
        self.episodes_total = int(meta["episodes_total"])
        self._ep_history.clear()
        self._ep_history.extend(meta.get("episode_history", []))
        self.sample_calls = int(meta.get("sample_calls", 0))
        es = path / f"env_state{sfx}.bin"
        if es.exists() and "current_obs" in tensors:
            self.env.load_state(np.fromfile(es, dtype=np.uint8))
            self.buf["obs"][0].copy_(tensors["current_obs"].to(self.device))
            self._carry = False
            self.env.episode_log(clear=True)
        else:
            # node-level envs default to checkpoint_env_state off (~1 GB per save at c3): weights,
            # Adam state and counters resume, the env lanes start fresh, so the run is not a
            # bit-exact continuation
            import warnings

            why = ("saved with checkpoint_env_state off" if not meta.get("env_state_saved", True)
                   else "its env_state file is missing")
            warnings.warn(f"checkpoint {path}: {why}; the env lanes keep their current state, so the resumed "
                          "run is not an exact continuation (set PPOConfig.checkpoint_env_state = True)",
                          RuntimeWarning, stacklevel=2)

    @classmethod
    def from_checkpoint(cls, checkpoint_path, config: PPOConfig | None = None, **kw):
        from .tables import Table

        path = Path(checkpoint_path)
        if config is None:
            config = PPOConfig.from_dict(json.loads((path / "algorithm_state.json").read_text())["config"])
            if (path / "table.npz").exists():
                config.table = Table.load(path / "table.npz")
        algo = cls(config=config, **kw)
        algo.restore(path)
        return algo

    def stop(self):
        self.env.close()
