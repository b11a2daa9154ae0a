"""Policy / value network parameters: RLlib's default torch FCNet with vf_share_layers=False.

Reference: `PPOConfig().framework("torch")` (train_ppo.py:12) with RLlib's default model config
(fcnet_hiddens [256, 256], fcnet_activation "tanh", vf_share_layers False).  RLlib builds
    _hidden_layers: SlimFC(D->256, tanh), SlimFC(256->256, tanh)   normc_initializer(1.0)
    _logits:        SlimFC(256->A)                                   normc_initializer(0.01)
    _value_branch_separate: SlimFC(D->256, tanh), SlimFC(256->256, tanh)  normc(1.0)
    _value_branch:  SlimFC(256->1)                                   normc_initializer(0.01)
with zero biases; normc(std) draws N(0,1) and scales each output row to L2 norm `std`.
135,939 parameters at D=6, A=2.  [RLlib is third-party and absent here: parity unpinned.]

The parameters live in ONE flat fp32 device buffer (include/rlks.h, rlks_mlp_layout) so that the
gradient all-reduce is a single RCCL call and Adam is one elementwise kernel.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

# flat tensor order of include/rlks.h and the RLlib state_dict key of each
TENSOR_NAMES = [
    ("_hidden_layers.0._model.0.weight", "w1", 0), ("_hidden_layers.0._model.0.bias", "b1", 0),
    ("_hidden_layers.1._model.0.weight", "w2", 0), ("_hidden_layers.1._model.0.bias", "b2", 0),
    ("_logits._model.0.weight", "w3", 0), ("_logits._model.0.bias", "b3", 0),
    ("_value_branch_separate.0._model.0.weight", "w1", 1), ("_value_branch_separate.0._model.0.bias", "b1", 1),
    ("_value_branch_separate.1._model.0.weight", "w2", 1), ("_value_branch_separate.1._model.0.bias", "b2", 1),
    ("_value_branch._model.0.weight", "w3", 1), ("_value_branch._model.0.bias", "b3", 1),
]


def tensor_shapes(D: int, H: int, A: int):
    return [(H, D), (H,), (H, H), (H,), (A, H), (A,), (H, D), (H,), (H, H), (H,), (1, H), (1,)]


def layout(D: int, H: int, A: int):
    """(offsets[12], padded_count, real_count) from the library (single source of truth)"""
    desc = _lib.MlpDesc(D, H, A, 0)
    offs = (C.c_int64 * 12)()
    padded, real = C.c_int64(), C.c_int64()
    _lib.call("rlks_mlp_layout", C.byref(desc), offs, C.byref(padded), C.byref(real))
    return list(offs), padded.value, real.value


def normc(shape, std, gen):
    import torch

    w = torch.randn(shape, generator=gen, dtype=torch.float32)
    return w * (std / torch.sqrt(w.pow(2).sum(1, keepdim=True)))


class PolicyParams:
    """Flat parameter buffer + named views (torch [out][in] layout)."""

    def __init__(self, obs_dim=6, hidden=256, n_actions=2, device=None, seed=0):
        import torch

        self.D, self.H, self.A = int(obs_dim), int(hidden), int(n_actions)
        self.desc = _lib.MlpDesc(self.D, self.H, self.A, 0)
        self.offsets, self.padded, self.real = layout(self.D, self.H, self.A)
        self.shapes = tensor_shapes(self.D, self.H, self.A)
        self.device = device
        self.flat = torch.zeros(self.padded, dtype=torch.float32, device=device)
        self.init(seed)

    def view(self, i):
        n = int(np.prod(self.shapes[i]))
        return self.flat[self.offsets[i]: self.offsets[i] + n].view(self.shapes[i])

    def init(self, seed=0):
        import torch

        gen = torch.Generator().manual_seed(int(seed))
        host = torch.zeros(self.padded, dtype=torch.float32)
        for i, (name, kind, net) in enumerate(TENSOR_NAMES):
            shp = self.shapes[i]
            if kind.startswith("w"):
                std = 0.01 if kind == "w3" else 1.0
                t = normc(shp, std, gen)
            else:
                t = torch.zeros(shp)
            n = t.numel()
            host[self.offsets[i]: self.offsets[i] + n] = t.reshape(-1)
        self.flat.copy_(host)

    def state_dict(self):
        """RLlib FCNet state_dict names -> CPU tensors"""
        return {name: self.view(i).detach().cpu().clone() for i, (name, _, _) in enumerate(TENSOR_NAMES)}

    def load_state_dict(self, sd):
        for i, (name, _, _) in enumerate(TENSOR_NAMES):
            self.view(i).copy_(sd[name].to(self.flat.device))

    def split(self, buf):
        """a buffer laid out like `flat` (the Adam moments, a gradient) -> {state_dict name: CPU
        tensor}: checkpoints keep per-parameter state per tensor, so a change of the flat storage
        order (mlp_common.h LAYOUT_ORDER) cannot move it onto the wrong tensor"""
        out = {}
        for i, (name, _, _) in enumerate(TENSOR_NAMES):
            n = int(np.prod(self.shapes[i]))
            out[name] = buf[self.offsets[i]: self.offsets[i] + n].view(self.shapes[i]).detach().cpu().clone()
        return out

    def join(self, buf, sd):
        """inverse of split(): copy {name: tensor} into `buf` at this layout's offsets"""
        for i, (name, _, _) in enumerate(TENSOR_NAMES):
            if tuple(sd[name].shape) != tuple(self.shapes[i]):
                raise ValueError(f"tensor {name} has shape {tuple(sd[name].shape)}, this policy {tuple(self.shapes[i])}")
            n = int(np.prod(self.shapes[i]))
            buf[self.offsets[i]: self.offsets[i] + n].copy_(sd[name].reshape(-1).to(buf.device))

    def forward(self, obs, logits=None, values=None):
        """logits [n, A], values [n] for obs [n, D] (device tensors)"""
        import torch

        n = obs.shape[0]
        if logits is None:
            logits = torch.empty(n, self.A, dtype=torch.float32, device=obs.device)
        if values is None:
            values = torch.empty(n, dtype=torch.float32, device=obs.device)
        obs = obs.contiguous()
        stream = torch.cuda.current_stream(obs.device).cuda_stream
        if self.wide():  # generic-width path: needs a workspace for the activations
            wsb = C.c_int64()
            _lib.call("rlks_ppo_workspace_bytes", C.byref(self.desc), max(1, n), C.byref(wsb))
            if getattr(self, "_fws", None) is None or self._fws.numel() < wsb.value:
                self._fws = torch.empty(wsb.value, dtype=torch.uint8, device=obs.device)
            _lib.call("rlks_policy_forward_ws", C.byref(self.desc), _lib.ptr(self.flat), _lib.ptr(obs), n,
                      _lib.ptr(logits), _lib.ptr(values), _lib.ptr(self._fws), self._fws.numel(), stream)
        else:
            _lib.call("rlks_policy_forward", C.byref(self.desc), _lib.ptr(self.flat), _lib.ptr(obs), n,
                      _lib.ptr(logits), _lib.ptr(values), stream)
        return logits, values

    def wide(self):
        """True when the generic-width path runs (the fused kernels cover hidden 256, obs < 32 and
        2 / 4 / 8 actions)"""
        return (self.desc.precision == _lib.RLKS_PRECISION_WIDE or self.H != 256 or self.A not in (2, 4, 8)
                or self.D + 1 > 32)
