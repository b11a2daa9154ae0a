"""ctypes binding of librlks.so (the C ABI declared in include/rlks.h).

The library is the only compute path: there is no CPU fallback.  Loading fails loudly when
librlks.so is missing (run ``python -c "import __graft_entry__ as g; g.build()"`` or
``make -C rl-k8s-scheduler_amd/csrc``).  Device pointers come from torch tensors
(``tensor.data_ptr()``); the stream is torch's current HIP stream.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("RLKS_LIB", PKG_DIR / "librlks.so"))

RLKS_NOISE_PHILOX = 0
RLKS_NOISE_MT19937 = 1
RLKS_N_TENSORS = 12
RLKS_DYN_SIZE = 8
RLKS_DYN_ADV_MEAN, RLKS_DYN_ADV_INVSTD, RLKS_DYN_KL_COEFF, RLKS_DYN_INV_COUNT = 0, 1, 2, 3
RLKS_STAT_SIZE = 8
RLKS_PHASE_FWD, RLKS_PHASE_DW2, RLKS_PHASE_DH1, RLKS_PHASE_REDUCE, RLKS_PHASE_ALL = 1, 2, 4, 8, 15
RLKS_PHASE_FWD_PI, RLKS_PHASE_FWD_VF, RLKS_PHASE_PREP, RLKS_PHASE_F1A, RLKS_PHASE_F1B = 16, 32, 64, 128, 256
RLKS_PRECISION_FP32, RLKS_PRECISION_SF16, RLKS_PRECISION_WIDE, RLKS_PRECISION_F16 = 0, 1, 2, 3
RLKS_STAT_POLICY_LOSS, RLKS_STAT_VF_LOSS, RLKS_STAT_KL, RLKS_STAT_ENTROPY, RLKS_STAT_ROWS = 0, 1, 2, 3, 4
RLKS_EPLOG_CAP = 128


class EnvCfg(C.Structure):
    """mirror of rlks_env_cfg (include/rlks_types.h)"""

    _fields_ = [
        ("n_envs", C.c_int32), ("n_rows", C.c_int32), ("n_clouds", C.c_int32), ("max_steps", C.c_int32),
        ("noise_mode", C.c_int32), ("autoreset", C.c_int32), ("env_offset", C.c_int32), ("skip_returns", C.c_int32),
        ("seed", C.c_uint64), ("cpu_lo", C.c_double), ("cpu_hi", C.c_double), ("w_cost", C.c_double),
        ("w_lat", C.c_double), ("scale", C.c_double),
        ("nodes_per_cluster", C.c_int32), ("pod_cpu_m", C.c_int32), ("pod_mem_mi", C.c_int32),
        ("arrival_mode", C.c_int32), ("arrival_rate", C.c_double), ("depart_prob", C.c_double),
        ("init_occupancy", C.c_double), ("reject_penalty", C.c_double),
    ]


class GemmDesc(C.Structure):
    _fields_ = [("a", C.c_void_p), ("b", C.c_void_p), ("c", C.c_void_p), ("bias", C.c_void_p), ("aux", C.c_void_p),
                ("m", C.c_int32), ("n", C.c_int32), ("k", C.c_int32), ("lda", C.c_int32), ("ldb", C.c_int32),
                ("ldc", C.c_int32), ("ldaux", C.c_int32), ("trans_a", C.c_int32), ("trans_b", C.c_int32),
                ("epilogue", C.c_int32), ("accumulate", C.c_int32), ("reserved", C.c_int32),
                ("a_max", C.c_void_p), ("b_max", C.c_void_p), ("c_max", C.c_void_p)]


RLKS_GEMM_STORE, RLKS_GEMM_TANH_BIAS, RLKS_GEMM_BIAS, RLKS_GEMM_DTANH = 0, 1, 2, 3


class MlpDesc(C.Structure):
    _fields_ = [("obs_dim", C.c_int32), ("hidden", C.c_int32), ("n_actions", C.c_int32), ("precision", C.c_int32)]


class PpoCoeffs(C.Structure):
    _fields_ = [("clip_param", C.c_float), ("vf_clip_param", C.c_float), ("vf_loss_coeff", C.c_float),
                ("entropy_coeff", C.c_float)]


class RolloutBufs(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("logits", C.c_void_p), ("values", C.c_void_p), ("actions", C.c_void_p),
                ("logp", C.c_void_p), ("rewards", C.c_void_p), ("dones", C.c_void_p), ("adv", C.c_void_p),
                ("vtarg", C.c_void_p), ("T", C.c_int32), ("N", C.c_int32), ("global_lanes", C.c_int32)]


class GatherNext(C.Structure):
    """rlks_gather_next: the next SGD step's packed gather (rlks_ppo_sgd_step_next)"""
    _fields_ = [("packed", C.c_void_p), ("mb", C.c_void_p), ("perm_seed", C.c_uint64), ("row0", C.c_int64),
                ("T", C.c_int32), ("N", C.c_int32), ("epoch", C.c_int32), ("groups", C.c_int32),
                ("group0", C.c_int32), ("rows", C.c_int32)]


_P = C.c_void_p
_I = C.c_int
_I64 = C.c_int64
_F = C.c_float

# name -> argtypes (restype is int unless listed in _RESTYPES)
SIGNATURES = {
    "rlks_last_error": [],
    "rlks_version": [],
    "rlks_env_create": [C.POINTER(EnvCfg), _P, _P, C.POINTER(_P)],
    "rlks_env_create_ext": [C.POINTER(EnvCfg), _P, _P, _P, _P, _P, _I, C.POINTER(_P)],
    "rlks_env_destroy": [_P],
    "rlks_env_node_state": [_P, _P, _P, _P, _P],
    "rlks_env_counters": [_P, _I, _P, _P],
    "rlks_env_config": [_P, C.POINTER(EnvCfg)],
    "rlks_env_seed": [_P, _P, _P, _P, _I, _P],
    "rlks_env_mt_discard": [_P, _P, _P, _P],
    "rlks_env_mt_words": [_P, C.c_int, _P, C.c_int, _P],
    "rlks_debug_checks": [_P],
    "rlks_debug_sf_handoff": [C.POINTER(MlpDesc), _I, _P, _P],
    "rlks_debug_wide_bufs": [C.POINTER(MlpDesc), _I, _P, _P],
    "rlks_sample_categorical": [_P, C.c_int, C.c_int, _P, C.c_ulonglong, C.c_int, _P, _P, _P],
    "rlks_env_reset": [_P, _P, _P, _P],
    "rlks_env_step": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "rlks_env_sample_step": [_P, _P, _I, _P, _P, _P, _P, _P, _P],
    "rlks_env_episode_stats": [_P, _P, _I, _P],
    "rlks_env_lane_state": [_P, _P, _P, _P],
    "rlks_env_episode_log": [_P, _P, _P, _P, _I, _P],
    "rlks_env_state_bytes": [_P, C.POINTER(_I64)],
    "rlks_env_save_state": [_P, _P, _P],
    "rlks_env_load_state": [_P, _P, _P],
    "rlks_philox4x32_10": [_P, _P, _P, _I, _P],
    "rlks_mt_random": [_P, _I, _P, _I, _P],
    "rlks_gae": [_P, _P, _P, _F, _F, _I, _I, _P, _P, _P, _P],
    "rlks_gae_partials_count": [_I],
    "rlks_adv_stats": [_P, _I, C.c_double, _P, _P],
    "rlks_adv_finalize": [_P, _P, _P],
    "rlks_mlp_layout": [C.POINTER(MlpDesc), C.POINTER(_I64), C.POINTER(_I64), C.POINTER(_I64)],
    "rlks_policy_forward": [C.POINTER(MlpDesc), _P, _P, _I, _P, _P, _P],
    "rlks_rollout": [_P, C.POINTER(MlpDesc), _P, C.POINTER(RolloutBufs), _I, _P],
    "rlks_gemm_sf16": [C.POINTER(GemmDesc), _P],
    "rlks_absmax": [_P, _I, _I, _I, _P, _P],
    "rlks_policy_forward_ws": [C.POINTER(MlpDesc), _P, _P, _I, _P, _P, _P, _I64, _P],
    "rlks_rollout_ws": [_P, C.POINTER(MlpDesc), _P, C.POINTER(RolloutBufs), _I, _P, _I64, _P],
    "rlks_minibatch_stride": [C.POINTER(MlpDesc)],
    "rlks_ppo_gather": [C.POINTER(MlpDesc), C.POINTER(RolloutBufs), C.c_uint64, _I, _I64, _I, _P, _P, _P],
    "rlks_ppo_gather_grouped": [C.POINTER(MlpDesc), C.POINTER(RolloutBufs), C.c_uint64, _I, _I, _I, _I64, _I, _P,
                                _P, _P],
    "rlks_packed_stride": [C.POINTER(MlpDesc)],
    "rlks_ppo_pack": [C.POINTER(MlpDesc), C.POINTER(RolloutBufs), _P, _P],
    "rlks_ppo_gather_packed": [C.POINTER(MlpDesc), _P, _I, _I, C.c_uint64, _I, _I, _I, _I64, _I, _P, _P],
    "rlks_ppo_workspace_bytes": [C.POINTER(MlpDesc), _I, C.POINTER(_I64)],
    "rlks_ppo_grad": [C.POINTER(MlpDesc), C.POINTER(PpoCoeffs), _P, _P, _P, _I, _P, _P, _P, _I64, _P],
    "rlks_ppo_grad_phases": [C.POINTER(MlpDesc), C.POINTER(PpoCoeffs), _P, _P, _P, _I, _P, _P, _P, _I64, _I, _P],
    "rlks_ppo_grad_profile": [C.POINTER(MlpDesc), C.POINTER(PpoCoeffs), _P, _P, _P, _I, _P, _P, _P, _I64, _I, _P, _P],
    "rlks_sf_f1_fused": [C.POINTER(MlpDesc)],
    "rlks_adam_step": [_P, _P, _P, _P, _I64, _F, _F, _F, _F, _I, _P],
    "rlks_ppo_sgd_step": [C.POINTER(MlpDesc), C.POINTER(PpoCoeffs), _P, _P, _P, _I, _P, _P, _P, _P, _I64, _F, _F, _F,
                          _F, _I, _I, _P, _I64, _P],
    "rlks_ppo_sgd_step_next": [C.POINTER(MlpDesc), C.POINTER(PpoCoeffs), _P, _P, _P, _I, _P, _P, _P, _P, _I64, _F,
                               _F, _F, _F, _I, _I, C.POINTER(GatherNext), _P, _I64, _P],
    "rlks_ppo_grad_step": [C.POINTER(MlpDesc), C.POINTER(PpoCoeffs), _P, _P, _P, _I, _P, _P, _I, _I, _P, _I64, _P],
    "rlks_ppo_grad_step_next": [C.POINTER(MlpDesc), C.POINTER(PpoCoeffs), _P, _P, _P, _I, _P, _P, _I, _I,
                                C.POINTER(GatherNext), _P, _I64, _P],
    "rlks_ppo_grad_step_part": [C.POINTER(MlpDesc), C.POINTER(PpoCoeffs), _P, _P, _P, _I, _P, _P, _I, _I, _I,
                                C.POINTER(GatherNext), _P, _I64, _P],
    "rlks_ppo_adam_apply": [C.POINTER(MlpDesc), _P, _P, _P, _P, _I64, _F, _F, _F, _F, _I, _P, _I64, _I, _P],
    "rlks_kl_update": [_P, _P, _F, _P],
}
_RESTYPES = {"rlks_last_error": C.c_char_p, "rlks_version": C.c_char_p}


class RlksError(RuntimeError):
    pass


_lib = None
# entry points an older variant library (RLKS_LIB, same-box A/B runs) may lack: diagnostics and build
# introspection, never compute.  The product library must export all of them (tests/test_abi_host.py)
_OPTIONAL = {n for n in SIGNATURES if n.startswith("rlks_debug_")} | {"rlks_sf_f1_fused"}


def _warn_if_stale() -> None:
    """Warn when a HIP source or header is newer than the library about to be loaded: a library
    left over from an earlier build would otherwise be measured and tested silently."""
    if "RLKS_LIB" in os.environ:
        return
    csrc = PKG_DIR.parent / "csrc"
    srcs = [p for pat in ("*.hip", "*.h") for p in csrc.glob(pat)]
    srcs += list((PKG_DIR.parent.parent / "include").glob("*.h"))
    if not srcs:
        return
    newest = max(srcs, key=lambda p: p.stat().st_mtime)
    if newest.stat().st_mtime > LIB_PATH.stat().st_mtime + 1.0:
        import warnings

        warnings.warn(f"{LIB_PATH} is older than {newest.name}; rebuild with `make -C {csrc}`", stacklevel=3)


def lib() -> C.CDLL:
    """Load librlks.so once; raises if it is absent (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RlksError(f"librlks.so not found at {LIB_PATH}; build it with `make -C {PKG_DIR.parent / 'csrc'}`")
        _warn_if_stale()
        handle = C.CDLL(str(LIB_PATH))
        for name, argtypes in SIGNATURES.items():
            if name in _OPTIONAL and "RLKS_LIB" in os.environ and not hasattr(handle, name):
                continue  # entry points of later builds, absent from an older variant library (A/B runs)
            fn = getattr(handle, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, C.c_int)
        _lib = handle
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().rlks_last_error().decode(errors="replace")
        raise RlksError(f"{what or 'rlks'} failed ({rc}): {msg}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


def ptr(t) -> int | None:
    """device pointer of a torch tensor (None passes NULL)"""
    return None if t is None else t.data_ptr()


def stream_handle(torch_mod=None):
    import torch

    return torch.cuda.current_stream().cuda_stream
