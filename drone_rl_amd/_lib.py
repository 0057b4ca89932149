"""ctypes binding of libdronerl.so (the C ABI declared in include/dronerl.h).

The product path has no CPU fallback: if the shared library is missing or
does not export the ABI, importing this module's `lib()` raises.  torch is
imported first so that the process has exactly one HIP runtime (torch's
bundled libamdhip64.so.7 satisfies the library's DT_NEEDED by soname).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, c_char_p, c_double, c_float, c_int, c_int32,
                    c_int64, c_size_t, c_uint8, c_uint64, c_void_p)

import torch  # noqa: F401  (must precede the CDLL load: one HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DRONERL_LIB", os.path.join(_HERE, "libdronerl.so"))

DR_OK = 0
DR_ERR_INVALID = -1
DR_ERR_HIP = -2
DR_ERR_NOMEM = -3
DR_ERR_UNSUPPORTED = -4

ABI_VERSION = 16                # DR_ABI_VERSION in include/dronerl.h
DR_VARIANT_GYM = 0
DR_VARIANT_VECTORIZED = 1
DR_VARIANT_MOVING = 2
DR_STATE_F64 = 0
DR_STATE_F32 = 1
DR_RNG_PHILOX = 0
DR_RNG_HOST_UNIFORMS = 1

FIELDS = {"pos": 0, "vel": 1, "euler": 2, "omega": 3, "target": 4,
          "current_step": 5, "ep_num": 6, "eps": 7, "ep_return": 8,
          "ep_length": 9, "motion": 10}


class dr_config(ctypes.Structure):
    _fields_ = [("num_envs", c_int64), ("variant", c_int32),
                ("state_dtype", c_int32), ("rng_mode", c_int32),
                ("auto_reset", c_int32), ("device", c_int32),
                ("max_steps", c_int32), ("seed", c_uint64),
                ("env_id_offset", c_int64), ("dt", c_double)]


class dr_grad_finish(ctypes.Structure):
    """include/dronerl.h dr_grad_finish (deferred gradient reductions)."""
    _fields_ = [("head_workspace", c_void_p), ("head_m", c_int64), ("head_hd", c_int64),
                ("log_std", c_void_p), ("ent_coef", c_float), ("vf_coef", c_float),
                ("g_w_act", c_void_p), ("g_b_act", c_void_p), ("g_w_val", c_void_p),
                ("g_b_val", c_void_p), ("g_b_pi", c_void_p), ("g_b_vf", c_void_p),
                ("g_log_std", c_void_p), ("stats", c_void_p),
                ("first_workspace", c_void_p), ("first_m", c_int64), ("first_k", c_int64),
                ("first_n", c_int64),
                ("g_w0", c_void_p), ("g_b0", c_void_p), ("g_w1", c_void_p), ("g_b1", c_void_p),
                ("chunks", c_void_p), ("chunk_groups", c_int64), ("chunk_count", c_int64),
                ("chunk_size", c_int64), ("chunk_dst", c_void_p), ("first_rows", c_int64),
                ("head_direct", c_int64)]


class DroneRLError(RuntimeError):
    """A libdronerl entry point returned a negative status."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"libdronerl error {code}: {msg}")
        self.code = code


# name -> (restype, argtypes); the complete exported ABI of include/dronerl.h
_P = c_void_p
SIGNATURES = {
    "dr_abi_version": (c_int, []),
    "dr_create": (c_int, [POINTER(dr_config), POINTER(c_void_p)]),
    "dr_destroy": (c_int, [_P]),
    "dr_num_envs": (c_int64, [_P]),
    "dr_obs_dim": (c_int, [_P]),
    "dr_reset": (c_int, [_P, _P, _P]),
    "dr_reset_masked": (c_int, [_P, _P, _P, _P]),
    "dr_step": (c_int, [_P, _P, _P, _P, _P, _P, _P]),
    "dr_step_monitored": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "dr_step_monitored_trunc": (c_int, [_P] * 10),
    "dr_get_state": (c_int, [_P, c_int, _P, _P]),
    "dr_gather_state": (c_int, [_P, c_int, _P, c_int64, _P, _P]),
    "dr_set_state": (c_int, [_P, c_int, _P, _P]),
    "dr_set_reset_uniforms": (c_int, [_P, _P]),
    "dr_set_seed": (c_int, [_P, c_uint64]),
    "dr_rollout": (c_int, [_P, c_int32, _P, _P, _P, _P, _P]),
    "dr_rollout_timed": (c_int, [_P, c_int32, _P, _P, _P, _P, _P, _P, _P]),
    "dr_rollout_random": (c_int, [_P, c_int32, c_uint64, c_int64, c_float, c_float, _P, _P,
                                  _P, _P, _P]),
    "dr_random_actions": (c_int, [c_int64, c_uint64, c_int64, c_int64, c_float,
                                  c_float, _P, _P]),
    "dr_last_error": (c_char_p, [_P]),
    "dr_gae": (c_int, [c_int64, c_int64, _P, _P, _P, _P, _P, c_double, c_double,
                       _P, _P, _P]),
    "dr_policy_sample": (c_int, [c_int64, _P, _P, c_uint64, c_uint64, c_float,
                                 c_float, _P, _P, _P, _P]),
    "dr_policy_sample_dev": (c_int, [c_int64, _P, _P, c_uint64, _P, c_uint64, c_float,
                                     c_float, _P, _P, _P, _P]),
    "dr_permutation_workspace_bytes": (c_size_t, [c_int64]),
    "dr_permutation": (c_int, [c_int64, c_uint64, c_uint64, _P, _P, c_size_t, _P]),
    "dr_permutation_dev": (c_int, [c_int64, c_uint64, _P, c_uint64, _P, _P, c_size_t, _P]),
    "dr_gather_rows": (c_int, [c_int64, c_int64, _P, _P, _P, _P]),
    "dr_gather_minibatch": (c_int, [c_int64, _P, c_int64] + [_P] * 8),
    "dr_pack_rollout_records": (c_int, [c_int64, c_int64] + [_P] * 7),
    "dr_gather_records": (c_int, [c_int64, _P, c_int64] + [_P] * 6),
    "dr_linear_tanh2": (c_int, [c_int64, c_int64, c_int64] + [_P] * 9),
    "dr_first_layer_backward2_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "dr_first_layer_backward2": (c_int, [c_int64, c_int64, c_int64] + [_P] * 10 +
                                 [c_int, _P, c_size_t, _P]),
    "dr_tanh_backward_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "dr_tanh_backward": (c_int, [c_int64, c_int64, _P, _P, _P, _P, _P, c_size_t, _P]),
    "dr_linear_tanh": (c_int, [c_int64, c_int64, c_int64, _P, _P, _P, _P, _P, _P]),
    "dr_first_layer_backward_workspace_bytes": (c_size_t, [c_int64, c_int64, c_int64]),
    "dr_first_layer_backward": (c_int, [c_int64, c_int64, c_int64, _P, _P, _P, _P, _P, _P,
                                        _P, c_size_t, _P]),
    "dr_policy_heads": (c_int, [c_int64, c_int64, c_int] + [_P] * 11),
    "dr_ppo_head_workspace_bytes": (c_size_t, [c_int64, c_int64]),
    "dr_ppo_head_loss_backward": (c_int, [c_int64, c_int64, c_int] + [_P] * 12 +
                                  [c_float, c_float, c_float, c_int] + [_P] * 10 +
                                  [c_int, _P, c_size_t, _P]),
    "dr_ppo_loss_workspace_bytes": (c_size_t, [c_int64]),
    "dr_ppo_loss": (c_int, [c_int64, _P, _P, _P, _P, _P, _P, _P, c_int64, c_float,
                            c_float, c_float, c_int, _P, _P, _P, _P, _P,
                            c_size_t, _P]),
    "dr_adam_workspace_bytes": (c_size_t, [c_int64]),
    "dr_clip_adam": (c_int, [c_int64, _P, _P, _P, _P, c_double, c_double, c_double,
                             c_double, c_float, c_int64, _P, _P, c_size_t, _P]),
    "dr_grad_finish_workspace_bytes": (c_size_t, [_P]),
    "dr_grad_finish_clip_adam": (c_int, [_P, c_int64, _P, _P, _P, _P, c_double, c_double,
                                         c_double, c_double, c_float, c_int64, _P, _P,
                                         c_size_t, _P]),
    "dr_adam_schedule": (c_int, [c_double, c_double, c_double, c_int64, _P]),
    "dr_grad_finish_clip_adam_sched": (c_int, [_P, c_int64, _P, _P, _P, _P, c_double, c_double,
                                               c_double, c_double, c_float, _P, _P, _P,
                                               c_size_t, _P]),
    "dr_grad_finish_run": (c_int, [_P, _P, c_size_t, _P]),
    "dr_clip_adam_sched": (c_int, [c_int64, _P, _P, _P, _P, c_double, c_double, c_double,
                                   c_float, c_float, _P, _P, _P, c_size_t, _P]),
    "dr_gemm_x6_weights_bytes": (c_size_t, [c_int64]),
    "dr_gemm_x6_split_weights": (c_int, [c_int64, _P, c_int, _P, _P]),
    "dr_gemm_x6": (c_int, [c_int64, c_int64, _P, _P, _P, _P]),
    "dr_gemm_x6_wgrad": (c_int, [c_int64, c_int64, c_int64, _P, _P, _P, _P]),
    "dr_gemm_x6_x_bytes": (c_size_t, [c_int64]),
    "dr_gemm_x6_split_x": (c_int, [c_int64, c_int64, _P, _P, _P]),
    "dr_gemm_x6_bwd_first": (c_int, [c_int64, c_int64, c_int64, _P, _P, _P, _P, _P, c_size_t,
                                     c_int, _P]),
    "dr_gemm_x6_bwd_first_rows": (c_int64, [c_int64]),
    "dr_linear_tanh2_x6": (c_int, [c_int64, c_int64, c_int64, _P, _P, _P, _P, _P, _P, _P, _P,
                                   _P, _P, _P, _P]),
}

_lib = None


def lib() -> ctypes.CDLL:
    """Load libdronerl.so once; raise if it is missing or incomplete."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libdronerl.so not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback for the GPU env)")
    l = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(l, name)  # AttributeError = missing export: loud
        fn.restype = res
        fn.argtypes = args
    if l.dr_abi_version() != ABI_VERSION:
        raise ImportError("libdronerl.so ABI version mismatch")
    _lib = l
    return l


def last_error(handle=None) -> str:
    msg = lib().dr_last_error(handle)
    return msg.decode() if msg else ""


def check(rc: int, handle=None) -> None:
    if rc != DR_OK:
        raise DroneRLError(rc, last_error(handle))


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(stream=None) -> int:
    s = torch.cuda.current_stream() if stream is None else stream
    return s.cuda_stream
