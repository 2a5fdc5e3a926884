"""ctypes binding of libasr.so (include/asr.h).

This is the ONLY way the package computes: every public operation ends in one
of these C entry points, which launch the hand-written gfx950 kernels.  If the
library is missing or cannot be loaded the package raises — there is no
CPU or PyTorch fallback for the hot path.
"""
from __future__ import annotations

import ctypes as ct
import os

try:  # torch must own the HIP runtime before libasr binds to it (one runtime per process)
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

from . import _build

ASR_OK = 0
ASR_E_ARG = -1
ASR_E_UNSUPPORTED = -2
ASR_E_WORKSPACE = -3
ASR_E_HIP = -4
ASR_E_DEVICE = -5

ASR_F32 = 0
ASR_BF16 = 1
ASR_PARAM_3BY3 = 0
ASR_PARAM_GENERAL = 1
ASR_PARAM_REGULAR = 2
ABI_VERSION = 8
ASR_MODE_EULER = 0
ASR_MODE_CONV = 1
ASR_INTEGRATOR_EULER = 0
ASR_INTEGRATOR_RK2 = 1
ASR_VARIANT_NO_FOLD = 1
ASR_VARIANT_STEM_FWD_VALU = 2
ASR_VARIANT_STEM_WGRAD_VALU = 4
ASR_VARIANT_PER_BLOCK_FWD = 8
ASR_VARIANT_PER_BLOCK_BWD = 16
ASR_VARIANT_INFERENCE = 32
ASR_VARIANT_TIMED = 64
ASR_VARIANT_FULL_DXL = 128
ASR_VARIANT_FULL_SLABS = 256
ASR_VARIANT_W_BF16 = 512
ASR_DIST_UNIQUE_ID_BYTES = 128
ASR_STAGES_MAX = 8


class AsrError(RuntimeError):
    pass


class AsrUnsupported(AsrError, NotImplementedError):
    pass


class NetConfig(ct.Structure):
    _fields_ = [
        ("N", ct.c_int), ("H", ct.c_int), ("W", ct.c_int), ("Cin", ct.c_int), ("C", ct.c_int), ("L", ct.c_int),
        ("num_classes", ct.c_int), ("h", ct.c_float), ("gamma", ct.c_float), ("subtract_mean", ct.c_float),
        ("divide_by_stddev", ct.c_float), ("use_norm", ct.c_int), ("dtype", ct.c_int), ("input_u8", ct.c_int),
        ("param_kind", ct.c_int), ("antisymmetric", ct.c_int), ("integrator", ct.c_int), ("variant", ct.c_int),
    ]


class StagesConfig(ct.Structure):
    """asr_stages_config (include/asr.h, ABI 7)."""
    _fields_ = [
        ("N", ct.c_int), ("H", ct.c_int), ("W", ct.c_int), ("Cin", ct.c_int), ("num_classes", ct.c_int),
        ("n_stages", ct.c_int), ("C", ct.c_int * 8), ("L", ct.c_int * 8), ("stride", ct.c_int * 8),
        ("h", ct.c_float), ("gamma", ct.c_float), ("subtract_mean", ct.c_float), ("divide_by_stddev", ct.c_float),
        ("use_norm", ct.c_int), ("input_u8", ct.c_int), ("param_kind", ct.c_int), ("antisymmetric", ct.c_int),
        ("dtype", ct.c_int),
    ]


_P = ct.c_void_p
_I = ct.c_int
_L = ct.c_long
_F = ct.c_float
_S = ct.c_size_t

# (name, restype, argtypes) — exactly the declarations of include/asr.h
SIGNATURES = [
    ("asr_last_error", ct.c_char_p, []),
    ("asr_abi_version", _I, []),
    ("asr_device_cu_count", _I, []),
    ("asr_theta_count", _L, [_I, _I, _I]),
    ("asr_param_map", _I, [_I, _I, _I, _P, _P]),
    ("asr_param_is_antisymmetric", _I, [_I, _I]),
    ("asr_param_map_transpose", _I, [_I, _P, _P]),
    ("asr_param_map_pair", _I, [_I, _P, ct.c_long, _P]),
    ("asr_theta_count_k", _L, [_I, _I, _I, _I]),
    ("asr_param_map_k", _I, [_I, _I, _I, _I, _P, _P]),
    ("asr_param_map_transpose_k", _I, [_I, _I, _P, _P]),
    ("asr_theta_to_w_k", _I, [_P, _L, _I, _I, _I, _P, _F, _P, _L, _P]),
    ("asr_conv_forward_k", _I, [_I, _I, _P, _P, _P, _P, _P, _F, _I, _I, _I, _I, _P]),
    ("asr_conv_backward_workspace_bytes_k", _S, [_I, _I, _I, _I, _I]),
    ("asr_conv_backward_k", _I, [_I, _I, _P, _P, _P, _P, _P, _L, _F, _F, _I, _I, _I, _I, _P, _P, _P, _P, _P, _S, _P]),
    ("asr_wpack_elems", _L, [_I]),
    ("asr_theta_to_w", _I, [_P, _L, _I, _I, _P, _F, _P, _L, _I, _P]),
    ("asr_conv_forward", _I, [_I, _P, _P, _P, _P, _P, _F, _I, _I, _I, _I, _I, _P]),
    ("asr_mask_bytes", _L, [_I, _I, _I, _I]),
    ("asr_block_stack_forward", _I, [_P, _P, _L, _P, _L, _P, _L, _P, _L, _F, _I, _I, _I, _I, _I, _I, _I, _P]),
    ("asr_block_stack_backward_workspace_bytes", _S, [_I, _I, _I, _I, _I, _I]),
    ("asr_block_stack_backward", _I, [_P, _P, _L, _P, _L, _P, _L, _P, _L, _F, _F, _I, _I, _I, _I, _I, _I, _P, _P, _P,
                                      _S, _P]),
    ("asr_conv_backward_workspace_bytes", _S, [_I, _I, _I, _I, _I]),
    ("asr_conv_backward", _I, [_I, _P, _P, _P, _P, _P, _L, _F, _F, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _S, _P]),
    ("asr_rk2_forward", _I, [_P, _P, _P, _P, _P, _P, _P, _F, _I, _I, _I, _I, _I, _P]),
    ("asr_rk2_backward_workspace_bytes", _S, [_I, _I, _I, _I, _I]),
    ("asr_rk2_backward", _I, [_P, _P, _P, _P, _P, _P, _P, _L, _F, _F, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _S,
                              _P]),
    ("asr_net_param_count", _L, [ct.POINTER(NetConfig)]),
    ("asr_net_workspace_bytes", _S, [ct.POINTER(NetConfig)]),
    ("asr_net_prepare", _I, [ct.POINTER(NetConfig), _P, _S]),
    ("asr_net_forward", _I, [ct.POINTER(NetConfig), _P, _P, _P, _P, _S, _P]),
    ("asr_net_forward_backward", _I, [ct.POINTER(NetConfig), _P, _P, _P, _P, _P, _P, _P, _S, _P]),
    ("asr_net_check_status", _I, [ct.POINTER(NetConfig), _P, _S, _P]),
    ("asr_net_kernel_times", _I, [_P]),
    ("asr_stack_status", _I, [_I]),
    ("asr_debug_stack_backward", _I, [_I]),
    ("asr_rk2_stack_forward", _I, [_P, _P, _P, _L, _P, _P, _L, _P, _L, _P, _L, _F, _I, _I, _I, _I, _I, _I, _P]),
    ("asr_rk2_stack_backward_workspace_bytes", _S, [_I, _I, _I, _I, _I, _I]),
    ("asr_rk2_stack_backward", _I, [_P, _P, _P, _L, _P, _P, _L, _P, _L, _P, _L, _F, _F, _I, _I, _I, _I, _I, _I, _P,
                                    _P, _P, _S, _P]),
    ("asr_transition_forward", _I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    ("asr_transition_backward_workspace_bytes", _S, [_I, _I, _I, _I, _I, _I]),
    ("asr_transition_backward", _I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _S, _P]),
    ("asr_stages_check", ct.c_int, [ct.POINTER(StagesConfig)]),
    ("asr_stages_param_count", _L, [ct.POINTER(StagesConfig)]),
    ("asr_stages_workspace_bytes", _S, [ct.POINTER(StagesConfig)]),
    ("asr_stages_prepare", _I, [ct.POINTER(StagesConfig), _P, _S]),
    ("asr_stages_forward", _I, [ct.POINTER(StagesConfig), _P, _P, _P, _P, _S, _P]),
    ("asr_stages_forward_backward", _I, [ct.POINTER(StagesConfig), _P, _P, _P, _P, _P, _P, _P, _S, _P]),
    ("asr_adam_update", _I, [_P, _P, _P, _P, _L, _F, _F, _F, _F, _L, _F, _P]),
    ("asr_segment_sq_norms", _I, [_P, _P, _I, _P, _P]),
    ("asr_batch_metrics", _I, [_P, _P, _P, _I, _I, _P, _P]),
    ("asr_dist_unique_id", _I, [_P]),
    ("asr_dist_init", _I, [_I, _I, _P]),
    ("asr_dist_allreduce_sum", _I, [_P, _S, _I, _P]),
    ("asr_dist_broadcast", _I, [_P, _S, _I, _I, _P]),
    ("asr_dist_world_size", _I, []),
    ("asr_dist_finalize", _I, []),
]

_lib = None


def lib_path() -> str:
    return _build.LIB


def load(build_if_missing: bool = True, path: str | None = None):
    """Load (building first if needed) libasr.so and bind its C ABI.

    `path` (development tools only: A/B timing of variant builds) loads
    another build of the same sources; it must be given before the first
    load of the process."""
    global _lib
    if _lib is not None:
        if path is not None and getattr(_lib, "_asr_path", None) != path:
            raise AsrError(f"libasr already loaded from {_lib._asr_path}")
        return _lib
    path = path or _build.LIB
    if not os.path.exists(path):
        if not build_if_missing:
            raise AsrError(f"libasr.so not found at {path}; run differential_equations_resnet_amd._build.build()")
        _build.build()
    lib = ct.CDLL(path, mode=ct.RTLD_GLOBAL)
    lib._asr_path = path
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().asr_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = "") -> None:
    if rc == ASR_OK:
        return
    msg = f"{what}: {last_error()} (code {rc})"
    if rc == ASR_E_UNSUPPORTED:
        raise AsrUnsupported(msg)
    if rc == ASR_E_ARG:
        raise ValueError(msg)
    raise AsrError(msg)


def call(name: str, *args):
    rc = getattr(load(), name)(*args)
    check(rc, name)
    return rc
