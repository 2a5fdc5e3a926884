"""Typed Python wrappers over the C ABI, with PyTorch-ROCm tensors used only as
device-memory containers (data_ptr) and for the current HIP stream.

Every function here launches libasr kernels; none computes anything in torch.
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import (ASR_BF16, ASR_F32, ASR_INTEGRATOR_EULER, ASR_INTEGRATOR_RK2, ASR_MODE_CONV, ASR_MODE_EULER,
                   ASR_PARAM_3BY3, ASR_PARAM_GENERAL, ASR_PARAM_REGULAR, ASR_VARIANT_NO_FOLD, ASR_VARIANT_STEM_FWD_VALU,
                   ASR_VARIANT_STEM_WGRAD_VALU, ASR_VARIANT_PER_BLOCK_FWD,
                   ASR_VARIANT_PER_BLOCK_BWD, ASR_VARIANT_INFERENCE, ASR_VARIANT_TIMED, ASR_VARIANT_FULL_DXL,
                   ASR_VARIANT_FULL_SLABS, ASR_VARIANT_W_BF16, NetConfig, StagesConfig)

__all__ = [
    "require_gpu", "dtype_code", "torch_dtype", "ParamMap", "param_map", "theta_count", "theta_to_w",
    "conv_forward", "block_stack_forward", "block_stack_backward", "conv_backward", "rk2_forward", "rk2_backward",
    "integrator_code", "NetExecutor", "adam_update", "stack_status", "transition_forward", "transition_backward",
    "StagesExecutor",
]


def stack_status(reset: bool = False) -> int:
    """Blocking: how many in-launch slab hand-offs of the C=64 stacked
    backward degraded since the last reset (asr_stack_status): a workgroup's
    bounded wait for the other workgroups' slabs ran out, so the flagged
    blocks were reduced after the launch instead: slower, the same gradients.
    reset clears the count after reading it."""
    rc = int(_lib.load().asr_stack_status(int(bool(reset))))
    if rc < 0:
        _lib.check(rc, "asr_stack_status")
    return rc


def integrator_code(integrator) -> int:
    if integrator in ("euler", ASR_INTEGRATOR_EULER, None):
        return ASR_INTEGRATOR_EULER
    if integrator in ("rk2", "midpoint", ASR_INTEGRATOR_RK2):
        return ASR_INTEGRATOR_RK2
    raise ValueError(f"unknown integrator {integrator!r} ('euler' or 'rk2')")


def require_gpu() -> torch.device:
    if not torch.cuda.is_available():
        raise _lib.AsrError("a gfx950 (MI355X) HIP device is required: libasr has no CPU path")
    _lib.load()
    return torch.device("cuda", torch.cuda.current_device())


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def dtype_code(dtype) -> int:
    if dtype in (torch.float32, "float32", np.float32, ASR_F32):
        return ASR_F32
    if dtype in (torch.bfloat16, "bfloat16", "bf16", ASR_BF16):
        return ASR_BF16
    raise ValueError(f"unsupported activation dtype {dtype!r} (float32 or bfloat16)")


def torch_dtype(code: int):
    return torch.float32 if code == ASR_F32 else torch.bfloat16


def theta_count(C: int, kind: int = ASR_PARAM_3BY3, antisymmetric: bool = True, k: int = 3) -> int:
    n = _lib.load().asr_theta_count_k(C, k, kind, int(antisymmetric))
    if n < 0:
        raise ValueError(f"bad theta_count arguments C={C} kind={kind} kernel_size={k}")
    return int(n)


@dataclass
class ParamMap:
    C: int
    kind: int
    antisymmetric: bool
    w_src: np.ndarray      # int32 [k*k*C*C]
    theta_dst: np.ndarray  # int32 [2*n_theta]
    _dev: dict
    k: int = 3             # kernel_size

    @property
    def operator_antisymmetric(self) -> bool:
        return bool(_lib.load().asr_param_is_antisymmetric(self.kind, int(self.antisymmetric)))

    def w_src_bwd(self, device):
        """Device map of W_bwd = -flip(W)^T (asr_param_map_transpose), for
        parametrisations whose operator is not antisymmetric."""
        key = ("bwd", str(device))
        if key not in self._dev:
            wb = np.empty_like(self.w_src)
            _lib.call("asr_param_map_transpose_k", self.C, self.k, self.w_src.ctypes.data, wb.ctypes.data)
            self._dev[key] = torch.from_numpy(wb).to(device)
        return self._dev[key]

    @property
    def n_theta(self) -> int:
        return self.theta_dst.size // 2

    def device(self, device) -> tuple:
        key = str(device)
        if key not in self._dev:
            self._dev[key] = (torch.from_numpy(self.w_src).to(device), torch.from_numpy(self.theta_dst).to(device))
        return self._dev[key]


_MAPS: dict = {}


def param_map(C: int, kind: int = ASR_PARAM_3BY3, antisymmetric: bool = True, k: int = 3) -> ParamMap:
    """Element map of W(theta) and its pull-back (asr_param_map_k, host)."""
    key = (C, kind, bool(antisymmetric), int(k))
    if key not in _MAPS:
        nt = theta_count(C, kind, antisymmetric, k)
        w_src = np.empty(k * k * C * C, dtype=np.int32)
        dst = np.empty(2 * nt, dtype=np.int32)
        _lib.call("asr_param_map_k", C, k, kind, int(antisymmetric), w_src.ctypes.data, dst.ctypes.data)
        _MAPS[key] = ParamMap(C, kind, bool(antisymmetric), w_src, dst, {}, int(k))
    return _MAPS[key]


def wpack_elems(C: int) -> int:
    n = _lib.load().asr_wpack_elems(C)
    if n < 0:
        raise _lib.AsrUnsupported(f"bf16 packed W needs C % 16 == 0 (C={C})")
    return int(n)


def theta_to_w(theta: torch.Tensor, C: int, pmap: ParamMap, gamma: float, dtype: int, layers: int = 1,
               theta_stride: int | None = None) -> torch.Tensor:
    """Materialise W for `layers` layers whose thetas are theta_stride floats
    apart.  bf16 -> MFMA-packed layout, f32 -> HWIO [layers, k, k, C, C]."""
    dev = theta.device
    w_src, _ = pmap.device(dev)
    stride = pmap.n_theta if theta_stride is None else theta_stride
    if pmap.k != 3:  # Conv2DAntisymmetric(kernel_size != 3): fp32 HWIO only
        if dtype != ASR_F32:
            raise _lib.AsrUnsupported(f"kernel_size {pmap.k}: the k x k kernels are fp32")
        per = pmap.k * pmap.k * C * C
        out = torch.empty(layers * per, dtype=torch.float32, device=dev)
        _lib.call("asr_theta_to_w_k", _p(theta), stride, layers, C, pmap.k, _p(w_src), float(gamma), _p(out), per,
                  _stream())
        return out.view(layers, pmap.k, pmap.k, C, C)
    if dtype == ASR_BF16:
        per = wpack_elems(C)
        out = torch.empty(layers * per, dtype=torch.bfloat16, device=dev)
    else:
        per = 9 * C * C
        out = torch.empty(layers * per, dtype=torch.float32, device=dev)
    _lib.call("asr_theta_to_w", _p(theta), stride, layers, C, _p(w_src), float(gamma), _p(out), per, dtype, _stream())
    if dtype == ASR_F32:
        return out.view(layers, 3, 3, C, C)
    return out.view(layers, per)


def theta_to_w_transposed(theta: torch.Tensor, C: int, pmap: ParamMap, dtype: int) -> torch.Tensor:
    """W_bwd = -flip(W)^T for the backward of a non-antisymmetric operator
    (pass it to conv_backward with gamma 0)."""
    dev = theta.device
    wb = pmap.w_src_bwd(dev)
    if pmap.k != 3:
        if dtype != ASR_F32:
            raise _lib.AsrUnsupported(f"kernel_size {pmap.k}: the k x k kernels are fp32")
        per = pmap.k * pmap.k * C * C
        out = torch.empty(per, dtype=torch.float32, device=dev)
        _lib.call("asr_theta_to_w_k", _p(theta), pmap.n_theta, 1, C, pmap.k, _p(wb), 0.0, _p(out), per, _stream())
        return out.view(1, pmap.k, pmap.k, C, C)
    if dtype == ASR_BF16:
        per = wpack_elems(C)
        out = torch.empty(per, dtype=torch.bfloat16, device=dev)
    else:
        per = 9 * C * C
        out = torch.empty(per, dtype=torch.float32, device=dev)
    _lib.call("asr_theta_to_w", _p(theta), pmap.n_theta, 1, C, _p(wb), 0.0, _p(out), per, dtype, _stream())
    return out.view(1, 3, 3, C, C) if dtype == ASR_F32 else out.view(1, per)


def segment_sq_norms(x: torch.Tensor, offsets: torch.Tensor) -> torch.Tensor:
    """out[i] = sum(x[offsets[i]:offsets[i+1]]**2) (asr_segment_sq_norms)."""
    n = offsets.numel() - 1
    out = torch.empty(n, dtype=torch.float32, device=x.device)
    _lib.call("asr_segment_sq_norms", _p(x), _p(offsets), n, _p(out), _stream())
    return out


def batch_metrics(probs, targets, loss, accum):
    """Streaming loss/accuracy accumulation (asr_batch_metrics): probs and
    targets are contiguous float32 device [N, K]; loss a device float or None."""
    N, K = probs.shape
    for name, t in (("probs", probs), ("targets", targets), ("accum", accum)) + ((("loss", loss),) if loss is not None
                                                                                  else ()):
        if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError(f"batch_metrics: {name} must be a contiguous float32 device tensor")
    if tuple(targets.shape) != (N, K) or accum.numel() < 4:
        raise ValueError(f"batch_metrics: targets must be [{N}, {K}] and accum hold 4 floats")
    _lib.call("asr_batch_metrics", _p(probs), _p(targets), _p(loss), N, K, _p(accum), _stream())


def conv_forward(mode: int, x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, h: float = 1.0,
                 mask: torch.Tensor | None = None, k: int = 3) -> torch.Tensor:
    N, H, W, C = x.shape
    dt = dtype_code(x.dtype)
    if not x.is_contiguous():
        raise ValueError("x must be contiguous NHWC")
    y = torch.empty_like(x)
    if k != 3:
        if dt != ASR_F32:
            raise _lib.AsrUnsupported(f"kernel_size {k}: the k x k kernels are fp32")
        _lib.call("asr_conv_forward_k", mode, k, _p(x), _p(y), _p(mask), _p(w), _p(bias), float(h), N, H, W, C,
                  _stream())
        return y
    _lib.call("asr_conv_forward", mode, _p(x), _p(y), _p(mask), _p(w), _p(bias), float(h), N, H, W, C, dt, _stream())
    return y


def block_stack_forward(x0: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, h: float, store_all=True,
                        want_masks=True):
    """L Euler blocks (asr_block_stack_forward).  w: [L, per-layer W] as
    theta_to_w(..., layers=L) returns; bias: [L, C] float32 or None.
    Returns (ys [L,N,H,W,C] with ys[l] = x_{l+1}, masks [L, mask_bytes]) or,
    with store_all=False, (x_L, None)."""
    N, H, W, C = x0.shape
    dt = dtype_code(x0.dtype)
    L = int(w.shape[0])
    if not x0.is_contiguous():
        raise ValueError("x0 must be contiguous NHWC")
    P = N * H * W * C
    ys = torch.empty((L if store_all else 1, N, H, W, C), dtype=x0.dtype, device=x0.device)
    mb = mask_bytes(N, H, W, C)
    masks = torch.zeros(L, mb, dtype=torch.uint8, device=x0.device) if (want_masks and store_all) else None
    if bias is not None and (tuple(bias.shape) != (L, C) or bias.dtype != torch.float32 or not bias.is_contiguous()):
        raise ValueError(f"bias must be contiguous float32 [{L}, {C}]")
    per = w[0].numel()
    _lib.call("asr_block_stack_forward", _p(x0), _p(ys), P, _p(masks), mb, _p(w), per, _p(bias), C, float(h), N, H, W,
              C, L, dt, int(bool(store_all)), _stream())
    return (ys, masks) if store_all else (ys[0], None)


def block_stack_backward(dyL, x0, ys, masks, w, pmap: ParamMap, h: float, gamma: float, want_dparams=True):
    """Backward of block_stack_forward (asr_block_stack_backward): returns
    (dx0, dparams [L, n_theta + C] or None).  The inputs of the L blocks are
    x0, ys[0], ..., ys[L-2]; they are passed as one [L, N, H, W, C] stack."""
    L = int(w.shape[0])
    N, H, W, C = x0.shape
    dt = dtype_code(x0.dtype)
    xs = torch.cat([x0.unsqueeze(0), ys[:L - 1]]) if L > 1 else x0.unsqueeze(0)
    xs = xs.contiguous()
    P = N * H * W * C
    mb = mask_bytes(N, H, W, C)
    wsb = int(_lib.load().asr_block_stack_backward_workspace_bytes(N, H, W, C, L, dt))
    ws = torch.empty(wsb, dtype=torch.uint8, device=x0.device)
    dx0 = torch.empty_like(x0)
    dparams = torch.empty(L, pmap.n_theta + C, dtype=torch.float32, device=x0.device) if want_dparams else None
    _, theta_dst = pmap.device(x0.device)
    _lib.call("asr_block_stack_backward", _p(dyL), _p(xs), P, _p(masks), mb, _p(w), w[0].numel(), _p(theta_dst),
              pmap.n_theta, float(h), float(gamma), N, H, W, C, L, dt, _p(dx0), _p(dparams), _p(ws), wsb, _stream())
    return dx0, dparams


def mask_bytes(N: int, H: int, W: int, C: int) -> int:
    return int(_lib.load().asr_mask_bytes(N, H, W, C))


def conv_backward(mode: int, dy: torch.Tensor, x: torch.Tensor, mask: torch.Tensor | None, w: torch.Tensor,
                  pmap: ParamMap, h: float, gamma: float, want_dx=True, want_dtheta=True, want_dbias=True,
                  want_dw=False):
    N, H, W, C = dy.shape
    dt = dtype_code(dy.dtype)
    dev = dy.device
    k = pmap.k
    if k != 3 and dt != ASR_F32:
        raise _lib.AsrUnsupported(f"kernel_size {k}: the k x k kernels are fp32")
    if k != 3:
        ws_bytes = int(_lib.load().asr_conv_backward_workspace_bytes_k(N, H, W, C, k))
    else:
        ws_bytes = int(_lib.load().asr_conv_backward_workspace_bytes(N, H, W, C, dt))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    dx = torch.empty_like(dy) if want_dx else None
    dth = torch.empty(pmap.n_theta, dtype=torch.float32, device=dev) if want_dtheta else None
    db = torch.empty(C, dtype=torch.float32, device=dev) if want_dbias else None
    dw = torch.empty(k, k, C, C, dtype=torch.float32, device=dev) if want_dw else None
    _, theta_dst = pmap.device(dev)
    if k != 3:
        _lib.call("asr_conv_backward_k", mode, k, _p(dy), _p(x), _p(mask), _p(w), _p(theta_dst), pmap.n_theta,
                  float(h), float(gamma), N, H, W, C, _p(dx), _p(dth), _p(db), _p(dw), _p(ws), ws_bytes, _stream())
        return dx, dth, db, dw
    _lib.call("asr_conv_backward", mode, _p(dy), _p(x), _p(mask), _p(w), _p(theta_dst), pmap.n_theta, float(h),
              float(gamma), N, H, W, C, dt, _p(dx), _p(dth), _p(db), _p(dw), _p(ws), ws_bytes, _stream())
    return dx, dth, db, dw


def rk2_forward(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, h: float, want_masks=True):
    """RK2 midpoint block (asr_rk2_forward): returns (y, xmid, mask1, mask2)."""
    N, H, W, C = x.shape
    dt = dtype_code(x.dtype)
    if not x.is_contiguous():
        raise ValueError("x must be contiguous NHWC")
    y = torch.empty_like(x)
    xm = torch.empty_like(x)
    mb = mask_bytes(N, H, W, C)
    m1 = torch.zeros(mb, dtype=torch.uint8, device=x.device) if want_masks else None
    m2 = torch.zeros(mb, dtype=torch.uint8, device=x.device) if want_masks else None
    _lib.call("asr_rk2_forward", _p(x), _p(xm), _p(y), _p(m1), _p(m2), _p(w), _p(bias), float(h), N, H, W, C, dt,
              _stream())
    return y, xm, m1, m2


def rk2_backward(dy, x, xmid, mask1, mask2, w, pmap: ParamMap, h: float, gamma: float, want_dx=True,
                 want_dtheta=True, want_dbias=True, want_dw=False):
    """Backward of rk2_forward (asr_rk2_backward): (dx, dtheta, dbias, dw)."""
    N, H, W, C = dy.shape
    dt = dtype_code(dy.dtype)
    dev = dy.device
    ws_bytes = int(_lib.load().asr_rk2_backward_workspace_bytes(N, H, W, C, dt))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    dx = torch.empty_like(dy) if want_dx else None
    dth = torch.empty(pmap.n_theta, dtype=torch.float32, device=dev) if want_dtheta else None
    db = torch.empty(C, dtype=torch.float32, device=dev) if want_dbias else None
    dw = torch.empty(3, 3, C, C, dtype=torch.float32, device=dev) if want_dw else None
    _, theta_dst = pmap.device(dev)
    _lib.call("asr_rk2_backward", _p(dy), _p(x), _p(xmid), _p(mask1), _p(mask2), _p(w), _p(theta_dst), pmap.n_theta,
              float(h), float(gamma), N, H, W, C, dt, _p(dx), _p(dth), _p(db), _p(dw), _p(ws), ws_bytes, _stream())
    return dx, dth, db, dw


def rk2_stack_forward(x0: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, h: float):
    """L RK2 blocks in one call (asr_rk2_stack_forward; bf16, C=64): returns
    (ys [L,N,H,W,C] with ys[l] = x_{l+1}, xmids [L,N,H,W,C], masks1, masks2 [L, mask_bytes])."""
    N, H, W, C = x0.shape
    L = int(w.shape[0])
    if not x0.is_contiguous():
        raise ValueError("x0 must be contiguous NHWC")
    P = N * H * W * C
    ys = torch.empty((L, N, H, W, C), dtype=x0.dtype, device=x0.device)
    xm = torch.empty_like(ys)
    mb = mask_bytes(N, H, W, C)
    m1 = torch.zeros(L, mb, dtype=torch.uint8, device=x0.device)
    m2 = torch.zeros(L, mb, dtype=torch.uint8, device=x0.device)
    if bias is not None and (tuple(bias.shape) != (L, C) or bias.dtype != torch.float32 or not bias.is_contiguous()):
        raise ValueError(f"bias must be contiguous float32 [{L}, {C}]")
    _lib.call("asr_rk2_stack_forward", _p(x0), _p(ys), _p(xm), P, _p(m1), _p(m2), mb, _p(w), w[0].numel(), _p(bias),
              C, float(h), N, H, W, C, L, dtype_code(x0.dtype), _stream())
    return ys, xm, m1, m2


def rk2_stack_backward(dyL, x0, ys, xmids, masks1, masks2, w, pmap: ParamMap, h: float, gamma: float):
    """Backward of rk2_stack_forward (asr_rk2_stack_backward): (dx0, dparams [L, n_theta + C])."""
    L = int(w.shape[0])
    N, H, W, C = x0.shape
    dt = dtype_code(x0.dtype)
    xs = (torch.cat([x0.unsqueeze(0), ys[:L - 1]]) if L > 1 else x0.unsqueeze(0)).contiguous()
    P = N * H * W * C
    mb = mask_bytes(N, H, W, C)
    wsb = int(_lib.load().asr_rk2_stack_backward_workspace_bytes(N, H, W, C, L, dt))
    ws = torch.empty(wsb, dtype=torch.uint8, device=x0.device)
    dx0 = torch.empty_like(x0)
    dparams = torch.empty(L, pmap.n_theta + C, dtype=torch.float32, device=x0.device)
    _, theta_dst = pmap.device(x0.device)
    _lib.call("asr_rk2_stack_backward", _p(dyL), _p(xs), _p(xmids), P, _p(masks1), _p(masks2), mb, _p(w),
              w[0].numel(), _p(theta_dst), pmap.n_theta, float(h), float(gamma), N, H, W, C, L, dt, _p(dx0),
              _p(dparams), _p(ws), wsb, _stream())
    return dx0, dparams


def adam_update(params, grads, m, v, lr, beta1, beta2, eps, step, grad_scale=1.0):
    _lib.call("asr_adam_update", _p(params), _p(grads), _p(m), _p(v), params.numel(), float(lr), float(beta1),
              float(beta2), float(eps), int(step), float(grad_scale), _stream())


class NetExecutor:
    """Native executor of the single-block antisymmetric ResNet
    (asr_net_* in include/asr.h).  Owns the device workspace; parameters,
    gradients and Adam moments are flat float32 buffers in Keras
    get_weights() order.  inference=True builds the forward-only workspace
    (ASR_VARIANT_INFERENCE: x_0 and two ping-pong activation slots)."""

    def __init__(self, N, H, W, Cin, C, L, num_classes, h, gamma=0.0, subtract_mean=None, divide_by_stddev=None,
                 dtype="bfloat16", input_u8=True, device=None, param_kind=ASR_PARAM_3BY3, antisymmetric=True,
                 integrator="euler", variant=0, inference=False):
        if inference:
            variant |= ASR_VARIANT_INFERENCE
        self.device = torch.device(device) if device is not None else require_gpu()
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        use_norm = subtract_mean is not None or divide_by_stddev is not None
        self.cfg = NetConfig(int(N), int(H), int(W), int(Cin), int(C), int(L), int(num_classes), float(h),
                             float(gamma), float(subtract_mean or 0.0),
                             float(divide_by_stddev if divide_by_stddev is not None else 1.0), int(use_norm),
                             dtype_code(dtype), int(bool(input_u8)), int(param_kind), int(bool(antisymmetric)),
                             integrator_code(integrator), int(variant))
        lib = _lib.load()
        with torch.cuda.device(self.device):  # the layout (slab rows) follows the device's CU count
            self.n_params = int(lib.asr_net_param_count(ct.byref(self.cfg)))
            if self.n_params < 0:
                _lib.check(_lib.ASR_E_ARG, "asr_net_param_count")
            self.ws_bytes = int(lib.asr_net_workspace_bytes(ct.byref(self.cfg)))
            if self.ws_bytes == 0:
                _lib.check(_lib.ASR_E_ARG, "asr_net_workspace_bytes")
            self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)
            _lib.call("asr_net_prepare", ct.byref(self.cfg), _p(self.ws), self.ws_bytes)
        self.inference = bool(inference)
        self.grads = None if inference else torch.zeros(self.n_params, dtype=torch.float32, device=self.device)
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.probs = torch.zeros(N, num_classes, dtype=torch.float32, device=self.device)

    def _check_inputs(self, params, images):
        c = self.cfg
        if params.numel() != self.n_params or params.dtype != torch.float32 or not params.is_cuda:
            raise ValueError(f"params must be a float32 device buffer of {self.n_params} elements")
        want = torch.uint8 if c.input_u8 else torch.float32
        if tuple(images.shape) != (c.N, c.H, c.W, c.Cin) or images.dtype != want or not images.is_contiguous():
            raise ValueError(f"images must be contiguous {want} [{c.N},{c.H},{c.W},{c.Cin}] (NHWC)")

    def forward(self, params, images) -> torch.Tensor:
        self._check_inputs(params, images)
        with torch.cuda.device(self.device):
            _lib.call("asr_net_forward", ct.byref(self.cfg), _p(params), _p(images), _p(self.probs), _p(self.ws),
                      self.ws_bytes, _stream())
        return self.probs

    @property
    def variant(self) -> int:
        return int(self.cfg.variant)

    @variant.setter
    def variant(self, bits: int):
        """Select ASR_VARIANT_* kernel compositions (tests) or the timing
        instrumentation for later calls; an inference executor keeps its
        ASR_VARIANT_INFERENCE bit (its workspace layout)."""
        self.cfg.variant = int(bits) | (ASR_VARIANT_INFERENCE if self.inference else 0)

    def check_status(self):
        """Blocking: synchronises the stream and raises AsrError when a launch
        failed (asr_net_check_status).  A degraded slab hand-off is not an
        error (it costs speed): see stack_status."""
        with torch.cuda.device(self.device):
            _lib.call("asr_net_check_status", ct.byref(self.cfg), _p(self.ws), self.ws_bytes, _stream())

    @staticmethod
    def kernel_times() -> dict:
        """Blocking: device microseconds of the block launches of the last
        call made with ASR_VARIANT_TIMED (asr_net_kernel_times): "fwd" the
        blocks' forward, "bwd" the blocks' backward kernels (the one stack
        launch where one runs), "bwd_reduce" the weight-gradient reductions
        left after them + the projection (None where that call ran no such
        part)."""
        out = (ct.c_float * 3)()
        _lib.call("asr_net_kernel_times", ct.cast(out, ct.c_void_p))
        return {k: (float(v) if v >= 0 else None) for k, v in zip(("fwd", "bwd", "bwd_reduce"), out)}

    def forward_backward(self, params, images, targets, want_probs=False):
        if self.inference:
            raise ValueError("an inference executor has no backward")
        self._check_inputs(params, images)
        if tuple(targets.shape) != (self.cfg.N, self.cfg.num_classes) or targets.dtype != torch.float32:
            raise ValueError("targets must be float32 one-hot [N, num_classes]")
        with torch.cuda.device(self.device):
            _lib.call("asr_net_forward_backward", ct.byref(self.cfg), _p(params), _p(images), _p(targets),
                      _p(self.grads), _p(self.loss), _p(self.probs) if want_probs else None, _p(self.ws),
                      self.ws_bytes, _stream())
        return self.loss, self.grads


def transition_forward(x: torch.Tensor, k2, b2, k1, b1, stride: int):
    """single_layer_conv_block (tfkeras_resnets.py:204-269) on fp32 NHWC x:
    (y, mask) with y = relu(conv3x3_same(x, k2, stride) + b2) + conv1x1(x, k1,
    stride) + b1 and mask = [conv3x3 + b2 > 0] (asr_transition_forward)."""
    N, H, W, Ci = x.shape
    Co = int(k2.shape[-1])
    Ho, Wo = -(-H // stride), -(-W // stride)
    y = torch.empty((N, Ho, Wo, Co), dtype=torch.float32, device=x.device)
    mask = torch.empty((N, Ho, Wo, Co), dtype=torch.uint8, device=x.device)
    _lib.call("asr_transition_forward", _p(x), _p(y), _p(mask), _p(k2), _p(b2), _p(k1), _p(b1), N, H, W, Ci, Co,
              int(stride), _stream())
    return y, mask


def transition_backward(dy, x, mask, k2, k1, stride: int, want_dx=True, want_dparams=True):
    """Backward of transition_forward: (dx, dparams) with dparams =
    [dK2 | db2 | dK1 | db1] flat (asr_transition_backward)."""
    N, H, W, Ci = x.shape
    Co = int(k2.shape[-1])
    dx = torch.empty_like(x) if want_dx else None
    dparams = torch.empty(9 * Ci * Co + Co + Ci * Co + Co, dtype=torch.float32, device=x.device) if want_dparams else None
    nb = int(_lib.load().asr_transition_backward_workspace_bytes(N, H, W, Ci, Co, int(stride)))
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=x.device)
    _lib.call("asr_transition_backward", _p(dy), _p(x), _p(mask), _p(k2), _p(k1), N, H, W, Ci, Co, int(stride),
              _p(dx), _p(dparams), _p(ws), nb, _stream())
    return dx, dparams


class StagesExecutor:
    """Native executor of the multi-stage single-block ResNet (asr_stages_*
    in include/asr.h): stem, per stage an optional transition
    (single_layer_conv_block) and its identity Euler blocks, head.  float32
    (the reference's precision) or bfloat16 (the identity blocks' activations
    and convs in bf16 with fp32 accumulation; stem, transitions, head and every
    weight gradient in fp32; stages with blocks need C in {16, 32, 64} and
    W in {32, 16, 8}).  Parameters / gradients are flat float32 buffers in the
    asr_stages_config order; same call surface as NetExecutor."""

    def __init__(self, N, H, W, Cin, stages, num_classes, h, gamma=0.0, subtract_mean=None, divide_by_stddev=None,
                 dtype="float32", input_u8=True, device=None, param_kind=ASR_PARAM_3BY3, antisymmetric=True,
                 inference=False):
        """stages: [(C, L, stride)] per stage, stride 0 for no transition."""
        if not 1 <= len(stages) <= _lib.ASR_STAGES_MAX:
            raise _lib.AsrUnsupported(f"{len(stages)} stages (1..{_lib.ASR_STAGES_MAX})")
        self.device = torch.device(device) if device is not None else require_gpu()
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        use_norm = subtract_mean is not None or divide_by_stddev is not None
        c = StagesConfig()
        c.N, c.H, c.W, c.Cin, c.num_classes, c.n_stages = int(N), int(H), int(W), int(Cin), int(num_classes), len(stages)
        for i, (C, L, S) in enumerate(stages):
            c.C[i], c.L[i], c.stride[i] = int(C), int(L), int(S)
        c.h, c.gamma = float(h), float(gamma)
        c.subtract_mean = float(subtract_mean or 0.0)
        c.divide_by_stddev = float(divide_by_stddev if divide_by_stddev is not None else 1.0)
        c.use_norm, c.input_u8 = int(use_norm), int(bool(input_u8))
        c.param_kind, c.antisymmetric = int(param_kind), int(bool(antisymmetric))
        c.dtype = dtype_code(dtype)
        self.cfg = c
        self.dtype = dtype
        self.stages = [tuple(int(v) for v in st) for st in stages]
        lib = _lib.load()
        _lib.call("asr_stages_check", ct.byref(c))
        with torch.cuda.device(self.device):  # the layout (slab rows) follows the device's CU count
            self.n_params = int(lib.asr_stages_param_count(ct.byref(c)))
            if self.n_params < 0:
                _lib.check(_lib.ASR_E_ARG, "asr_stages_param_count")
            self.ws_bytes = int(lib.asr_stages_workspace_bytes(ct.byref(c)))
            if self.ws_bytes == 0:
                _lib.check(_lib.ASR_E_ARG, "asr_stages_workspace_bytes")
            self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=self.device)
            _lib.call("asr_stages_prepare", ct.byref(c), _p(self.ws), self.ws_bytes)
        self.inference = bool(inference)
        self.grads = None if inference else torch.zeros(self.n_params, dtype=torch.float32, device=self.device)
        self.loss = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.probs = torch.zeros(N, num_classes, dtype=torch.float32, device=self.device)

    def _check_inputs(self, params, images):
        c = self.cfg
        if params.numel() != self.n_params or params.dtype != torch.float32 or not params.is_cuda:
            raise ValueError(f"params must be a float32 device buffer of {self.n_params} elements")
        want = torch.uint8 if c.input_u8 else torch.float32
        if tuple(images.shape) != (c.N, c.H, c.W, c.Cin) or images.dtype != want or not images.is_contiguous():
            raise ValueError(f"images must be contiguous {want} [{c.N},{c.H},{c.W},{c.Cin}] (NHWC)")

    def forward(self, params, images) -> torch.Tensor:
        self._check_inputs(params, images)
        with torch.cuda.device(self.device):
            _lib.call("asr_stages_forward", ct.byref(self.cfg), _p(params), _p(images), _p(self.probs), _p(self.ws),
                      self.ws_bytes, _stream())
        return self.probs

    def check_status(self):
        """Blocking: synchronises the stream (a failed launch raises there; the
        launches' own errors are raised by the calls that made them)."""
        torch.cuda.current_stream().synchronize()

    def forward_backward(self, params, images, targets, want_probs=False):
        if self.inference:
            raise ValueError("an inference executor has no backward")
        self._check_inputs(params, images)
        if tuple(targets.shape) != (self.cfg.N, self.cfg.num_classes) or targets.dtype != torch.float32:
            raise ValueError("targets must be float32 one-hot [N, num_classes]")
        with torch.cuda.device(self.device):
            _lib.call("asr_stages_forward_backward", ct.byref(self.cfg), _p(params), _p(images), _p(targets),
                      _p(self.grads), _p(self.loss), _p(self.probs) if want_probs else None, _p(self.ws),
                      self.ws_bytes, _stream())
        return self.loss, self.grads
