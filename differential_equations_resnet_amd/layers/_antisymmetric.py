"""Shared machinery of the two drop-in antisymmetric conv layers: weight
layout through the native parameter map, kernel readback, and the eager
device call (conv + bias through asr_conv_forward / asr_conv_backward, wired
into torch autograd so a layer can be used directly on device tensors).

The weights are created exactly as the reference's add_weight calls create
them (names, shapes, order, initialiser); see the two layer modules for the
file:line of each."""
from __future__ import annotations

import numpy as np

from .. import _lib
from ..graph import Layer

__all__ = ["AntisymmetricConvBase"]


def _torch():
    import torch
    return torch


class AntisymmetricConvBase(Layer):
    """Base of Conv2DAntisymmetric3By3 / Conv2DAntisymmetric.  Subclasses set
    `param_kind`, `antisymmetric`, `kernel_size` and create the theta
    variables in build()."""

    param_kind = _lib.ASR_PARAM_3BY3
    kernel_size = 3
    antisymmetric = True

    def __init__(self, gamma=0.0, strides=(1, 1), use_bias=True, kernel_initializer="he_normal",
                 kernel_regularizer=None, **kwargs):
        super().__init__(**kwargs)
        self.gamma = gamma
        self.strides = strides
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.kernel_regularizer = kernel_regularizer
        self.theta_vars = []
        self.bias = None
        self._dev = None  # (device, theta tensor, bias tensor) for eager calls

    # -- creation ------------------------------------------------------------
    def _theta_initializer(self):
        if self.kernel_initializer == "he_normal":
            # tf.initializers.truncated_normal(stddev=sqrt(2/(k*k*C))) (…3By3.py:95-98)
            return "antisymmetric_he_normal"
        return self.kernel_initializer

    def _add_theta(self, name, shape):
        v = self.add_weight(name, shape, self._theta_initializer(), self.kernel_regularizer,
                            kernel_size=self.kernel_size, channels=self.num_channels)
        self.theta_vars.append(v)
        return v

    def _add_bias(self):
        if self.use_bias:
            self.bias = self.add_weight("bias", (self.num_channels,), "zeros")

    def compute_output_shape(self, input_shape):
        # …3By3.py:173-175: the input shape, whatever the strides
        return input_shape

    # -- readback --------------------------------------------------------------
    def theta_flat(self) -> np.ndarray:
        return np.concatenate([v.value.ravel() for v in self.theta_vars]).astype(np.float32)

    def _check_native(self, dtype=None):
        k = self.kernel_size
        if k < 1 or k % 2 == 0 or k > 15:
            raise _lib.AsrUnsupported(f"{self.name}: kernel_size {k} (odd 1..15 have native kernels)")
        if k != 3 and dtype is not None and str(dtype) != "torch.float32":
            raise _lib.AsrUnsupported(f"{self.name}: kernel_size {k} runs the fp32 k x k kernels (input {dtype})")

    def param_map(self):
        from .. import runtime
        self._check_native()
        return runtime.param_map(self.num_channels, self.param_kind, self.antisymmetric, self.kernel_size)

    def get_kernel(self) -> np.ndarray:
        """The assembled kernel [k,k,C,C] (HWIO).  Reads theta through the
        native element map (asr_param_map, the same map the device
        materialisation consumes), so W here is bit-identical to the W the
        kernels run with (…3By3.py:188-199)."""
        pm = self.param_map()
        th = self.theta_flat()
        src = pm.w_src
        W = np.where(src >= 0, th[np.maximum(src, 0) >> 1] * np.where(src & 1, -1.0, 1.0), self.gamma)
        k = self.kernel_size
        return W.astype(np.float32).reshape(k, k, self.num_channels, self.num_channels)

    def get_bias(self) -> np.ndarray:
        if self.bias is None:
            raise ValueError(f"{self.name} was built with use_bias=False")
        return self.bias.value.copy()

    def get_config(self):
        c = super().get_config()
        # the reference's get_config omits gamma (…3By3.py:177-186)
        c.update({"strides": self.strides, "use_bias": self.use_bias,
                  "kernel_initializer": self.kernel_initializer, "kernel_regularizer": self.kernel_regularizer})
        return c

    # -- eager device execution --------------------------------------------------
    def _weights_changed(self):
        self._dev = None

    def device_variables(self, device):
        """(theta, bias) leaf device tensors (requires_grad) holding this
        layer's weights; gradients of eager calls accumulate in their .grad.
        Use sync_from_device() to write updated values back."""
        torch = _torch()
        if self._dev is None or self._dev[0] != device:
            th = torch.from_numpy(self.theta_flat()).to(device).requires_grad_(self.trainable)
            b = None
            if self.bias is not None:
                b = torch.from_numpy(self.bias.value.copy()).to(device).requires_grad_(self.trainable)
            self._dev = (device, th, b)
        return self._dev[1], self._dev[2]

    def sync_from_device(self):
        if self._dev is None:
            return
        _, th, b = self._dev
        flat = th.detach().float().cpu().numpy()
        off = 0
        for v in self.theta_vars:
            n = v.value.size
            v.assign(flat[off:off + n].reshape(v.shape))
            off += n
        if b is not None:
            self.bias.assign(b.detach().cpu().numpy())

    def call_device(self, x, **kwargs):
        """output = conv2d(x, W(theta), SAME, stride 1) + bias on a device NHWC
        tensor (float32 or bfloat16), i.e. the layer's call() (…3By3.py:157-171)."""
        torch = _torch()
        if not isinstance(x, torch.Tensor) or not x.is_cuda:
            raise TypeError(f"{self.name}: eager calls take a device (HIP) tensor; use a Model for host arrays")
        if tuple(self.strides) != (1, 1):
            raise _lib.AsrUnsupported(f"{self.name}: strides {self.strides} (native kernels are stride 1)")
        if x.dim() != 4 or x.shape[-1] != self.num_channels:
            raise ValueError(f"{self.name}: expected NHWC input with {self.num_channels} channels, got {tuple(x.shape)}")
        self._check_native(x.dtype)
        th, b = self.device_variables(x.device)
        return _AntisymConv2D.apply(x, th, b, self)


def _make_fn():
    torch = _torch()
    from .. import runtime

    class AntisymConv2D(torch.autograd.Function):
        """Forward: asr_theta_to_w + asr_conv_forward(MODE_CONV).
        Backward: asr_conv_backward(MODE_CONV): dx = A^T dy, dtheta (the
        projection of dW through the map), dbias."""

        @staticmethod
        def forward(ctx, x, theta, bias, layer):
            dt = runtime.dtype_code(x.dtype)
            pm = layer.param_map()
            C = layer.num_channels
            x = x.contiguous()
            w = runtime.theta_to_w(theta.detach(), C, pm, layer.gamma, dt)
            y = runtime.conv_forward(runtime.ASR_MODE_CONV, x, w, None if bias is None else bias.detach(), 1.0,
                                     k=pm.k)
            ctx.layer = layer
            ctx.has_bias = bias is not None
            ctx.save_for_backward(x, theta)
            ctx.w = w
            return y

        @staticmethod
        def backward(ctx, dy):
            x, theta = ctx.saved_tensors
            layer = ctx.layer
            pm = layer.param_map()
            dt = runtime.dtype_code(dy.dtype)
            if _lib.load().asr_param_is_antisymmetric(layer.param_kind, int(layer.antisymmetric)):
                w, gamma = ctx.w, layer.gamma  # A^T = -A + 2 gamma I, with the forward W
            else:
                w, gamma = runtime.theta_to_w_transposed(theta.detach(), layer.num_channels, pm, dt), 0.0
            need_dx, need_th, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2]
            dx, dth, db, _ = runtime.conv_backward(runtime.ASR_MODE_CONV, dy.contiguous().to(x.dtype), x, None, w, pm,
                                                   1.0, gamma, want_dx=need_dx, want_dtheta=need_th,
                                                   want_dbias=need_b and ctx.has_bias)
            return dx, dth, db, None

    return AntisymConv2D


class _Lazy:
    _fn = None

    @classmethod
    def apply(cls, *args):
        if cls._fn is None:
            cls._fn = _make_fn()
        return cls._fn.apply(*args)


_AntisymConv2D = _Lazy
