"""Drop-in for layers/tfkeras_layer_Conv2DAntisymmetric3By3.py: a 3x3 conv
layer whose convolution matrix is antisymmetric (plus gamma on the diagonal).

Same constructor (…3By3.py:60-83), the same weights in the same order and
shapes — a, b, c, d [1,1,1,C] (:219-245), input_kernels_for_output_kernel_{o}
[3,3,C-o-1] for o = 0..C-2 (:113-124), bias [C] (:147-153) — the same
initialiser (truncated normal, stddev sqrt(2/(9C)), :95-98), get_kernel /
get_bias / get_config / compute_output_shape (:173-208).  Instead of the
per-output-channel slice/neg/concat/stack graph, W(theta) is one gather over
a precomputed element map on the device, and the conv runs in the native
kernels (libasr, include/asr.h)."""
from __future__ import annotations

from .. import _lib
from ._antisymmetric import AntisymmetricConvBase


class Conv2DAntisymmetric3By3(AntisymmetricConvBase):
    param_kind = _lib.ASR_PARAM_3BY3
    kernel_size = 3
    antisymmetric = True

    def __init__(self, gamma=0.0, strides=(1, 1), use_bias=True, kernel_initializer="he_normal",
                 kernel_regularizer=None, **kwargs):
        super().__init__(gamma=gamma, strides=strides, use_bias=use_bias, kernel_initializer=kernel_initializer,
                         kernel_regularizer=kernel_regularizer, **kwargs)

    def build(self, input_shape):
        # C_out == C_in: antisymmetry of the conv matrix needs a square operator
        self.num_channels = int(input_shape[-1])
        C = self.num_channels
        # the diagonal blocks' four free values, then the off-diagonal blocks
        self.a, self.b, self.c, self.d = (self._add_theta(n, (1, 1, 1, C)) for n in "abcd")
        self.independent_kernels = [self._add_theta(f"input_kernels_for_output_kernel_{o}", (3, 3, C - o - 1))
                                    for o in range(C - 1)]
        self._add_bias()
        self.built = True
