"""Drop-in for layers/tfkeras_layer_Conv2DAntisymmetric.py: the general
(anti-)centrosymmetric-diagonal layer.

Constructor as …Conv2DAntisymmetric.py:60-88 (kernel_size first,
antisymmetric flag).  Weights per output channel o, in creation order: the
centro_sym_{i}_{j} scalars [1,1,1,1] of its diagonal block (free positions
(0,0),(0,1),(0,2)[,(1,1) if not antisymmetric],(1,2); :227-264), then
input_kernels_for_output_kernel_{o} [k,k,C-o-1,1] (:123-128); bias [C] last
(:150-156).  Dependent off-diagonal blocks are -J K J (:139).  get_config
omits gamma like the reference (:181-192).

Every odd kernel_size (1..15) executes natively: 3 on the fp32 / bf16 kernels
of the network path, other sizes on the fp32 k x k kernels
(asr_conv_forward_k / asr_conv_backward_k, the reference's precision)."""
from __future__ import annotations

from .. import _lib
from ._antisymmetric import AntisymmetricConvBase


def _free_positions(k, antisymmetric):
    out = []
    for i in range(k):
        for j in range(i, k):
            if j > i or (j == i and i <= k // 2 - 1):
                out.append((i, j))
            elif j == i and i == k // 2 and k % 2 == 1 and not antisymmetric:
                out.append((i, j))
    return out


class Conv2DAntisymmetric(AntisymmetricConvBase):
    param_kind = _lib.ASR_PARAM_GENERAL

    def __init__(self, kernel_size, gamma=0.0, strides=(1, 1), use_bias=True, kernel_initializer="he_normal",
                 kernel_regularizer=None, antisymmetric=True, **kwargs):
        super().__init__(gamma=gamma, strides=strides, use_bias=use_bias, kernel_initializer=kernel_initializer,
                         kernel_regularizer=kernel_regularizer, **kwargs)
        self.kernel_size = int(kernel_size)
        self.antisymmetric = bool(antisymmetric)

    def build(self, input_shape):
        self.num_channels = int(input_shape[-1])
        C, k = self.num_channels, self.kernel_size
        free = _free_positions(k, self.antisymmetric)
        self.independent_kernels = []
        for o in range(C):
            for (i, j) in free:
                self._add_theta(f"centro_sym_{i}_{j}", (1, 1, 1, 1))
            if C - o - 1 > 0:
                self.independent_kernels.append(
                    self._add_theta(f"input_kernels_for_output_kernel_{o}", (k, k, C - o - 1, 1)))
        self._add_bias()
        self.built = True

    def get_config(self):
        c = super().get_config()
        c.update({"kernel_size": self.kernel_size, "antisymmetric": self.antisymmetric})
        return c
