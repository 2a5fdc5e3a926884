"""Flat parameter buffers of the single-block antisymmetric ResNet in Keras
get_weights() order (the layout asr_net_* consumes, include/asr.h):

  conv1 kernel [3,3,Cin,C], conv1 bias [C],
  L x (a, b, c, d [1,1,1,C], input_kernels_for_output_kernel_{0..C-2} [3,3,C-o-1], bias [C]),
  fc kernel [C,K], fc bias [K]

(models/tfkeras_resnets.py:547-597; layer weight order
layers/tfkeras_layer_Conv2DAntisymmetric3By3.py:113-153).
"""
from __future__ import annotations

import numpy as np

from . import initializers


def antisym_theta_shapes(C: int):
    return [(1, 1, 1, C)] * 4 + [(3, 3, C - o - 1) for o in range(C - 1)]


def net_param_shapes(C: int, L: int, Cin: int = 3, K: int = 10):
    s = [(3, 3, Cin, C), (C,)]
    for _ in range(L):
        s += antisym_theta_shapes(C) + [(C,)]
    s += [(C, K), (K,)]
    return s


def init_net_params(C: int, L: int, Cin: int = 3, K: int = 10, seed: int = 0, bias_std: float = 0.0) -> np.ndarray:
    """Reference initialisation (he_normal kernels, antisymmetric truncated
    normal thetas, zero biases unless bias_std > 0), flattened."""
    rng = np.random.default_rng(seed)
    out = [initializers.he_normal(rng, (3, 3, Cin, C)), _bias(rng, C, bias_std)]
    std = initializers.antisymmetric_kernel_stddev(3, C)
    for _ in range(L):
        for s in antisym_theta_shapes(C):
            out.append(initializers.truncated_normal(rng, s, std))
        out.append(_bias(rng, C, bias_std))
    out.append(initializers.he_normal(rng, (C, K)))
    out.append(np.zeros(K, np.float32))
    return np.concatenate([a.ravel() for a in out]).astype(np.float32)


def _bias(rng, C, std):
    if std == 0:
        return np.zeros(C, np.float32)
    return (rng.standard_normal(C) * std).astype(np.float32)
