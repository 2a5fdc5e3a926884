"""Weight initialisers of the reference, on the host (numpy, float32).

* Conv2DAntisymmetric3By3 / Conv2DAntisymmetric: tf.initializers.truncated_normal
  with stddev sqrt(2 / (k*k*C)) (layers/tfkeras_layer_Conv2DAntisymmetric3By3.py:95-98,
  …Conv2DAntisymmetric.py:100-103): normal draws re-sampled outside 2 sigma.
* Keras 'he_normal' (conv1 / Dense, models/tfkeras_resnets.py:563-572, :595-597):
  VarianceScaling(scale=2, mode='fan_in', distribution='truncated_normal'), whose
  stddev is sqrt(2/fan_in) / 0.87962566103423978 (the std of a 2-sigma truncated
  unit normal) in TF 1.12.
* biases: zeros.
"""
from __future__ import annotations

import math

import numpy as np

TRUNC_STD = 0.87962566103423978


def truncated_normal(rng: np.random.Generator, shape, stddev: float) -> np.ndarray:
    out = rng.standard_normal(size=shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(size=int(bad.sum()))
        bad = np.abs(out) > 2.0
    return (out * stddev).astype(np.float32)


def antisymmetric_kernel_stddev(kernel_size: int, channels: int) -> float:
    return math.sqrt(2.0 / (kernel_size * kernel_size * channels))


def he_normal(rng: np.random.Generator, shape) -> np.ndarray:
    fan_in = int(np.prod(shape[:-1])) if len(shape) > 1 else int(shape[0])
    return truncated_normal(rng, shape, math.sqrt(2.0 / max(fan_in, 1)) / TRUNC_STD)


def _fans(shape):
    if len(shape) < 2:
        return int(shape[0]) if shape else 1, int(shape[0]) if shape else 1
    rf = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    return rf * int(shape[-2]), rf * int(shape[-1])


def glorot_uniform(rng: np.random.Generator, shape) -> np.ndarray:
    """Keras default kernel initialiser: U(-l, l), l = sqrt(6/(fan_in+fan_out))."""
    fi, fo = _fans(shape)
    lim = math.sqrt(6.0 / max(fi + fo, 1))
    return rng.uniform(-lim, lim, size=shape).astype(np.float32)


def zeros(shape) -> np.ndarray:
    return np.zeros(shape, dtype=np.float32)


def get(identifier):
    """Resolve a Keras-style initializer identifier to fn(rng, shape, **ctx)
    (callables are used as such and must accept that signature)."""
    if callable(identifier):
        return identifier
    if identifier in (None, "zeros"):
        return lambda rng, shape, **_: zeros(shape)
    if identifier == "ones":
        return lambda rng, shape, **_: np.ones(shape, np.float32)
    if identifier == "glorot_uniform":
        return lambda rng, shape, **_: glorot_uniform(rng, shape)
    if identifier == "he_normal":
        return lambda rng, shape, **_: he_normal(rng, shape)
    if identifier == "antisymmetric_he_normal":
        return lambda rng, shape, kernel_size=3, channels=1, **_: truncated_normal(
            rng, shape, antisymmetric_kernel_stddev(kernel_size, channels))
    raise ValueError(f"unknown initializer {identifier!r}")
