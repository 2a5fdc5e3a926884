"""Per-layer weight files and depth doubling (reference:
model_utils/weight_utils.py:23-79).

The reference pickles a list of {'kernel', 'bias'} dicts, one per layer with
weights, which only works for two-weight layers.  Here the file is an npz
(no pickle): for layer i with weights, arrays 'L{i:04d}_{j:03d}' hold its
j-th weight in creation order, so the C+4-variable antisymmetric layers
round-trip too.  double_load_weights loads an (l+2)-layer single-block
ResNet into a (2l+2)-layer one, each saved block feeding two consecutive
blocks (conv1 and fc once)."""
from __future__ import annotations

import numpy as np

__all__ = ["save_model_weights", "pickle_model_weights", "load_layer_weights", "double_load_weights"]


def _weighted_layers(model):
    return [layer for layer in model.layers if layer.weights]


def save_model_weights(model, save_filename):
    model._pull()
    arrays = {}
    for i, layer in enumerate(_weighted_layers(model)):
        for j, w in enumerate(layer.get_weights()):
            arrays[f"L{i:04d}_{j:03d}"] = w
    np.savez(save_filename, **arrays)


# the reference's name, same role (the format is npz, not pickle)
pickle_model_weights = save_model_weights


def load_layer_weights(weights_file):
    """List (per layer with weights) of lists of arrays."""
    with np.load(weights_file, allow_pickle=False) as f:
        keys = sorted(f.files)
        layers: dict = {}
        for k in keys:
            i, j = int(k[1:5]), int(k[6:9])
            layers.setdefault(i, {})[j] = f[k]
    return [[d[j] for j in sorted(d)] for _, d in sorted(layers.items())]


def double_load_weights(model, weights_file):
    saved = load_layer_weights(weights_file)
    target = _weighted_layers(model)
    if len(target) != 2 * (len(saved) - 2) + 2:
        raise ValueError(f"model has {len(target)} weighted layers; a doubled {len(saved)}-layer model has "
                         f"{2 * (len(saved) - 2) + 2}")
    target[0].set_weights(saved[0])
    for l in range(1, len(saved) - 1):
        target[2 * l - 1].set_weights(saved[l])
        target[2 * l].set_weights(saved[l])
    target[-1].set_weights(saved[-1])
    model._push()
