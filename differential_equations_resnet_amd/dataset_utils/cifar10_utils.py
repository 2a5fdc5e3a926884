"""CIFAR-10 loading (reference: dataset_utils/cifar10_utils.py:24-75), to
NHWC uint8.

Reads either the binary distribution (data_batch_{1..5}.bin, test_batch.bin,
batches.meta.txt: 1 label byte + 3072 CHW bytes per record) or the Python
distribution the reference reads (data_batch_{1..5}, test_batch,
batches.meta).  The Python files are pickles; they are read with an
unpickler that only admits plain containers, bytes and numpy arrays (no
other globals), so a tampered file cannot execute code."""
from __future__ import annotations

import io
import os
import pickle

import numpy as np

__all__ = ["build_cifar10_dataset", "one_hot"]

_TRAIN = [f"data_batch_{i}" for i in range(1, 6)]


class _DataOnlyUnpickler(pickle.Unpickler):
    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
                ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
                ("numpy._core.multiarray", "scalar")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing global {module}.{name} in a dataset file")


def _load_py(path):
    with open(path, "rb") as f:
        return _DataOnlyUnpickler(io.BytesIO(f.read()), encoding="bytes").load()


def _chw_to_nhwc(flat):
    return np.ascontiguousarray(np.asarray(flat, dtype=np.uint8).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))


def _read_bin(path):
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 3073)
    return _chw_to_nhwc(raw[:, 1:]), raw[:, 0].astype(np.int64)


def build_cifar10_dataset(cifar10_directory):
    """Returns (train_images [50000,32,32,3] u8, train_labels [50000],
    test_images [10000,32,32,3] u8, test_labels [10000], label_names)."""
    d = cifar10_directory
    if os.path.exists(os.path.join(d, "data_batch_1.bin")):
        parts = [_read_bin(os.path.join(d, f + ".bin")) for f in _TRAIN]
        xtr = np.concatenate([p[0] for p in parts])
        ytr = np.concatenate([p[1] for p in parts])
        xte, yte = _read_bin(os.path.join(d, "test_batch.bin"))
        meta = os.path.join(d, "batches.meta.txt")
        names = [l.strip() for l in open(meta).read().splitlines() if l.strip()] if os.path.exists(meta) else []
        return xtr, ytr, xte, yte, names
    tr = [_load_py(os.path.join(d, f)) for f in _TRAIN]
    xtr = _chw_to_nhwc(np.concatenate([np.asarray(t[b"data"]) for t in tr]))
    ytr = np.concatenate([np.asarray(t[b"labels"], dtype=np.int64) for t in tr])
    te = _load_py(os.path.join(d, "test_batch"))
    xte = _chw_to_nhwc(te[b"data"])
    yte = np.asarray(te[b"labels"], dtype=np.int64)
    meta = _load_py(os.path.join(d, "batches.meta"))
    names = [b.decode("utf-8") for b in meta[b"label_names"]]
    return xtr, ytr, xte, yte, names


def one_hot(labels, num_classes=10):
    return np.eye(num_classes, dtype=np.float32)[np.asarray(labels, dtype=np.int64)]
