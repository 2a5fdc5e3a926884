"""Device-resident dataset from in-memory arrays: the replacement of
dataset_utils/tf_dataset_creator_from_arrays.py:22-58 (from_tensor_slices ->
shuffle(full buffer, reshuffle each iteration) -> repeat -> batch).

The whole uint8 image array lives in HBM (CIFAR-10 train: 153.6 MB); a batch
is an index gather on the device, so no host copy sits on the training step.
As with shuffle -> repeat -> batch, batches run across epoch boundaries
(successive independent permutations) and are always full.  For data
parallelism every rank draws the same permutation stream and takes its own
contiguous slice of each global batch (rank r of R gets images
[r*B, (r+1)*B) of the R*B-image global batch).
"""
from __future__ import annotations

import numpy as np

__all__ = ["ArrayDataset", "create_tf_dataset_from_arrays"]


class ArrayDataset:
    def __init__(self, features, labels, batch_size, preprocessors=None, repeat=True, num_epochs=None, shuffle=True,
                 seed=0, num_classes=None, rank=0, world_size=1, device=None):
        import torch
        features = np.asarray(features)
        labels = np.asarray(labels)
        if features.shape[0] != labels.shape[0]:
            raise ValueError("features and labels must have the same number of rows")
        if labels.ndim == 1:
            if num_classes is None:
                num_classes = int(labels.max()) + 1
            labels = np.eye(num_classes, dtype=np.float32)[labels]
        self.n = int(features.shape[0])
        self.batch_size = int(batch_size)
        self.preprocessors = list(preprocessors or [])
        self.repeat = repeat
        self.num_epochs = num_epochs
        self.shuffle = shuffle
        self.seed = int(seed)
        self.rank, self.world_size = int(rank), int(world_size)
        if self.batch_size * self.world_size > self.n:
            raise ValueError("global batch larger than the dataset")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        fdt = torch.uint8 if features.dtype == np.uint8 else torch.float32
        self.features = torch.from_numpy(np.ascontiguousarray(features)).to(self.device, fdt)
        self.labels = torch.from_numpy(np.ascontiguousarray(labels, dtype=np.float32)).to(self.device)
        self.output_shapes = ((self.batch_size,) + tuple(features.shape[1:]), (self.batch_size, labels.shape[1]))

    def _order(self):
        rng = np.random.default_rng(self.seed)
        epoch = 0
        while self.num_epochs is None or epoch < self.num_epochs:
            yield rng.permutation(self.n) if self.shuffle else np.arange(self.n)
            epoch += 1
            if not self.repeat:
                return

    def __iter__(self):
        import torch
        G = self.batch_size * self.world_size
        pending = np.empty(0, dtype=np.int64)
        for perm in self._order():
            pending = np.concatenate([pending, perm])
            while pending.size >= G:
                idx = pending[self.rank * self.batch_size:(self.rank + 1) * self.batch_size]
                pending = pending[G:]
                it = torch.from_numpy(idx).to(self.device, non_blocking=True)
                x = self.features.index_select(0, it)
                y = self.labels.index_select(0, it)
                for p in self.preprocessors:
                    x, y = p(x, y)
                yield x, y
        # a non-repeating stream ends with its (dropped) partial batch


def create_tf_dataset_from_arrays(features, labels, batch_size, preprocessors=None, repeat=True, num_epochs=None,
                                  shuffle=True, prefetch=None, **kwargs):
    """Same call as the reference; returns (dataset, features, labels) where
    the reference returned its two feed placeholders (nothing needs feeding
    here)."""
    ds = ArrayDataset(features, labels, batch_size, preprocessors=preprocessors, repeat=repeat,
                      num_epochs=num_epochs, shuffle=shuffle, **kwargs)
    return ds, features, labels
