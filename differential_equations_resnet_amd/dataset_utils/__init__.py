"""Input pipeline (reference: dataset_utils/)."""
from .array_dataset import ArrayDataset, create_tf_dataset_from_arrays
from .cifar10_utils import build_cifar10_dataset, one_hot

__all__ = ["ArrayDataset", "create_tf_dataset_from_arrays", "build_cifar10_dataset", "one_hot"]
