"""Weight I/O (reference: model_utils/)."""
from .weight_utils import double_load_weights, pickle_model_weights, save_model_weights

__all__ = ["double_load_weights", "pickle_model_weights", "save_model_weights"]
