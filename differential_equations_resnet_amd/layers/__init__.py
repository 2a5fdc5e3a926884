"""Drop-in layers (reference: layers/)."""
from .tfkeras_layer_Conv2DAntisymmetric import Conv2DAntisymmetric
from .tfkeras_layer_Conv2DAntisymmetric3By3 import Conv2DAntisymmetric3By3

__all__ = ["Conv2DAntisymmetric", "Conv2DAntisymmetric3By3"]
