"""Model builders (reference: models/)."""
from .tfkeras_resnets import (bottleneck_conv_block, bottleneck_identity_block, build_resnet,
                              build_single_block_resnet, get_resnet_build_function,
                              get_single_block_resnet_build_function, single_layer_conv_block,
                              single_layer_identity_block)

__all__ = ["bottleneck_conv_block", "bottleneck_identity_block", "build_resnet", "build_single_block_resnet",
           "get_resnet_build_function", "get_single_block_resnet_build_function", "single_layer_conv_block",
           "single_layer_identity_block"]
