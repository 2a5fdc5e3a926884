"""Drop-in for models/tfkeras_resnets.py: the ResNet builders, same function
names, keyword arguments, defaults, layer names and errors, composing the
graph layers of this framework (graph.py) and the native antisymmetric
layers.  Models built here run through Model.compile_native / Training,
which lower the single-block antisymmetric (or regular) ResNet onto the
fused native executor.

Layer naming (so notebook code like model.get_layer('res2_3_branch2') keeps
working): block convs res{stage}_{block}_branch2[a|b|c] / _branch1 (shortcut),
BN bn{stage}_{block}_branch..., h-scaling Lambdas scale{stage}_{block}, stem
identity_layer / input_mean_shift / input_scaling / conv1 / bn_conv1, head
global_average_pooling / fc (tfkeras_resnets.py:66-67, :91, :555-597)."""
from __future__ import annotations

import numpy as np

from ..graph import (Activation, BatchNormalization, Conv2D, Dense, GlobalAveragePooling2D, Input, Lambda,
                     MaxPooling2D, Model, ZeroPadding2D, add, l2)
from ..layers.tfkeras_layer_Conv2DAntisymmetric3By3 import Conv2DAntisymmetric3By3

__all__ = [
    "single_layer_identity_block", "bottleneck_identity_block", "single_layer_conv_block", "bottleneck_conv_block",
    "build_single_block_resnet", "get_single_block_resnet_build_function", "build_resnet",
    "get_resnet_build_function",
]


def _names(stage, block):
    tag = f"{stage}_{block}_branch"
    return "res" + tag, "bn" + tag


def _scale(h):
    def scale(x):
        return h * x
    return scale


def _antisym_conv_layer(gamma, strides, kernel_regularizer, name):
    return Conv2DAntisymmetric3By3(gamma=gamma, strides=strides, use_bias=True, kernel_initializer="he_normal",
                                   kernel_regularizer=kernel_regularizer, name=name)


def _antisym_conv(x, gamma, strides, kernel_regularizer, name):
    return _antisym_conv_layer(gamma, strides, kernel_regularizer, name)(x)


def _conv(x, filters, kernel_size, name, strides=(1, 1), padding="same", kernel_regularizer=None,
          bias_regularizer=None):
    return Conv2D(filters=filters, kernel_size=kernel_size, strides=strides, padding=padding,
                  kernel_initializer="he_normal", kernel_regularizer=kernel_regularizer,
                  bias_regularizer=bias_regularizer, name=name)(x)


def single_layer_identity_block(input_tensor, kernel_size, antisymmetric, use_batch_norm, stage, block, h=1.0,
                                gamma=0.0, kernel_regularizer=None, bias_regularizer=None, integrator="euler"):
    """One Euler step x + h*relu(conv(x)) (tfkeras_resnets.py:28-94): the
    conv is Conv2DAntisymmetric3By3 when `antisymmetric`, else a regular
    'same' Conv2D with C filters; optional BN after it; the h-scaling Lambda
    exists only when h != 1.

    integrator="rk2" (extension, not in the reference; BASELINE config 5)
    builds the explicit midpoint step with the SAME conv layer (shared
    weights) applied twice:
        xm = x + (h/2)*relu(conv(x)),   out = x + h*relu(conv(xm))
    with the half-step scaling Lambda named scale{stage}_{block}_half."""
    if integrator not in ("euler", "rk2"):
        raise ValueError(f"integrator must be 'euler' or 'rk2', got {integrator!r}")
    conv_name, bn_name = _names(stage, block)
    if antisymmetric:
        conv = _antisym_conv_layer(gamma, (1, 1), kernel_regularizer, conv_name + "2")
    else:
        conv = Conv2D(filters=int(input_tensor.shape[-1]), kernel_size=kernel_size, strides=(1, 1), padding="same",
                      kernel_initializer="he_normal", kernel_regularizer=kernel_regularizer,
                      bias_regularizer=bias_regularizer, name=conv_name + "2")
    if integrator == "rk2":
        if use_batch_norm:
            raise ValueError("integrator='rk2' does not support use_batch_norm")
        k1 = Activation("relu")(conv(input_tensor))
        if 0.5 * h != 1.0:
            k1 = Lambda(_scale(0.5 * h), name=f"scale{stage}_{block}_half")(k1)
        xm = add([k1, input_tensor])
        x = Activation("relu")(conv(xm))
        if h != 1.0:
            x = Lambda(_scale(h), name=f"scale{stage}_{block}")(x)
        return add([x, input_tensor])
    x = conv(input_tensor)
    if use_batch_norm:
        x = BatchNormalization(axis=3, name=bn_name + "2")(x)
    x = Activation("relu")(x)
    if h != 1.0:
        x = Lambda(_scale(h), name=f"scale{stage}_{block}")(x)
    return add([x, input_tensor])


def bottleneck_identity_block(input_tensor, kernel_size, num_filters, antisymmetric, use_batch_norm, stage, block,
                              gamma=0.0, kernel_regularizer=None, bias_regularizer=None):
    """1x1 -> kxk -> 1x1 bottleneck with identity shortcut
    (tfkeras_resnets.py:96-202); the kxk conv is antisymmetric when
    `antisymmetric` and num_filters[1] is None."""
    conv_name, bn_name = _names(stage, block)
    regs = dict(kernel_regularizer=kernel_regularizer, bias_regularizer=bias_regularizer)
    x = _conv(input_tensor, num_filters[0], (1, 1), conv_name + "2a", padding="valid", **regs)
    if use_batch_norm:
        x = BatchNormalization(axis=3, name=bn_name + "2a")(x)
    x = Activation("relu")(x)
    if antisymmetric and num_filters[1] is None:
        x = _antisym_conv(x, gamma, (1, 1), kernel_regularizer, conv_name + "2b")
    else:
        x = _conv(x, num_filters[1], kernel_size, conv_name + "2b", **regs)
    if use_batch_norm:
        x = BatchNormalization(axis=3, name=bn_name + "2b")(x)
    x = Activation("relu")(x)
    x = _conv(x, num_filters[2], (1, 1), conv_name + "2c", padding="valid", **regs)
    if use_batch_norm:
        x = BatchNormalization(axis=3, name=bn_name + "2c")(x)
    x = add([x, input_tensor])
    return Activation("relu")(x)


def single_layer_conv_block(input_tensor, kernel_size, num_filters, strides, use_batch_norm, stage, block,
                            kernel_regularizer=None, bias_regularizer=None):
    """Stage transition: relu(conv(x)) + 1x1 projection shortcut
    (tfkeras_resnets.py:204-269)."""
    conv_name, bn_name = _names(stage, block)
    regs = dict(kernel_regularizer=kernel_regularizer, bias_regularizer=bias_regularizer)
    x = _conv(input_tensor, num_filters, kernel_size, conv_name + "2", strides=strides, **regs)
    shortcut = _conv(input_tensor, num_filters, (1, 1), conv_name + "1", strides=strides, padding="valid", **regs)
    if use_batch_norm:
        x = BatchNormalization(axis=3, name=bn_name + "2")(x)
        shortcut = BatchNormalization(axis=3, name=bn_name + "1")(shortcut)
    x = Activation("relu")(x)
    return add([x, shortcut])


def bottleneck_conv_block(input_tensor, kernel_size, num_filters, antisymmetric, use_batch_norm, stage, block,
                          version=1, strides=(1, 1), gamma=0.0, kernel_regularizer=None, bias_regularizer=None):
    """Bottleneck with projection shortcut (tfkeras_resnets.py:271-425);
    version 1 strides in the first 1x1, version 1.5 in the kxk conv."""
    if version == 1:
        s_1x1, s_kxk = strides, (1, 1)
    elif version == 1.5:
        s_1x1, s_kxk = (1, 1), strides
    else:
        raise ValueError("Supported values for `version` are 1 and 1.5.")
    conv_name, bn_name = _names(stage, block)
    regs = dict(kernel_regularizer=kernel_regularizer, bias_regularizer=bias_regularizer)
    x = _conv(input_tensor, num_filters[0], (1, 1), conv_name + "2a", strides=s_1x1, padding="valid", **regs)
    if use_batch_norm:
        x = BatchNormalization(axis=3, name=bn_name + "2a")(x)
    x = Activation("relu")(x)
    if antisymmetric and num_filters[1] is None:
        x = _antisym_conv(x, gamma, s_kxk, kernel_regularizer, conv_name + "2b")
    else:
        x = _conv(x, num_filters[1], kernel_size, conv_name + "2b", strides=s_kxk, **regs)
    if use_batch_norm:
        x = BatchNormalization(axis=3, name=bn_name + "2b")(x)
    x = Activation("relu")(x)
    x = _conv(x, num_filters[2], (1, 1), conv_name + "2c", padding="valid", **regs)
    if use_batch_norm:
        x = BatchNormalization(axis=3, name=bn_name + "2c")(x)
    shortcut = Conv2D(filters=num_filters[2], kernel_size=(1, 1), strides=strides, kernel_initializer="he_normal",
                      name=conv_name + "1")(input_tensor)
    if use_batch_norm:
        shortcut = BatchNormalization(axis=3, name=bn_name + "1")(shortcut)
    x = add([x, shortcut])
    return Activation("relu")(x)


def _input_lambdas(input_tensor, subtract_mean, divide_by_stddev):
    """identity_layer, then optional mean shift and scaling Lambdas
    (tfkeras_resnets.py:552-559)."""
    shape = list(input_tensor.shape)
    x = Lambda(lambda v: v, output_shape=shape, name="identity_layer")(input_tensor)
    if subtract_mean is not None:
        x = Lambda(lambda v: v - subtract_mean, output_shape=shape, name="input_mean_shift")(x)
    if divide_by_stddev is not None:
        x = Lambda(lambda v: v / divide_by_stddev, output_shape=shape, name="input_scaling")(x)
    return x


def _model_name(base, kernel_type):
    return base + ("_antisymmetric" if kernel_type == "antisymmetric" else "_regular")


def get_single_block_resnet_build_function(kernel_type="antisymmetric", kernel_size=3, h=1.0, gamma=0.0,
                                           num_stages=5, blocks_per_stage=[3, 4, 6, 3],
                                           filters_per_block=[64, 128, 256, 512],
                                           strides=[(2, 2), (2, 2), (2, 2), (2, 2)], include_top=True,
                                           fc_activation="softmax", num_classes=None, use_batch_norm=False,
                                           use_max_pooling=[False, False, False, False], l2_regularization=0.0,
                                           subtract_mean=None, divide_by_stddev=None, verbose=False,
                                           integrator="euler"):
    """Returns build(input_tensor) -> Model for the single-conv-per-block
    ResNet (tfkeras_resnets.py:511-604).  `integrator` (extension, default
    the reference's forward Euler) is passed to every identity block."""
    if include_top and num_classes is None:
        raise ValueError("You must pass a positive integer for `num_classes` if `include_top` is `True`.")
    antisymmetric = kernel_type == "antisymmetric"
    name = _model_name("single_block_resnet", kernel_type)
    mean = None if subtract_mean is None else np.array(subtract_mean)
    std = None if divide_by_stddev is None else np.array(divide_by_stddev)

    def _build_function(input_tensor):
        x = _input_lambdas(input_tensor, mean, std)
        if verbose:
            print("Building stage 1")
        x = Conv2D(filters=filters_per_block[0], kernel_size=kernel_size, strides=strides[0], padding="same",
                   kernel_initializer="he_normal", kernel_regularizer=l2(l2_regularization), name="conv1")(x)
        if use_batch_norm:
            x = BatchNormalization(axis=3, name="bn_conv1")(x)
        x = Activation("relu")(x)

        def identity(x, stage, b):
            if verbose:
                print(f"Building identity block {stage}-{b + 1}")
            return single_layer_identity_block(x, kernel_size, antisymmetric, use_batch_norm, stage=stage, block=b,
                                               h=h, gamma=gamma, kernel_regularizer=l2(l2_regularization),
                                               integrator=integrator)

        for s in range(num_stages - 1):
            stage = s + 2
            if use_max_pooling[s]:
                x = MaxPooling2D(pool_size=(2, 2), strides=None, name=f"stage{stage}_pooling")(x)
            same_shape = not use_max_pooling[s] and (
                s == 0 or (filters_per_block[s] == filters_per_block[s - 1] and strides[s] == (1, 1)))
            if same_shape:
                for b in range(blocks_per_stage[s]):
                    x = identity(x, stage, b)
            else:
                if verbose:
                    print(f"Building conv block {stage}-1")
                x = single_layer_conv_block(x, kernel_size, filters_per_block[s], strides[s], use_batch_norm,
                                            stage=stage, block=0, kernel_regularizer=l2(l2_regularization))
                for b in range(1, blocks_per_stage[s]):
                    x = identity(x, stage, b)
        if include_top:
            x = GlobalAveragePooling2D(name="global_average_pooling")(x)
            x = Dense(num_classes, activation=fc_activation, kernel_initializer="he_normal",
                      kernel_regularizer=l2(l2_regularization), name="fc")(x)
        return Model(input_tensor, x, name=name)

    return _build_function


def build_single_block_resnet(image_shape, kernel_type="antisymmetric", kernel_size=3, h=1.0, gamma=0.0,
                              num_stages=5, blocks_per_stage=[3, 4, 6, 3], filters_per_block=[64, 128, 256, 512],
                              strides=[(2, 2), (2, 2), (2, 2), (2, 2)], include_top=True, fc_activation="softmax",
                              num_classes=None, use_batch_norm=False, use_max_pooling=[False, False, False, False],
                              l2_regularization=0.0, subtract_mean=None, divide_by_stddev=None, verbose=False,
                              integrator="euler"):
    """tfkeras_resnets.py:427-509: build function applied to Input(image_shape)."""
    fn = get_single_block_resnet_build_function(
        kernel_type=kernel_type, kernel_size=kernel_size, h=h, gamma=gamma, num_stages=num_stages,
        blocks_per_stage=blocks_per_stage, filters_per_block=filters_per_block, strides=strides,
        include_top=include_top, fc_activation=fc_activation, num_classes=num_classes, use_batch_norm=use_batch_norm,
        use_max_pooling=use_max_pooling, l2_regularization=l2_regularization, subtract_mean=subtract_mean,
        divide_by_stddev=divide_by_stddev, verbose=verbose, integrator=integrator)
    return fn(Input(shape=image_shape))


_PRESETS = {"resnet50": [3, 4, 6, 3], "resnet101": [3, 4, 23, 3], "resnet152": [3, 8, 36, 3]}
_BOTTLENECK_FILTERS = [[64, 64, 256], [128, 128, 512], [256, 256, 1024], [512, 512, 2048]]


def get_resnet_build_function(kernel_type="antisymmetric", include_top=True, fc_activation="softmax",
                              num_classes=None, l2_regularization=0.0, subtract_mean=None, divide_by_stddev=None,
                              version=1, preset=None, blocks_per_stage=[3, 4, 6, 3],
                              filters_per_block=_BOTTLENECK_FILTERS, use_batch_norm=True):
    """Bottleneck ResNet-50/101/152 family (tfkeras_resnets.py:698-818).
    Graph description only: the native executor runs the single-block
    family (the antisymmetric hot path); compiling this one raises
    AsrUnsupported."""
    if include_top and num_classes is None:
        raise ValueError("You must pass a positive integer for `num_classes` if `include_top` is `True`.")
    name = "resnet"
    if preset is not None:
        if preset not in _PRESETS:
            raise ValueError("`preset` must be either `None` or one of 'resnet50', 'resnet101', and 'resnet152', "
                             f"but you passed `preset={preset}`.")
        blocks_per_stage = _PRESETS[preset]
        filters_per_block = _BOTTLENECK_FILTERS
        use_batch_norm = True
        name += preset[len("resnet"):]
    antisymmetric = kernel_type == "antisymmetric"
    name = _model_name(name, kernel_type)
    mean = None if subtract_mean is None else np.array(subtract_mean)
    std = None if divide_by_stddev is None else np.array(divide_by_stddev)

    def _build_function(input_tensor):
        x = _input_lambdas(input_tensor, mean, std)
        x = ZeroPadding2D(padding=(3, 3), name="conv1_pad")(x)
        x = Conv2D(filters=64, kernel_size=(7, 7), strides=(2, 2), padding="valid", kernel_initializer="he_normal",
                   kernel_regularizer=l2(l2_regularization), name="conv1")(x)
        if use_batch_norm:
            x = BatchNormalization(axis=3, name="bn_conv1")(x)
        x = Activation("relu")(x)
        x = ZeroPadding2D(padding=(1, 1), name="pool1_pad")(x)
        x = MaxPooling2D(pool_size=(3, 3), strides=(2, 2), name="stage1_pooling")(x)
        for si, stage in enumerate(range(2, 6)):
            x = bottleneck_conv_block(x, 3, filters_per_block[si], antisymmetric, use_batch_norm, stage=stage,
                                      block=0, version=version, strides=(1, 1) if stage == 2 else (2, 2),
                                      kernel_regularizer=l2(l2_regularization))
            for i in range(1, blocks_per_stage[si]):
                x = bottleneck_identity_block(x, 3, filters_per_block[si], antisymmetric, use_batch_norm,
                                              stage=stage, block=i, kernel_regularizer=l2(l2_regularization))
        if include_top:
            x = GlobalAveragePooling2D(name="global_average_pooling")(x)
            x = Dense(num_classes, activation=fc_activation, kernel_initializer="he_normal",
                      kernel_regularizer=l2(l2_regularization), name="fc")(x)
        return Model(input_tensor, x, name=name)

    return _build_function


def build_resnet(image_shape, kernel_type="antisymmetric", include_top=True, fc_activation="softmax",
                 num_classes=None, l2_regularization=0.0, subtract_mean=None, divide_by_stddev=None, version=1,
                 preset=None, blocks_per_stage=[3, 4, 6, 3], filters_per_block=_BOTTLENECK_FILTERS,
                 use_batch_norm=True):
    """tfkeras_resnets.py:606-696."""
    fn = get_resnet_build_function(kernel_type=kernel_type, include_top=include_top, fc_activation=fc_activation,
                                   num_classes=num_classes, l2_regularization=l2_regularization,
                                   subtract_mean=subtract_mean, divide_by_stddev=divide_by_stddev, version=version,
                                   preset=preset, blocks_per_stage=blocks_per_stage,
                                   filters_per_block=filters_per_block, use_batch_norm=use_batch_norm)
    return fn(Input(shape=image_shape))
