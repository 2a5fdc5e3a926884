"""A small Keras-style functional graph: the layer/model surface the
reference's builders and training driver are written against
(tf.keras.layers.* as imported at models/tfkeras_resnets.py:23-26,
tf.keras.models.Model at :600, Layer.add_weight/get_weights/get_config).

This module only DESCRIBES networks — symbolic tensors, layers, weights held
as host float32 arrays in creation order.  Nothing here computes: a Model is
executed by lowering it onto the native executor (lowering.py), and the two
antisymmetric layers additionally run eagerly on device tensors through the
C ABI (layers/).  A layer with no native lowering raises AsrUnsupported when
a model containing it is compiled; it never falls back to a host or torch
implementation.
"""
from __future__ import annotations

import itertools
import re
from collections import defaultdict

import numpy as np

from . import initializers

__all__ = [
    "set_seed", "Variable", "SymbolicTensor", "Layer", "InputLayer", "Input", "Lambda", "Conv2D", "Activation",
    "Add", "add", "GlobalAveragePooling2D", "Dense", "BatchNormalization", "MaxPooling2D", "ZeroPadding2D", "Model",
    "L2", "l2",
]

_rng = np.random.default_rng(0)
_name_counts: dict = defaultdict(itertools.count)


def set_seed(seed: int) -> None:
    """Seed the host RNG used by the weight initialisers (the analogue of
    tf.set_random_seed for this framework)."""
    global _rng
    _rng = np.random.default_rng(seed)


def rng() -> np.random.Generator:
    return _rng


def _snake(name: str) -> str:
    s = re.sub(r"(.)([A-Z][a-z]+)", r"\1_\2", name)
    return re.sub(r"([a-z0-9])([A-Z])", r"\1_\2", s).lower()


def _unique_name(base: str) -> str:
    n = next(_name_counts[base])
    return base if n == 0 else f"{base}_{n}"


class L2:
    """tf.keras.regularizers.l2.  Kept for signature compatibility: the
    reference's training driver ignores regularisation losses
    (training/training.py:290-296, '#TODO regularization_losses'), and so does
    this framework's."""

    def __init__(self, l=0.01):
        self.l2 = float(l)

    def get_config(self):
        return {"l2": self.l2}

    def __repr__(self):
        return f"L2({self.l2})"


def l2(l=0.01) -> L2:
    return L2(l)


class Variable:
    """A named weight: host float32 value in Keras creation order."""

    def __init__(self, name, value, trainable=True, regularizer=None):
        self.name = name
        self.value = np.ascontiguousarray(value, dtype=np.float32)
        self.trainable = trainable
        self.regularizer = regularizer

    @property
    def shape(self):
        return self.value.shape

    def numpy(self):
        return self.value

    def assign(self, value):
        value = np.asarray(value, dtype=np.float32)
        if value.shape != self.value.shape:
            raise ValueError(f"{self.name}: shape {value.shape} != {self.value.shape}")
        self.value[...] = value

    def __repr__(self):
        return f"<Variable {self.name} shape={self.shape}>"


class SymbolicTensor:
    """Output of a layer applied to symbolic inputs (the Keras tensor)."""

    def __init__(self, shape, layer, inbound):
        self.shape = tuple(shape)
        self.layer = layer
        self.inbound = list(inbound)

    @property
    def name(self):
        return f"{self.layer.name}/output"

    def __repr__(self):
        return f"<SymbolicTensor {self.name} shape={self.shape}>"


def _as_list(x):
    return list(x) if isinstance(x, (list, tuple)) else [x]


class Layer:
    """Base layer: lazy build on the first symbolic call, weights created with
    add_weight in a fixed order (Keras get_weights() order)."""

    def __init__(self, name=None, trainable=True, dtype="float32", **kwargs):
        unknown = set(kwargs) - {"input_shape", "batch_input_shape", "weights"}
        if unknown:
            raise TypeError(f"{type(self).__name__}: unexpected keyword arguments {sorted(unknown)}")
        self.name = name or _unique_name(_snake(type(self).__name__))
        self.trainable = trainable
        self.dtype = dtype
        self.built = False
        self._weights: list[Variable] = []
        self.inbound_nodes: list = []
        self._initial_weights = kwargs.get("weights")

    # -- weights -----------------------------------------------------------
    def add_weight(self, name, shape, initializer="zeros", regularizer=None, trainable=True, **init_ctx):
        init = initializers.get(initializer)
        value = init(_rng, tuple(shape), **init_ctx)
        v = Variable(f"{self.name}/{name}", value, trainable and self.trainable, regularizer)
        self._weights.append(v)
        return v

    @property
    def weights(self):
        return list(self._weights)

    @property
    def trainable_weights(self):
        return [w for w in self._weights if w.trainable]

    @property
    def non_trainable_weights(self):
        return [w for w in self._weights if not w.trainable]

    def get_weights(self):
        return [w.value.copy() for w in self._weights]

    def set_weights(self, weights):
        weights = list(weights)
        if len(weights) != len(self._weights):
            raise ValueError(f"{self.name}: expected {len(self._weights)} arrays, got {len(weights)}")
        for v, a in zip(self._weights, weights):
            v.assign(a)
        self._weights_changed()

    def _weights_changed(self):
        """Hook: device-side caches of this layer are stale."""

    def count_params(self):
        return int(sum(w.value.size for w in self._weights))

    # -- graph ---------------------------------------------------------------
    def build(self, input_shape):
        self.built = True

    def compute_output_shape(self, input_shape):
        return input_shape

    def get_config(self):
        return {"name": self.name, "trainable": self.trainable, "dtype": self.dtype}

    def __call__(self, inputs, **kwargs):
        ins = _as_list(inputs)
        if all(isinstance(t, SymbolicTensor) for t in ins):
            shapes = [t.shape for t in ins]
            shape_arg = shapes if isinstance(inputs, (list, tuple)) else shapes[0]
            if not self.built:
                self.build(shape_arg)
                self.built = True
                if self._initial_weights is not None:
                    self.set_weights(self._initial_weights)
            out = SymbolicTensor(self.compute_output_shape(shape_arg), self, ins)
            self.inbound_nodes.append(out)
            return out
        if any(isinstance(t, SymbolicTensor) for t in ins):
            raise TypeError(f"{self.name}: cannot mix symbolic and concrete inputs")
        return self.call_device(inputs, **kwargs)

    def call_device(self, inputs, **kwargs):
        from ._lib import AsrUnsupported
        raise AsrUnsupported(
            f"layer {self.name} ({type(self).__name__}) has no eager device kernel; run it inside a Model, "
            f"which is lowered onto the native executor")

    def __repr__(self):
        return f"<{type(self).__name__} {self.name}>"


class InputLayer(Layer):
    def __init__(self, shape, batch_size=None, name=None, dtype="float32"):
        super().__init__(name=name or _unique_name("input"), dtype=dtype)
        self.batch_shape = (batch_size,) + tuple(shape)
        self.built = True


def Input(shape=None, batch_size=None, name=None, dtype="float32", tensor=None, batch_shape=None):
    """tf.keras.layers.Input.  `tensor` may be a device array whose shape
    fixes the batch (as training.py:159 passes the dataset iterator's
    features): only its shape is used."""
    if batch_shape is not None:
        batch_size, shape = batch_shape[0], tuple(batch_shape[1:])
    if tensor is not None and shape is None:
        batch_size, shape = int(tensor.shape[0]), tuple(int(d) for d in tensor.shape[1:])
    if shape is None:
        raise ValueError("Input needs `shape`, `batch_shape` or `tensor`")
    layer = InputLayer(tuple(shape), batch_size, name, dtype)
    t = SymbolicTensor(layer.batch_shape, layer, [])
    layer.inbound_nodes.append(t)
    return t


class Lambda(Layer):
    """tf.keras.layers.Lambda.  Lowering treats a Lambda as an elementwise
    affine map x -> s*x + t, recovered by evaluating `function` on numpy
    probes (the builders' Lambdas are exactly that: identity, x - mean,
    x / std, h * x — tfkeras_resnets.py:91, :555-559)."""

    def __init__(self, function, output_shape=None, arguments=None, name=None, **kwargs):
        super().__init__(name=name, **kwargs)
        self.function = function
        self.output_shape = output_shape
        self.arguments = dict(arguments or {})

    def compute_output_shape(self, input_shape):
        if self.output_shape is None:
            return input_shape
        if callable(self.output_shape):
            return tuple(self.output_shape(input_shape))
        shp = tuple(self.output_shape)
        return shp if len(shp) == len(input_shape) else (input_shape[0],) + shp

    def affine(self, feature_shape):
        """(scale, shift) float64 arrays broadcast to feature_shape if the
        function is elementwise affine, else None."""
        f = lambda x: np.asarray(self.function(x, **self.arguments), dtype=np.float64)
        shape = (1,) + tuple(feature_shape)
        try:
            t = np.broadcast_to(f(np.zeros(shape)), shape)
            s = np.broadcast_to(f(np.ones(shape)), shape) - t
            probe = np.random.default_rng(7).standard_normal(shape) * 100.0
            ok = np.allclose(f(probe), s * probe + t, rtol=1e-9, atol=1e-9)
        except Exception:  # an arbitrary user function: not lowerable
            return None
        return (s[0], t[0]) if ok else None

    def get_config(self):
        c = super().get_config()
        c.update({"function": getattr(self.function, "__name__", "lambda"), "output_shape": self.output_shape,
                  "arguments": self.arguments})
        return c


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class Conv2D(Layer):
    """tf.keras.layers.Conv2D (NHWC, HWIO kernel, weights [kernel, bias])."""

    def __init__(self, filters, kernel_size, strides=(1, 1), padding="valid", activation=None, use_bias=True,
                 kernel_initializer="glorot_uniform", bias_initializer="zeros", kernel_regularizer=None,
                 bias_regularizer=None, dilation_rate=(1, 1), name=None, **kwargs):
        super().__init__(name=name, **kwargs)
        self.filters = int(filters)
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower()
        self.activation = activation
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer
        self.kernel_regularizer = kernel_regularizer
        self.bias_regularizer = bias_regularizer
        self.dilation_rate = _pair(dilation_rate)

    def build(self, input_shape):
        cin = int(input_shape[-1])
        self.kernel = self.add_weight("kernel", self.kernel_size + (cin, self.filters), self.kernel_initializer,
                                      self.kernel_regularizer)
        self.bias = self.add_weight("bias", (self.filters,), self.bias_initializer,
                                    self.bias_regularizer) if self.use_bias else None
        self.built = True

    def compute_output_shape(self, input_shape):
        n, h, w, _ = input_shape
        (kh, kw), (sh, sw) = self.kernel_size, self.strides

        def out(d, k, s):
            if d is None:
                return None
            return -(-d // s) if self.padding == "same" else (d - k) // s + 1
        return (n, out(h, kh, sh), out(w, kw, sw), self.filters)

    def get_config(self):
        c = super().get_config()
        c.update({"filters": self.filters, "kernel_size": self.kernel_size, "strides": self.strides,
                  "padding": self.padding, "activation": self.activation, "use_bias": self.use_bias,
                  "kernel_initializer": self.kernel_initializer, "kernel_regularizer": self.kernel_regularizer,
                  "bias_regularizer": self.bias_regularizer})
        return c


class Activation(Layer):
    def __init__(self, activation, name=None, **kwargs):
        super().__init__(name=name, **kwargs)
        self.activation = activation

    def get_config(self):
        c = super().get_config()
        c["activation"] = self.activation
        return c


class Add(Layer):
    def compute_output_shape(self, input_shape):
        shapes = list(input_shape)
        if any(s != shapes[0] for s in shapes):
            raise ValueError(f"Add: operands have different shapes {shapes}")
        return shapes[0]


def add(inputs, **kwargs):
    return Add(**kwargs)(list(inputs))


class GlobalAveragePooling2D(Layer):
    def compute_output_shape(self, input_shape):
        return (input_shape[0], input_shape[-1])


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer="glorot_uniform",
                 bias_initializer="zeros", kernel_regularizer=None, bias_regularizer=None, name=None, **kwargs):
        super().__init__(name=name, **kwargs)
        self.units = int(units)
        self.activation = activation
        self.use_bias = use_bias
        self.kernel_initializer = kernel_initializer
        self.bias_initializer = bias_initializer
        self.kernel_regularizer = kernel_regularizer
        self.bias_regularizer = bias_regularizer

    def build(self, input_shape):
        cin = int(input_shape[-1])
        self.kernel = self.add_weight("kernel", (cin, self.units), self.kernel_initializer, self.kernel_regularizer)
        self.bias = self.add_weight("bias", (self.units,), self.bias_initializer,
                                    self.bias_regularizer) if self.use_bias else None
        self.built = True

    def compute_output_shape(self, input_shape):
        return tuple(input_shape[:-1]) + (self.units,)

    def get_config(self):
        c = super().get_config()
        c.update({"units": self.units, "activation": self.activation, "use_bias": self.use_bias})
        return c


class BatchNormalization(Layer):
    """Described for graph compatibility (use_batch_norm=True builders);
    the antisymmetric experiments never enable it, and the
    native executor rejects it."""

    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, name=None, **kwargs):
        super().__init__(name=name, **kwargs)
        self.axis, self.momentum, self.epsilon = axis, momentum, epsilon

    def build(self, input_shape):
        c = int(input_shape[self.axis])
        self.add_weight("gamma", (c,), lambda r, s, **_: np.ones(s, np.float32))
        self.add_weight("beta", (c,), "zeros")
        self.add_weight("moving_mean", (c,), "zeros", trainable=False)
        self.add_weight("moving_variance", (c,), lambda r, s, **_: np.ones(s, np.float32), trainable=False)
        self.built = True


class MaxPooling2D(Layer):
    def __init__(self, pool_size=(2, 2), strides=None, padding="valid", name=None, **kwargs):
        super().__init__(name=name, **kwargs)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        self.padding = padding

    def compute_output_shape(self, input_shape):
        n, h, w, c = input_shape
        (ph, pw), (sh, sw) = self.pool_size, self.strides
        f = (lambda d, p, s: -(-d // s)) if self.padding == "same" else (lambda d, p, s: (d - p) // s + 1)
        return (n, None if h is None else f(h, ph, sh), None if w is None else f(w, pw, sw), c)


class ZeroPadding2D(Layer):
    def __init__(self, padding=(1, 1), name=None, **kwargs):
        super().__init__(name=name, **kwargs)
        self.padding = _pair(padding)

    def compute_output_shape(self, input_shape):
        n, h, w, c = input_shape
        ph, pw = self.padding
        return (n, None if h is None else h + 2 * ph, None if w is None else w + 2 * pw, c)


class Model:
    """tf.keras.models.Model(inputs, outputs, name): the layer DAG in
    topological (creation) order; weights in Keras get_weights() order."""

    def __init__(self, inputs, outputs, name=None):
        self.inputs = _as_list(inputs)
        self.outputs = _as_list(outputs)
        self.name = name or _unique_name("model")
        self.layers = self._topo_layers()
        self._native = None  # lowered executor cache (lowering.NativeModel)

    @property
    def input(self):
        return self.inputs[0] if len(self.inputs) == 1 else self.inputs

    @property
    def output(self):
        return self.outputs[0] if len(self.outputs) == 1 else self.outputs

    def _topo_layers(self):
        order, seen = [], set()

        def visit(t):
            if id(t) in seen:
                return
            seen.add(id(t))
            for p in t.inbound:
                visit(p)
            order.append(t)
        for o in self.outputs:
            visit(o)
        reached = {id(t.layer) for t in order if not t.inbound}
        for i in self.inputs:
            if id(i.layer) not in reached:
                raise ValueError(f"output is not connected to input {i.name}")
        layers, ids = [], set()
        for t in order:
            if id(t.layer) not in ids:
                ids.add(id(t.layer))
                layers.append(t.layer)
        return layers

    def nodes(self):
        """Symbolic tensors in topological order (each layer application)."""
        order, seen = [], set()

        def visit(t):
            if id(t) in seen:
                return
            seen.add(id(t))
            for p in t.inbound:
                visit(p)
            order.append(t)
        for o in self.outputs:
            visit(o)
        return order

    def get_layer(self, name=None, index=None):
        if index is not None:
            return self.layers[index]
        for layer in self.layers:
            if layer.name == name:
                return layer
        raise ValueError(f"No such layer: {name}")

    @property
    def weights(self):
        return [w for layer in self.layers for w in layer.weights]

    @property
    def trainable_weights(self):
        return [w for layer in self.layers for w in layer.trainable_weights]

    @property
    def trainable_variables(self):
        return self.trainable_weights

    def get_weights(self):
        self._pull()
        return [w.value.copy() for w in self.weights]

    def set_weights(self, weights):
        weights = list(weights)
        ws = self.weights
        if len(weights) != len(ws):
            raise ValueError(f"expected {len(ws)} arrays, got {len(weights)}")
        for v, a in zip(ws, weights):
            v.assign(a)
        for layer in self.layers:
            layer._weights_changed()
        self._push()

    def count_params(self):
        return int(sum(w.value.size for w in self.weights))

    def summary(self, print_fn=print):
        print_fn(f'Model: "{self.name}"')
        for t in self.nodes():
            print_fn(f"  {t.layer.name:<40s} {type(t.layer).__name__:<26s} {str(t.shape):<22s} "
                     f"{t.layer.count_params() if t is t.layer.inbound_nodes[0] else 0}")
        print_fn(f"Total params: {self.count_params()}")

    # -- weight files (reference-order npz; model_utils/weight_utils.py:23-39 pickles the same list) --
    def save_weights(self, path):
        ws = self.get_weights()
        names = [w.name for w in self.weights]
        np.savez(path, **{f"{i:05d}": a for i, a in enumerate(ws)}, __names__=np.array(names))

    def load_weights(self, path):
        with np.load(path, allow_pickle=False) as f:
            keys = sorted(k for k in f.files if k != "__names__")
            self.set_weights([f[k] for k in keys])

    # -- native execution ------------------------------------------------------
    def _pull(self):
        if self._native is not None:
            self._native.pull_weights()

    def _push(self):
        if self._native is not None:
            self._native.push_weights()

    def compile_native(self, batch_size, dtype=None, device=None):
        """Lower this model onto the native executor (lowering.py).  The
        model owns one device parameter set; every (batch size, dtype) view
        returned here shares it.  dtype None: the executor's own precision
        (bfloat16 for single-stage nets, float32 for multi-stage ones)."""
        from .lowering import NativeModel
        if self._native is None:
            self._native = NativeModel(self, device)
        return self._native.view(batch_size, dtype)

    def predict(self, x, batch_size=None, dtype=None):
        """Softmax outputs for images `x` (numpy or device, NHWC), in batches
        of `batch_size` (default: min(len(x), 256), so the executor's
        training-sized workspace stays bounded)."""
        n = int(x.shape[0])
        bs = int(batch_size or min(n, 256))
        return self.compile_native(bs, dtype).predict(x)

    def __call__(self, *args, **kwargs):
        raise TypeError("Model objects are executed with predict()/Training, not called as layers")
