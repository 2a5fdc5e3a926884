"""Lowering of a graph Model onto the native executor (asr_net_*).

The pattern recognised is the reference's single-block ResNet as built by
get_single_block_resnet_build_function with one stage of identity blocks
(tfkeras_resnets.py:547-597), which is what every antisymmetric experiment
runs (_v6.ipynb cells 5-9):

    Input -> Lambda* (elementwise affine: identity / x-mean / x/std)
          -> Conv2D 3x3 'same' stride 1 (conv1) -> relu
          -> L x [ conv 3x3 (Conv2DAntisymmetric3By3 | Conv2DAntisymmetric(k=3) | Conv2D)
                   -> relu -> Lambda(h*x)? -> add(branch, block input) ]
          -> GlobalAveragePooling2D -> Dense(K, softmax)

or, with integrator="rk2" (extension, BASELINE config 5), every block as
the midpoint step built by single_layer_identity_block:

          xm = add(Lambda(h/2*x)?(relu(conv(x))), x);  add(Lambda(h*x)?(relu(conv(xm))), x)

with the SAME conv layer applied twice.

With num_stages > 2 (e.g. the He-style ResNet-32, blocks [10, 10, 10] at
32^2 x 16, 16^2 x 32, 8^2 x 64; tfkeras_resnets.py:575-593) a stage whose
filters or stride change opens with single_layer_conv_block
(tfkeras_resnets.py:204-269):

          add(relu(Conv2D 3x3 'same' stride s (..._branch2)), Conv2D 1x1 'valid' stride s (..._branch1))

and the model lowers onto the multi-stage executor (asr_stages_*, fp32,
Euler blocks) as a StagesPlan.

Anything else (BN, pooling, strided stem, non-3x3 convs, per-block differing
h/gamma/integrator, RK2 blocks in a multi-stage net) raises AsrUnsupported
naming the layer: there is no fallback executor.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import warnings

import numpy as np

from . import _lib
from .graph import (Activation, Add, Conv2D, Dense, GlobalAveragePooling2D, InputLayer, Lambda, Model,
                    SymbolicTensor)
from .layers._antisymmetric import AntisymmetricConvBase

__all__ = ["NetPlan", "StagesPlan", "analyze", "NativeModel"]


@dataclass
class NetPlan:
    H: int
    W: int
    Cin: int
    C: int
    L: int
    num_classes: int
    h: float
    gamma: float
    subtract_mean: float | None
    divide_by_stddev: float | None
    param_kind: int
    antisymmetric: bool
    integrator: str = "euler"
    conv1: Conv2D = None
    blocks: list = field(default_factory=list)
    fc: Dense = None

    def weight_vars(self):
        """Variables in the executor's flat order (Keras get_weights order)."""
        out = [self.conv1.kernel, self.conv1.bias]
        for conv in self.blocks:
            out += conv.weights
        out += [self.fc.kernel, self.fc.bias]
        return out

    def block_theta_sizes(self):
        """Per block: number of theta (kernel) floats, excluding the bias."""
        return [sum(v.value.size for v in conv.weights) - self.C for conv in self.blocks]


@dataclass
class StagesPlan:
    """A multi-stage single-block ResNet (asr_stages_config): stage 0 holds
    conv1's filters; every later stage may open with a transition."""
    H: int
    W: int
    Cin: int
    num_classes: int
    h: float
    gamma: float
    subtract_mean: float | None
    divide_by_stddev: float | None
    param_kind: int
    antisymmetric: bool
    stages: list                 # [(C, L, stride)], stride 0 = no transition
    transitions: list            # per stage: None or (conv_3x3 '..._branch2', conv_1x1 '..._branch1')
    stage_blocks: list           # per stage: the identity blocks' convs
    integrator: str = "euler"
    conv1: Conv2D = None
    fc: Dense = None

    @property
    def blocks(self):
        return [b for bl in self.stage_blocks for b in bl]

    @property
    def L(self):
        return len(self.blocks)

    @property
    def C(self):
        return self.stages[-1][0]

    def stages_bf16_ok(self):
        """Whether the bf16 block kernels take every stage with blocks (C in
        {16, 32, 64}, W in {32, 16, 8}; asr_stages_config.dtype)."""
        W = self.W
        for C, L, S in self.stages:
            if S:
                W = (W + S - 1) // S
            if L > 0 and (C not in (16, 32, 64) or W not in (32, 16, 8)):
                return False
            if C % 8:
                return False
        return True

    def weight_vars(self):
        """Variables in the executor's flat order (asr_stages_config)."""
        out = [self.conv1.kernel, self.conv1.bias]
        for tr, blocks in zip(self.transitions, self.stage_blocks):
            if tr is not None:
                c2, c1 = tr
                out += [c2.kernel, c2.bias, c1.kernel, c1.bias]
            for conv in blocks:
                out += conv.weights
        out += [self.fc.kernel, self.fc.bias]
        return out


def _transition(t: SymbolicTensor):
    """Match t = add(relu(conv_3x3(x)), conv_1x1(x)) (single_layer_conv_block,
    tfkeras_resnets.py:238-269); return (conv_3x3, conv_1x1, x) or None."""
    if len(t.inbound) != 2:
        return None
    branch, short = t.inbound
    if not (isinstance(short.layer, Conv2D) and short.layer.kernel_size == (1, 1) and _is_relu(branch)
            and isinstance(branch.inbound[0].layer, Conv2D)):
        return None
    c2, c1 = branch.inbound[0].layer, short.layer
    x = short.inbound[0]
    if branch.inbound[0].inbound[0] is not x:
        raise _unsupported(t.layer, "transition branches must read the same tensor")
    if c2.kernel_size != (3, 3) or c2.padding != "same" or not c2.use_bias or c2.activation not in (None, "linear"):
        raise _unsupported(c2, "transition conv must be a 3x3 'same' conv with bias, no activation")
    if c1.padding != "valid" or not c1.use_bias or c1.activation not in (None, "linear"):
        raise _unsupported(c1, "transition shortcut must be a 1x1 'valid' conv with bias")
    if c2.strides != c1.strides or c2.strides[0] != c2.strides[1] or c2.strides[0] not in (1, 2):
        raise _unsupported(c2, f"transition strides {c2.strides} / {c1.strides} (equal, 1 or 2)")
    if c2.dilation_rate != (1, 1) or c1.dilation_rate != (1, 1) or c2.filters != c1.filters:
        raise _unsupported(c2, "transition convs must be undilated with equal filters")
    return c2, c1, x


def _unsupported(layer, why):
    return _lib.AsrUnsupported(f"cannot lower layer {layer.name} ({type(layer).__name__}): {why}")


def _is_relu(t: SymbolicTensor):
    return isinstance(t.layer, Activation) and t.layer.activation == "relu"


def _affine_scalar(layer: Lambda, shape):
    aff = layer.affine(shape[1:])
    if aff is None:
        raise _unsupported(layer, "not an elementwise affine function")
    s, t = aff
    if not (np.all(s == s.flat[0]) and np.all(t == t.flat[0])):
        raise _unsupported(layer, "per-element/per-channel normalisation (the native stem takes scalars)")
    return float(s.flat[0]), float(t.flat[0])


def _conv3x3_same(layer: Conv2D, what):
    if layer.kernel_size != (3, 3) or layer.strides != (1, 1) or layer.padding != "same" or not layer.use_bias:
        raise _unsupported(layer, f"{what} must be a 3x3 'same' stride-1 conv with bias")
    if layer.dilation_rate != (1, 1):
        raise _unsupported(layer, "dilated conv")


def _euler_step(t: SymbolicTensor):
    """Match t = add(Lambda(h*x)?(relu(conv(inner))), skip); return (conv, h, inner)."""
    if len(t.inbound) != 2:
        raise _unsupported(t.layer, "add of more than two tensors")
    branch, skip = t.inbound
    h = 1.0
    if isinstance(branch.layer, Lambda):
        s, off = _affine_scalar(branch.layer, branch.shape)
        if off != 0.0:
            raise _unsupported(branch.layer, "block scaling must be h*x")
        h = s
        branch = branch.inbound[0]
    if not _is_relu(branch):
        raise _unsupported(branch.layer, "expected relu in the block branch (BN is not supported)")
    conv_t = branch.inbound[0]
    conv = conv_t.layer
    if isinstance(conv, AntisymmetricConvBase):
        if conv.kernel_size != 3 or tuple(conv.strides) != (1, 1) or not conv.use_bias:
            raise _unsupported(conv, "antisymmetric block conv must be 3x3, stride 1, with bias")
    elif isinstance(conv, Conv2D):
        _conv3x3_same(conv, "regular block conv")
        if conv.activation not in (None, "linear"):
            raise _unsupported(conv, "conv activation inside an identity block")
    else:
        raise _unsupported(conv, "unsupported block conv")
    return conv, h, conv_t.inbound[0]


def analyze(model: Model) -> NetPlan:
    if len(model.inputs) != 1 or len(model.outputs) != 1:
        raise _lib.AsrUnsupported("the native executor runs single-input single-output models")
    t = model.outputs[0]
    # head: Dense(K, softmax) <- GAP
    if not isinstance(t.layer, Dense):
        raise _unsupported(t.layer, "model output must be the Dense 'fc' layer (include_top=True)")
    fc = t.layer
    if fc.activation != "softmax" or not fc.use_bias:
        raise _unsupported(fc, "the head must be Dense(num_classes, activation='softmax') with bias")
    t = t.inbound[0]
    if not isinstance(t.layer, GlobalAveragePooling2D):
        raise _unsupported(t.layer, "expected GlobalAveragePooling2D before fc")
    t = t.inbound[0]
    # identity blocks (and stage transitions), last to first
    blocks, hs, integ = [], [], []
    segs = []  # completed stages, top first: (transition, blocks top first)
    while isinstance(t.layer, Add):
        tr = _transition(t)
        if tr is not None:
            segs.append(((tr[0], tr[1]), blocks))
            blocks = []
            t = tr[2]
            continue
        conv, h, inner = _euler_step(t)
        skip = t.inbound[1]
        if inner is skip:
            integ.append("euler")
        else:
            # RK2: the conv's input is the midpoint xm = x + (h/2) relu(conv(x))
            if not isinstance(inner.layer, Add) or inner.inbound[1] is not skip:
                raise _unsupported(conv, "block branch must start at the block input (or its RK2 midpoint)")
            conv1_, h1, inner1 = _euler_step(inner)
            if conv1_ is not conv or inner1 is not skip:
                raise _unsupported(inner.layer, "RK2 midpoint must apply the block's own conv to the block input")
            if abs(h1 - 0.5 * h) > 1e-12 * max(1.0, abs(h)):
                raise _unsupported(inner.layer, f"RK2 midpoint scale {h1} is not h/2 (h = {h})")
            integ.append("rk2")
        blocks.append(conv)
        hs.append(h)
        t = skip
    segs.append((None, blocks))
    segs.reverse()
    blocks = [b for _, bl in segs for b in reversed(bl)]
    hs.reverse()
    if not blocks:
        raise _lib.AsrUnsupported("no identity blocks found")
    # stem: relu <- conv1 <- Lambda* <- Input
    if _is_relu(t):
        t = t.inbound[0]
        if not isinstance(t.layer, Conv2D) or t.layer.activation not in (None, "linear"):
            raise _unsupported(t.layer, "expected conv1 before the stem relu (BN is not supported)")
    elif not (isinstance(t.layer, Conv2D) and t.layer.activation == "relu"):
        raise _unsupported(t.layer, "expected relu(conv1) before the first block")
    conv1 = t.layer
    _conv3x3_same(conv1, "conv1")
    t = t.inbound[0]
    scale, shift = 1.0, 0.0
    while isinstance(t.layer, Lambda):
        s, off = _affine_scalar(t.layer, t.shape)
        scale, shift = scale * s, scale * off + shift  # walking backwards: acc o f
        t = t.inbound[0]
    if not isinstance(t.layer, InputLayer):
        raise _unsupported(t.layer, "unsupported stem layer")
    _, H, W, Cin = t.shape
    C = conv1.filters
    if scale == 0.0:
        raise _lib.AsrUnsupported("input normalisation scales by zero")
    # executor: (v - mean) * (1/std) == scale*v + shift
    mean = None if (scale == 1.0 and shift == 0.0) else -shift / scale
    std = None if mean is None else 1.0 / scale
    first = blocks[0]
    kinds = {(type(b), getattr(b, "param_kind", _lib.ASR_PARAM_REGULAR), getattr(b, "antisymmetric", False),
              float(getattr(b, "gamma", 0.0))) for b in blocks}
    if len(kinds) != 1 or len(set(hs)) != 1 or len(set(integ)) != 1:
        raise _lib.AsrUnsupported("all identity blocks must share conv type, gamma, h and integrator")
    if isinstance(first, AntisymmetricConvBase):
        kind, anti, gamma = first.param_kind, bool(first.antisymmetric), float(first.gamma)
    else:
        kind, anti, gamma = _lib.ASR_PARAM_REGULAR, False, 0.0
    if len(segs) > 1:
        return _stages_plan(segs, int(H), int(W), int(Cin), int(C), fc, float(hs[0]), gamma, mean, std, kind, anti,
                            integ[0], conv1)
    plan = NetPlan(H=int(H), W=int(W), Cin=int(Cin), C=int(C), L=len(blocks), num_classes=fc.units, h=float(hs[0]),
                   gamma=gamma, subtract_mean=mean, divide_by_stddev=std, param_kind=kind, antisymmetric=anti,
                   integrator=integ[0], conv1=conv1, blocks=blocks, fc=fc)
    for b in blocks:
        if b.weights[-1].shape != (C,):
            raise _unsupported(b, f"block channels must equal conv1 filters ({C})")
    return plan


def _stages_plan(segs, H, W, Cin, C0, fc, h, gamma, mean, std, kind, anti, integrator, conv1) -> StagesPlan:
    if integrator != "euler":
        raise _lib.AsrUnsupported("multi-stage nets run Euler identity blocks (integrator='rk2' is single-stage)")
    if len(segs) > _lib.ASR_STAGES_MAX:
        raise _lib.AsrUnsupported(f"{len(segs)} stages (at most {_lib.ASR_STAGES_MAX})")
    stages, transitions, stage_blocks = [], [], []
    Cp = C0
    for s, (tr, bl) in enumerate(segs):
        bl = list(reversed(bl))
        if tr is None:
            C, S = Cp, 0
        else:
            C, S = tr[0].filters, tr[0].strides[0]
        for b in bl:
            if b.weights[-1].shape != (C,):
                raise _unsupported(b, f"block channels must equal the stage's filters ({C})")
        stages.append((C, len(bl), S))
        transitions.append(tr)
        stage_blocks.append(bl)
        Cp = C
    return StagesPlan(H=H, W=W, Cin=Cin, num_classes=fc.units, h=h, gamma=gamma, subtract_mean=mean,
                      divide_by_stddev=std, param_kind=kind, antisymmetric=anti, stages=stages,
                      transitions=transitions, stage_blocks=stage_blocks, integrator=integrator, conv1=conv1, fc=fc)


class NativeModel:
    """The device state of one Model lowered onto the native executor.

    ONE instance per Model owns the flat fp32 device parameters (Keras
    order), the Adam moments and step, and every executor built for it,
    keyed by (batch size, activation dtype, input kind) — so a predict() at
    another batch size or dtype reads the trained parameters and a
    set_weights()/load_variables() reaches every executor.  Host-side
    Variables and the device buffer are kept coherent through
    push_weights/pull_weights.  Callers use views (view(batch, dtype)) that
    fix the batch size and dtype of their calls."""

    def __init__(self, model: Model, device=None):
        from . import runtime
        import torch
        self.model = model
        self.plan = analyze(model)
        self.device = device or runtime.require_gpu()
        self._torch = torch
        self._rt = runtime
        self._executors = {}
        self._warned_stages_dtype = False
        self.vars = self.plan.weight_vars()
        self.n_params = int(sum(v.value.size for v in self.vars))
        self.params = torch.empty(self.n_params, dtype=torch.float32, device=self.device)
        self.m = None
        self.v = None
        self.step = 0
        self._host_stale = False
        self.push_weights()

    def resolve_dtype(self, dtype):
        """The activation dtype an executor of this model runs in.  None: the
        plan's own (bfloat16 single-stage, float32 multi-stage: the reference's
        precision).  A multi-stage net runs in bfloat16 when asked and every
        stage with blocks is on the bf16 kernels' shapes (stages_bf16_ok);
        otherwise the request is warned about once and mapped to float32, so
        train and predict views share one executor per batch size."""
        if isinstance(self.plan, StagesPlan):
            if dtype in (None, "float32"):
                return "float32"
            if dtype == "bfloat16" and self.plan.stages_bf16_ok():
                return "bfloat16"
            if not self._warned_stages_dtype:
                warnings.warn(f"this multi-stage net runs in float32 on the native executor (dtype={dtype!r} "
                              "requested: bf16 needs C in {16, 32, 64} and W in {32, 16, 8} at every stage with "
                              "blocks)", stacklevel=3)
                self._warned_stages_dtype = True
            return "float32"
        return "bfloat16" if dtype is None else dtype

    def view(self, batch_size: int, dtype=None) -> "NativeView":
        return NativeView(self, int(batch_size), self.resolve_dtype(dtype))

    def check_status(self):
        """Blocking: synchronise and check every executor built for this model
        (a failed launch raises AsrError)."""
        for ex in self._executors.values():
            ex.check_status()

    # -- weights ---------------------------------------------------------------
    def push_weights(self):
        flat = np.concatenate([v.value.ravel() for v in self.vars]).astype(np.float32)
        self.params.copy_(self._torch.from_numpy(flat))
        self._host_stale = False

    def pull_weights(self):
        if not self._host_stale:
            return
        flat = self.params.detach().cpu().numpy()
        off = 0
        for v in self.vars:
            n = v.value.size
            v.assign(flat[off:off + n].reshape(v.shape))
            off += n
        for layer in self.model.layers:
            layer._weights_changed()
        self._host_stale = False

    def mark_updated(self):
        self._host_stale = True

    # -- execution ---------------------------------------------------------------
    def executor(self, batch_size: int, dtype, input_u8: bool, inference: bool = False):
        """The executor for (batch, dtype, input kind); inference=True gives the
        forward-only one (bounded workspace: x_0 + two activation slots)."""
        dtype = self.resolve_dtype(dtype)
        key = (int(batch_size), dtype, bool(input_u8), bool(inference))
        ex = self._executors.get(key)
        if ex is None and isinstance(self.plan, StagesPlan):
            p = self.plan
            ex = self._rt.StagesExecutor(int(batch_size), p.H, p.W, p.Cin, p.stages, p.num_classes, p.h, p.gamma,
                                         subtract_mean=p.subtract_mean, divide_by_stddev=p.divide_by_stddev,
                                         dtype=dtype, input_u8=input_u8, device=self.device,
                                         param_kind=p.param_kind, antisymmetric=p.antisymmetric, inference=inference)
            if ex.n_params != self.n_params:
                raise _lib.AsrError(f"executor expects {ex.n_params} parameters, model has {self.n_params}")
            self._executors[key] = ex
        if ex is None:
            p = self.plan
            ex = self._rt.NetExecutor(int(batch_size), p.H, p.W, p.Cin, p.C, p.L, p.num_classes, p.h, p.gamma,
                                      subtract_mean=p.subtract_mean, divide_by_stddev=p.divide_by_stddev,
                                      dtype=dtype, input_u8=input_u8, device=self.device,
                                      param_kind=p.param_kind, antisymmetric=p.antisymmetric,
                                      integrator=p.integrator, inference=inference)
            if ex.n_params != self.n_params:
                raise _lib.AsrError(f"executor expects {ex.n_params} parameters, model has {self.n_params}")
            self._executors[key] = ex
        return ex

    def _images(self, x):
        torch = self._torch
        if isinstance(x, np.ndarray):
            x = torch.from_numpy(np.ascontiguousarray(x))
        if x.dtype not in (torch.uint8, torch.float32):
            x = x.float()
        return x.to(self.device, non_blocking=True).contiguous()

    def apply_adam(self, grads, lr, beta1=0.9, beta2=0.999, epsilon=1e-7, grad_scale=1.0):
        torch = self._torch
        if self.m is None:
            self.m = torch.zeros_like(self.params)
            self.v = torch.zeros_like(self.params)
        self.step += 1
        self._rt.adam_update(self.params, grads, self.m, self.v, lr, beta1, beta2, epsilon, self.step, grad_scale)
        self._host_stale = True


class NativeView:
    """A NativeModel at a fixed batch size and dtype.  Everything else
    (parameters, Adam state, weight sync) is the shared NativeModel's."""

    _SHARED = ("params", "m", "v", "step")

    def __init__(self, state: NativeModel, batch_size: int, dtype):
        object.__setattr__(self, "state", state)
        object.__setattr__(self, "batch_size", int(batch_size))
        object.__setattr__(self, "dtype", dtype)

    def __getattr__(self, name):
        return getattr(self.state, name)

    def __setattr__(self, name, value):
        if name in self._SHARED:
            setattr(self.state, name, value)
        else:
            object.__setattr__(self, name, value)

    def matches(self, batch_size, dtype):
        return self.batch_size == int(batch_size) and self.dtype == self.state.resolve_dtype(dtype)

    def executor(self, input_u8: bool, inference: bool = False):
        return self.state.executor(self.batch_size, self.dtype, input_u8, inference)

    def predict(self, x):
        """Softmax outputs [n, K] (numpy) for n images, in batches of
        batch_size (the last batch is zero-padded), on the forward-only
        executor: device memory is one batch of images plus the inference
        workspace, whatever n is (host arrays are copied batch by batch)."""
        torch = self._torch
        if isinstance(x, np.ndarray):
            x = torch.from_numpy(np.ascontiguousarray(x))
        if x.dtype not in (torch.uint8, torch.float32):
            x = x.float()
        n = int(x.shape[0])
        ex = self.executor(x.dtype == torch.uint8, inference=True)
        out = np.empty((n, ex.cfg.num_classes), dtype=np.float32)
        B = self.batch_size
        buf = torch.zeros((B,) + tuple(x.shape[1:]), dtype=x.dtype, device=self.device)
        for i in range(0, n, B):
            m = min(B, n - i)
            buf[:m].copy_(x[i:i + m])
            if m < B:
                buf[m:].zero_()
            out[i:i + m] = ex.forward(self.params, buf)[:m].cpu().numpy()
        return out

    def forward_backward(self, images, targets, want_probs=False):
        """(loss, grads, probs): loss [1] and grads [n_params] are views of
        executor buffers, overwritten by the next call."""
        torch = self._torch
        x = self._images(images)
        if isinstance(targets, np.ndarray):
            targets = torch.from_numpy(np.ascontiguousarray(targets, dtype=np.float32))
        targets = targets.to(self.device, non_blocking=True).float().contiguous()
        ex = self.executor(x.dtype == torch.uint8)
        loss, grads = ex.forward_backward(self.params, x, targets, want_probs=want_probs)
        return loss, grads, ex.probs
