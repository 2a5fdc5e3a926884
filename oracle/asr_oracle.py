"""numpy restatement of the reference's antisymmetric-ResNet hot path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Every function cites the
reference file:line it restates.  All arithmetic is float64 unless the caller
passes float32 arrays and asks for dtype=np.float32.

Conventions (pinned by the reference notebook KAT, tests/golden/kat_conv7x7.json):
  activations NHWC, kernels HWIO [kh, kw, C_in, C_out], tf.nn.conv2d(padding
  "SAME") == zero-padded CROSS-correlation (no kernel flip).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# --------------------------------------------------------------------------
# parameter layouts ("reference order" = Keras add_weight order)
# --------------------------------------------------------------------------


def theta_count_3by3(C: int) -> int:
    """Number of free kernel parameters of Conv2DAntisymmetric3By3 (no bias).

    a,b,c,d: [1,1,1,C] each (…3By3.py:219-245); then for o = 0..C-2
    `input_kernels_for_output_kernel_{o}` [3,3,C-o-1] (…3By3.py:115-124).
    """
    return 4 * C + 9 * C * (C - 1) // 2


def theta_shapes_3by3(C: int):
    """Shapes of the layer's weights in reference order (excluding bias)."""
    shapes = [(1, 1, 1, C)] * 4
    for o in range(C - 1):
        shapes.append((3, 3, C - o - 1))
    return shapes


def theta_names_3by3(C: int):
    names = ["a", "b", "c", "d"]
    names += ["input_kernels_for_output_kernel_{}".format(o) for o in range(C - 1)]
    return names


def _cs_free_positions(k: int, antisymmetric: bool):
    """Free (trainable) positions of the general layer's diagonal block, in
    variable-creation order (…Conv2DAntisymmetric.py:231-264)."""
    pos = []
    for i in range(k):
        for j in range(i, k):
            if j > i or (j == i and i <= k // 2 - 1):
                pos.append((i, j))
            elif j == i and i == k // 2 and k % 2 == 1:
                if not antisymmetric:
                    pos.append((i, j))
    return pos


def theta_shapes_general(C: int, k: int = 3, antisymmetric: bool = True):
    """Weights of Conv2DAntisymmetric in reference order (no bias): per output
    channel o, the scalar `centro_sym_{i}_{j}` variables [1,1,1,1] in creation
    order, then `input_kernels_for_output_kernel_{o}` [k,k,C-o-1,1]
    (…Conv2DAntisymmetric.py:117-143)."""
    shapes, names = [], []
    free = _cs_free_positions(k, antisymmetric)
    for o in range(C):
        for (i, j) in free:
            shapes.append((1, 1, 1, 1))
            names.append("centro_sym_{}_{}".format(i, j))
        if C - o - 1 > 0:
            shapes.append((k, k, C - o - 1, 1))
            names.append("input_kernels_for_output_kernel_{}".format(o))
    return shapes, names


def theta_count_general(C: int, k: int = 3, antisymmetric: bool = True) -> int:
    shapes, _ = theta_shapes_general(C, k, antisymmetric)
    return int(sum(np.prod(s) for s in shapes))


def flatten(arrays) -> np.ndarray:
    return np.concatenate([np.asarray(a).ravel() for a in arrays]) if len(arrays) else np.zeros(0)


def unflatten(flat, shapes):
    out, off = [], 0
    for s in shapes:
        n = int(np.prod(s))
        out.append(np.asarray(flat[off:off + n]).reshape(s))
        off += n
    assert off == len(flat), (off, len(flat))
    return out


def truncated_normal(rng, shape, stddev, dtype=np.float64):
    """tf.initializers.truncated_normal: N(0, stddev) re-drawn outside 2 sigma
    (…3By3.py:95-98)."""
    out = rng.standard_normal(size=shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(size=int(bad.sum()))
        bad = np.abs(out) > 2.0
    return (out * stddev).astype(dtype)


def init_theta_3by3(C: int, rng, dtype=np.float64):
    """He-style init of the reference layer: truncated normal, stddev
    sqrt(2/(3*3*C)) for every kernel variable (…3By3.py:95-98)."""
    std = math.sqrt(2.0 / (9 * C))
    return [truncated_normal(rng, s, std, dtype) for s in theta_shapes_3by3(C)]


# --------------------------------------------------------------------------
# kernel assembly
# --------------------------------------------------------------------------


def anti_centrosymmetric_kernel(a, b, c, d, gamma):
    """`_get_anti_centrosymmetric_kernel` (…3By3.py:210-275): per channel
    [[a, b, c], [d, gamma, -d], [-c, -b, -a]], shape [3,3,1,C]."""
    a, b, c, d = (np.asarray(v).reshape(1, 1, 1, -1) for v in (a, b, c, d))
    e = np.full_like(a, gamma)
    row1 = np.concatenate([a, b, c], axis=1)
    row2 = np.concatenate([d, e, -d], axis=1)
    row3 = np.concatenate([-c, -b, -a], axis=1)
    return np.concatenate([row1, row2, row3], axis=0)


def anti_centrosymmetric_transpose(t):
    """`_get_anti_centrosymmetric_transpose` (…3By3.py:277-293):
    out[ky,kx,:] = -t[2-ky, 2-kx, :]."""
    t = np.asarray(t)
    a, b, c = -t[0, 0, :], -t[0, 1, :], -t[0, 2, :]
    d, e, f = -t[1, 0, :], -t[1, 1, :], -t[1, 2, :]
    g, h, i = -t[2, 0, :], -t[2, 1, :], -t[2, 2, :]
    row1 = np.stack([i, h, g], axis=0)
    row2 = np.stack([f, e, d], axis=0)
    row3 = np.stack([c, b, a], axis=0)
    return np.stack([row1, row2, row3], axis=0)


def assemble_3by3_literal(theta_list, gamma=0.0):
    """Literal restatement of the build loop (…3By3.py:104-141): returns the
    HWIO kernel [3,3,C,C] exactly as `self.kernel`."""
    a, b, c, d = theta_list[:4]
    C = np.asarray(a).size
    indeps = theta_list[4:]
    assert len(indeps) == C - 1
    acs = anti_centrosymmetric_kernel(a, b, c, d, gamma)  # (3,3,1,C)
    single_output_kernels, transposes = [], []
    for o in range(C):
        nind = C - o - 1
        if nind > 0:
            ind = np.asarray(indeps[o])
            act = anti_centrosymmetric_transpose(ind)
            single = np.concatenate([acs[:, :, :, o], ind], axis=-1)
        else:
            single = acs[:, :, :, o]
        for i in range(o):
            ct = np.expand_dims(transposes[-(i + 1)][:, :, i], axis=-1)
            single = np.concatenate([ct, single], axis=-1)
        single_output_kernels.append(single)
        if nind > 0:
            transposes.append(act)
    return np.stack(single_output_kernels, axis=-1)


def assemble_general_literal(theta_list, C, k=3, gamma=0.0, antisymmetric=True):
    """Literal restatement of Conv2DAntisymmetric.build (…Conv2DAntisymmetric.py:109-145)
    from its weights in reference order (see theta_shapes_general)."""
    J = np.eye(k)[::-1]
    free = _cs_free_positions(k, antisymmetric)
    it = iter(theta_list)
    single_output_kernels, independent = [], []
    for o in range(C):
        # _get_centrosymmetric_matrix (…Conv2DAntisymmetric.py:216-270)
        arr = np.zeros((k, k))
        for i in range(k):
            for j in range(i, k):
                if j > i or (j == i and i <= k // 2 - 1):
                    v = float(np.asarray(next(it)).ravel()[0])
                    arr[i, j] = v
                    arr[k - 1 - i, k - 1 - j] = -v if antisymmetric else v
                elif j == i and i == k // 2 and k % 2 == 1:
                    if antisymmetric:
                        arr[i, j] = gamma
                    else:
                        arr[i, j] = float(np.asarray(next(it)).ravel()[0])
        cs = arr.reshape(k, k, 1, 1)
        nind = C - o - 1
        if nind > 0:
            ind = np.asarray(next(it)).reshape(k, k, nind, 1)
            single = np.concatenate([cs, ind], axis=2)
        else:
            single = cs
        for i in range(o):
            ct = -(J @ (independent[-(i + 1)][:, :, i, 0] @ J))
            single = np.concatenate([ct[:, :, None, None], single], axis=2)
        single_output_kernels.append(single)
        if nind > 0:
            independent.append(ind)
    assert next(it, None) is None
    del free
    return np.concatenate(single_output_kernels, axis=3)


# Param map: for every W element (HWIO flat index e = ((ky*k+kx)*C+i)*C+o) the
# theta index it is read from and its sign; special values for the centre.
MAP_GAMMA = -1  # element equals gamma (non-trainable centre)


def param_map(C, kind="3by3", k=3, antisymmetric=True):
    """(src, sign) arrays of length k*k*C*C: W.flat[e] = sign[e]*theta[src[e]]
    or gamma where src[e] == MAP_GAMMA.  Derived from the assembly loops
    (…3By3.py:104-141, …Conv2DAntisymmetric.py:117-145)."""
    src = np.full((k, k, C, C), MAP_GAMMA, dtype=np.int64)
    sign = np.ones((k, k, C, C), dtype=np.int64)
    if kind == "3by3":
        assert k == 3 and antisymmetric
        base_ind = []
        off = 4 * C
        for o in range(C - 1):
            base_ind.append(off)
            off += 9 * (C - o - 1)
        diag = {(0, 0): (0, 1), (0, 1): (1, 1), (0, 2): (2, 1), (1, 0): (3, 1),
                (1, 2): (3, -1), (2, 0): (2, -1), (2, 1): (1, -1), (2, 2): (0, -1)}
        for o in range(C):
            for (ky, kx), (v, sg) in diag.items():
                src[ky, kx, o, o] = v * C + o
                sign[ky, kx, o, o] = sg
            for i in range(o + 1, C):  # W[:,:,i,o] = indep_o[:,:,i-o-1]
                m = i - o - 1
                for ky in range(3):
                    for kx in range(3):
                        src[ky, kx, i, o] = base_ind[o] + (ky * 3 + kx) * (C - o - 1) + m
                        src[2 - ky, 2 - kx, o, i] = src[ky, kx, i, o]
                        sign[2 - ky, 2 - kx, o, i] = -1
    elif kind == "general":
        free = _cs_free_positions(k, antisymmetric)
        off = 0
        base_cs, base_ind = [], []
        for o in range(C):
            base_cs.append(off)
            off += len(free)
            if C - o - 1 > 0:
                base_ind.append(off)
                off += k * k * (C - o - 1)
        for o in range(C):
            for n, (i, j) in enumerate(free):
                src[i, j, o, o] = base_cs[o] + n
                sign[i, j, o, o] = 1
                mi, mj = k - 1 - i, k - 1 - j
                if (mi, mj) != (i, j):
                    src[mi, mj, o, o] = base_cs[o] + n
                    sign[mi, mj, o, o] = -1 if antisymmetric else 1
            for i in range(o + 1, C):
                m = i - o - 1
                for ky in range(k):
                    for kx in range(k):
                        # indep shape [k,k,nind,1]
                        s = base_ind[o] + (ky * k + kx) * (C - o - 1) + m
                        src[ky, kx, i, o] = s
                        src[k - 1 - ky, k - 1 - kx, o, i] = s
                        sign[k - 1 - ky, k - 1 - kx, o, i] = -1
    else:
        raise ValueError(kind)
    return src.ravel(), sign.ravel()


def assemble_from_map(theta_flat, C, src, sign, gamma=0.0, k=3):
    theta_flat = np.asarray(theta_flat)
    W = np.where(src >= 0, sign * theta_flat[np.maximum(src, 0)], gamma)
    return W.reshape(k, k, C, C).astype(theta_flat.dtype)


def project_dW(dW, src, sign, n_theta):
    """Gradient of W(theta) pulled back onto theta (the autodiff of the
    slice/neg/concat/stack assembly, training.py:300 via …3By3.py:115-141):
    dtheta[j] = sum over W elements e with src[e]==j of sign[e]*dW[e]."""
    dW = np.asarray(dW).ravel()
    m = src >= 0
    out = np.zeros(n_theta, dtype=np.float64)
    np.add.at(out, src[m], sign[m] * dW[m])
    return out


# --------------------------------------------------------------------------
# conv + Euler block
# --------------------------------------------------------------------------


def conv2d_same(x, W, stride=1):
    """tf.nn.conv2d(x, W, strides=[1,s,s,1], padding="SAME", NHWC) as called at
    …3By3.py:159-166: zero-padded cross-correlation."""
    x = np.asarray(x)
    W = np.asarray(W)
    N, H, Wd, Ci = x.shape
    kh, kw, Ci2, Co = W.shape
    assert Ci == Ci2
    Ho, Wo = -(-H // stride), -(-Wd // stride)
    pad_h = max((Ho - 1) * stride + kh - H, 0)
    pad_w = max((Wo - 1) * stride + kw - Wd, 0)
    pt, pl = pad_h // 2, pad_w // 2
    xp = np.zeros((N, H + pad_h, Wd + pad_w, Ci), dtype=np.result_type(x, W))
    xp[:, pt:pt + H, pl:pl + Wd, :] = x
    out = np.zeros((N, Ho, Wo, Co), dtype=np.result_type(x, W))
    for ky in range(kh):
        for kx in range(kw):
            patch = xp[:, ky:ky + (Ho - 1) * stride + 1:stride, kx:kx + (Wo - 1) * stride + 1:stride, :]
            out += patch @ W[ky, kx]
    return out


def conv2d_backprop_input(dz, W, x_shape):
    """Conv2DBackpropInput for stride 1 SAME (generic transpose, no antisymmetry
    assumed): dx[q,i] = sum_{s,o} W[s,i,o] dz[q-s,o]."""
    Wt = np.transpose(W[::-1, ::-1], (0, 1, 3, 2))
    return conv2d_same(dz, Wt)


def conv2d_backprop_filter(x, dz, k=3):
    """Conv2DBackpropFilter for stride 1 SAME: dW[ky,kx,i,o] = sum_p x[p+s,i] dz[p,o]."""
    N, H, Wd, Ci = x.shape
    Co = dz.shape[-1]
    p = k // 2
    xp = np.zeros((N, H + 2 * p, Wd + 2 * p, Ci), dtype=np.result_type(x, dz))
    xp[:, p:p + H, p:p + Wd, :] = x
    dW = np.zeros((k, k, Ci, Co), dtype=np.result_type(x, dz))
    dz2 = dz.reshape(-1, Co)
    for ky in range(k):
        for kx in range(k):
            dW[ky, kx] = xp[:, ky:ky + H, kx:kx + Wd, :].reshape(-1, Ci).T @ dz2
    return dW


def euler_fwd(x, W, bias, h):
    """single_layer_identity_block, antisymmetric branch, no BN
    (tfkeras_resnets.py:69-92): z = conv(x) + b (…3By3.py:157-171);
    relu (:89); h*x only if h != 1 (:90-91); + input (:92).  Returns (y, z)."""
    z = conv2d_same(x, W)
    if bias is not None:
        z = z + np.asarray(bias)
    r = np.maximum(z, 0)
    if h != 1.0:
        r = h * r
    return x + r, z


def euler_bwd(dy, x, z, W, h, gamma=0.0):
    """Autodiff of euler_fwd (training.py:300): returns dx, dW, db.
    dz = h*dy*[z>0] (TF ReluGrad uses features > 0);
    dx = dy + A^T dz, with A^T = -A + 2*gamma*I for the assembled W."""
    dzr = dy * (z > 0)
    dz = h * dzr if h != 1.0 else dzr
    dx = dy - conv2d_same(dz, W) + 2.0 * gamma * dz
    dW = conv2d_backprop_filter(x, dz)
    db = dz.sum(axis=(0, 1, 2))
    return dx, dW, db


def euler_bwd_generic(dy, x, z, W, h):
    """Autodiff of euler_fwd for any W (no antisymmetry assumed): dx = dy +
    Conv2DBackpropInput(dz, W)."""
    dzr = dy * (z > 0)
    dz = h * dzr if h != 1.0 else dzr
    dx = dy + conv2d_backprop_input(dz, W, x.shape)
    return dx, conv2d_backprop_filter(x, dz), dz.sum(axis=(0, 1, 2))


def conv_bwd(dz, x, W, gamma=0.0):
    """Backward of the bare layer call (conv + bias): dx = A^T dz, dW, db."""
    dx = -conv2d_same(dz, W) + 2.0 * gamma * dz
    return dx, conv2d_backprop_filter(x, dz), dz.sum(axis=(0, 1, 2))


def rk2_fwd(x, W, bias, h):
    """Extension (not in the reference; BASELINE config 5): explicit midpoint
    step with the same W and bias in both stages, each stage composed of the
    reference's Euler-block operations (tfkeras_resnets.py:69-92):
        xm = x + (h/2) relu(conv(x) + b),   y = x + h relu(conv(xm) + b).
    Returns (y, cache) with cache = (xm, z1, z2)."""
    z1 = conv2d_same(x, W)
    if bias is not None:
        z1 = z1 + np.asarray(bias)
    xm = x + (0.5 * h) * np.maximum(z1, 0)
    z2 = conv2d_same(xm, W)
    if bias is not None:
        z2 = z2 + np.asarray(bias)
    return x + h * np.maximum(z2, 0), (xm, z1, z2)


def rk2_bwd(dy, x, cache, W, h, gamma=0.0, antisymmetric=True):
    """Autodiff of rk2_fwd: dz2 = h dy [z2>0]; g = A^T dz2 (gradient at xm);
    dz1 = (h/2) g [z1>0]; dx = dy + g + A^T dz1; dW = dW(x, dz1) + dW(xm, dz2);
    db = sum(dz1 + dz2).  A^T = -A + 2 gamma I when `antisymmetric`, else the
    generic Conv2DBackpropInput."""
    xm, z1, z2 = cache

    def at(dz):
        if antisymmetric:
            return -conv2d_same(dz, W) + 2.0 * gamma * dz
        return conv2d_backprop_input(dz, W, dz.shape)
    dz2 = h * dy * (z2 > 0)
    g = at(dz2)
    dz1 = (0.5 * h) * g * (z1 > 0)
    dx = dy + g + at(dz1)
    dW = conv2d_backprop_filter(x, dz1) + conv2d_backprop_filter(xm, dz2)
    db = dz1.sum(axis=(0, 1, 2)) + dz2.sum(axis=(0, 1, 2))
    return dx, dW, db


# --------------------------------------------------------------------------
# network: get_single_block_resnet_build_function (tfkeras_resnets.py:511-604)
# restricted to the antisymmetric single-stage topology of the notebooks
# (num_stages=2, strides=[(1,1)], no BN, no pooling)
# --------------------------------------------------------------------------


@dataclass
class NetSpec:
    C: int = 16
    L: int = 18
    h: float = 1.0
    gamma: float = 0.0
    num_classes: int = 10
    H: int = 32
    W: int = 32
    Cin: int = 3
    subtract_mean: float | None = 127.5
    divide_by_stddev: float | None = 127.5
    kind: str = "3by3"           # "3by3" | "general" | "regular" (identity-block conv type)
    antisymmetric: bool = True   # Conv2DAntisymmetric(antisymmetric=...)
    integrator: str = "euler"    # "euler" (the reference) | "rk2" (extension, rk2_fwd)

    def theta_shapes(self):
        """Block conv weights in creation order: Conv2DAntisymmetric3By3
        (…3By3.py:113-124, :219-245), Conv2DAntisymmetric (…Conv2DAntisymmetric.py:117-128,
        :231-264) or the regular Conv2D kernel (tfkeras_resnets.py:76-83)."""
        if self.kind == "3by3":
            return theta_shapes_3by3(self.C)
        if self.kind == "general":
            return theta_shapes_general(self.C, 3, self.antisymmetric)[0]
        if self.kind == "regular":
            return [(3, 3, self.C, self.C)]
        raise ValueError(self.kind)

    def operator_antisymmetric(self):
        return self.kind == "3by3" or (self.kind == "general" and self.antisymmetric)

    def param_shapes(self):
        """Keras `model.get_weights()` order: conv1 kernel/bias, then per
        block [theta..., bias], then fc kernel/bias."""
        s = [(3, 3, self.Cin, self.C), (self.C,)]
        for _ in range(self.L):
            s += self.theta_shapes() + [(self.C,)]
        s += [(self.C, self.num_classes), (self.num_classes,)]
        return s

    def n_params(self):
        return int(sum(np.prod(x) for x in self.param_shapes()))


def init_params(spec: NetSpec, rng, dtype=np.float64, bias_std=0.0):
    """he_normal (truncated, 2 sigma) for kernels, zeros for biases (Keras
    defaults used by the builder, tfkeras_resnets.py:563-572, :595-597)."""
    out = []
    out.append(truncated_normal(rng, (3, 3, spec.Cin, spec.C), math.sqrt(2.0 / (9 * spec.Cin)), dtype))
    out.append(np.zeros(spec.C, dtype) if bias_std == 0 else (rng.standard_normal(spec.C) * bias_std).astype(dtype))
    std = math.sqrt(2.0 / (9 * spec.C))
    for _ in range(spec.L):
        if spec.kind == "3by3":
            out += init_theta_3by3(spec.C, rng, dtype)
        else:
            out += [truncated_normal(rng, sh, std, dtype) for sh in spec.theta_shapes()]
        out.append(np.zeros(spec.C, dtype) if bias_std == 0 else (rng.standard_normal(spec.C) * bias_std).astype(dtype))
    out.append(truncated_normal(rng, (spec.C, spec.num_classes), math.sqrt(2.0 / spec.C), dtype))
    out.append(np.zeros(spec.num_classes, dtype))
    return out


def split_params(spec: NetSpec, params):
    nt = len(spec.theta_shapes())
    conv1_k, conv1_b = params[0], params[1]
    blocks = []
    i = 2
    for _ in range(spec.L):
        blocks.append((params[i:i + nt], params[i + nt]))
        i += nt + 1
    fc_k, fc_b = params[i], params[i + 1]
    return conv1_k, conv1_b, blocks, fc_k, fc_b


def normalize_input(images, spec: NetSpec, dtype=np.float64):
    """Lambda layers identity / x - subtract_mean / x / divide_by_stddev
    (tfkeras_resnets.py:555-559)."""
    x = np.asarray(images).astype(dtype)
    if spec.subtract_mean is not None:
        x = x - spec.subtract_mean
    if spec.divide_by_stddev is not None:
        x = x / spec.divide_by_stddev
    return x


def softmax(logits):
    m = logits.max(axis=-1, keepdims=True)
    e = np.exp(logits - m)
    return e / e.sum(axis=-1, keepdims=True)


KERAS_EPSILON = 1e-7


def keras_cce(probs, onehot):
    """tf.keras.backend.categorical_crossentropy(from_logits=False) as used at
    training.py:295 (TF 1.12): renormalise, clip to [eps, 1-eps], -sum y log p."""
    s = probs.sum(axis=-1, keepdims=True)
    q = probs / s
    qc = np.clip(q, KERAS_EPSILON, 1.0 - KERAS_EPSILON)
    return -(onehot * np.log(qc)).sum(axis=-1)


def keras_cce_grad_logits(probs, onehot, scale):
    """d(scale * sum_n cce_n)/d logits through renorm, clip (TF clip grad passes
    where eps <= q <= 1-eps) and softmax."""
    s = probs.sum(axis=-1, keepdims=True)
    q = probs / s
    inside = (q >= KERAS_EPSILON) & (q <= 1.0 - KERAS_EPSILON)
    qc = np.clip(q, KERAS_EPSILON, 1.0 - KERAS_EPSILON)
    dq = np.where(inside, -onehot / qc, 0.0) * scale
    dp = dq / s - (dq * probs).sum(axis=-1, keepdims=True) / (s * s)
    return probs * (dp - (probs * dp).sum(axis=-1, keepdims=True))


def net_forward(spec: NetSpec, params, images, dtype=np.float64):
    conv1_k, conv1_b, blocks, fc_k, fc_b = split_params(spec, params)
    x0 = normalize_input(images, spec, dtype)
    z1 = conv2d_same(x0, conv1_k) + conv1_b
    x = np.maximum(z1, 0)
    xs, zs, Ws = [x], [], []
    for theta, b in blocks:
        if spec.kind == "3by3" and spec.C <= 32:
            W = assemble_3by3_literal(theta, spec.gamma)
        elif spec.kind == "general" and spec.C <= 32:
            W = assemble_general_literal(theta, spec.C, 3, spec.gamma, spec.antisymmetric)
        elif spec.kind == "regular":
            W = np.asarray(theta[0])
        else:
            src, sign = _cached_map(spec.C, spec.kind, spec.antisymmetric)
            W = assemble_from_map(flatten(theta), spec.C, src, sign, spec.gamma)
        if spec.integrator == "rk2":
            x, z = rk2_fwd(x, W, b, spec.h)
        else:
            x, z = euler_fwd(x, W, b, spec.h)
        xs.append(x)
        zs.append(z)
        Ws.append(W)
    gap = x.mean(axis=(1, 2))
    logits = gap @ fc_k + fc_b
    probs = softmax(logits)
    cache = dict(x0=x0, z1=z1, xs=xs, zs=zs, Ws=Ws, gap=gap, logits=logits, probs=probs)
    return probs, cache


_MAPS = {}


def _cached_map(C, kind="3by3", antisymmetric=True):
    key = (C, kind, antisymmetric)
    if key not in _MAPS:
        if kind == "regular":
            _MAPS[key] = (np.arange(9 * C * C), np.ones(9 * C * C, dtype=np.int64))
        else:
            _MAPS[key] = param_map(C, kind, 3, antisymmetric)
    return _MAPS[key]


def net_loss(probs, onehot):
    return keras_cce(probs, onehot).mean()


def net_backward(spec: NetSpec, params, cache, onehot):
    """Gradients of the mean Keras CE loss w.r.t. every parameter, returned in
    reference (Keras weights) order."""
    conv1_k, conv1_b, blocks, fc_k, fc_b = split_params(spec, params)
    Nb = onehot.shape[0]
    dlogits = keras_cce_grad_logits(cache["probs"], onehot, 1.0 / Nb)
    d_fck = cache["gap"].T @ dlogits
    d_fcb = dlogits.sum(axis=0)
    dgap = dlogits @ fc_k.T
    xL = cache["xs"][-1]
    dx = np.broadcast_to(dgap[:, None, None, :] / (spec.H * spec.W), xL.shape).copy()
    src, sign = _cached_map(spec.C, spec.kind, spec.antisymmetric)
    shapes = spec.theta_shapes()
    ntheta = int(sum(np.prod(x) for x in shapes))
    block_grads = []
    for li in range(spec.L - 1, -1, -1):
        x_in = cache["xs"][li]
        if spec.integrator == "rk2":
            dx, dW, db = rk2_bwd(dx, x_in, cache["zs"][li], cache["Ws"][li], spec.h, spec.gamma,
                                 spec.operator_antisymmetric())
        elif spec.operator_antisymmetric():
            dx, dW, db = euler_bwd(dx, x_in, cache["zs"][li], cache["Ws"][li], spec.h, spec.gamma)
        else:
            dx, dW, db = euler_bwd_generic(dx, x_in, cache["zs"][li], cache["Ws"][li], spec.h)
        dth = project_dW(dW, src, sign, ntheta)
        block_grads.append((unflatten(dth, shapes), db))
    block_grads.reverse()
    dz1 = dx * (cache["z1"] > 0)
    d_c1k = conv2d_backprop_filter(cache["x0"], dz1)
    d_c1b = dz1.sum(axis=(0, 1, 2))
    grads = [d_c1k, d_c1b]
    for dth, db in block_grads:
        grads += dth + [db]
    grads += [d_fck, d_fcb]
    return grads


def adam_tf1(params, grads, m, v, t, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-7):
    """tf.train.AdamOptimizer.apply_gradients (training.py:300-301, epsilon=1e-7
    from _v6.ipynb cell 5): lr_t = lr*sqrt(1-b2^t)/(1-b1^t);
    m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr_t m/(sqrt(v)+eps).
    t is the 1-based step count.  Updates in place; returns (params, m, v)."""
    lr_t = lr * math.sqrt(1.0 - beta2 ** t) / (1.0 - beta1 ** t)
    for p, g, mm, vv in zip(params, grads, m, v):
        mm *= beta1
        mm += (1.0 - beta1) * g
        vv *= beta2
        vv += (1.0 - beta2) * g * g
        p -= lr_t * mm / (np.sqrt(vv) + eps)
    return params, m, v


# --------------------------------------------------------------------------
# multi-stage network: get_single_block_resnet_build_function with
# num_stages > 2 (tfkeras_resnets.py:547-597), stage transitions by
# single_layer_conv_block (tfkeras_resnets.py:204-269)
# --------------------------------------------------------------------------


def _same_pads(H, W, k, stride):
    Ho, Wo = -(-H // stride), -(-W // stride)
    ph = max((Ho - 1) * stride + k - H, 0)
    pw = max((Wo - 1) * stride + k - W, 0)
    return Ho, Wo, ph, pw


def conv2d_backprop_input_strided(dz, W, x_shape, stride):
    """Conv2DBackpropInput of conv2d_same(x, W, stride) (TF 'SAME': pad_top =
    pad_total // 2, the remainder at the bottom/right)."""
    N, H, Wd, Ci = x_shape
    kh, kw, _, Co = W.shape
    Ho, Wo, ph, pw = _same_pads(H, Wd, kh, stride)
    dxp = np.zeros((N, H + ph, Wd + pw, Ci), dtype=np.result_type(dz, W))
    for ky in range(kh):
        for kx in range(kw):
            dxp[:, ky:ky + (Ho - 1) * stride + 1:stride, kx:kx + (Wo - 1) * stride + 1:stride, :] += dz @ W[ky, kx].T
    return dxp[:, ph // 2:ph // 2 + H, pw // 2:pw // 2 + Wd, :]


def conv2d_backprop_filter_strided(x, dz, k, stride):
    """Conv2DBackpropFilter of conv2d_same(x, W[k,k], stride)."""
    N, H, Wd, Ci = x.shape
    Co = dz.shape[-1]
    Ho, Wo, ph, pw = _same_pads(H, Wd, k, stride)
    xp = np.zeros((N, H + ph, Wd + pw, Ci), dtype=np.result_type(x, dz))
    xp[:, ph // 2:ph // 2 + H, pw // 2:pw // 2 + Wd, :] = x
    dz2 = dz.reshape(-1, Co)
    dW = np.zeros((k, k, Ci, Co), dtype=xp.dtype)
    for ky in range(k):
        for kx in range(k):
            dW[ky, kx] = xp[:, ky:ky + (Ho - 1) * stride + 1:stride, kx:kx + (Wo - 1) * stride + 1:stride, :] \
                .reshape(-1, Ci).T @ dz2
    return dW


def transition_fwd(x, K2, b2, K1, b1, stride):
    """single_layer_conv_block without BN (tfkeras_resnets.py:238-269):
    x2 = Conv2D(k, strides, 'same')(x) (:238-245); shortcut = Conv2D(1x1,
    strides, default 'valid')(x) (:247-252); relu(x2) + shortcut (:261-262).
    Returns (y, z) with z the 3x3 branch's pre-activation."""
    z = conv2d_same(x, K2, stride) + b2
    sc = x[:, ::stride, ::stride, :] @ np.asarray(K1)[0, 0] + b1
    return np.maximum(z, 0) + sc, z


def transition_bwd(dy, x, z, K2, K1, stride):
    """Autodiff of transition_fwd: (dx, [dK2, db2, dK1, db1])."""
    dz = dy * (z > 0)
    dx = conv2d_backprop_input_strided(dz, K2, x.shape, stride)
    K1m = np.asarray(K1)[0, 0]
    dx[:, ::stride, ::stride, :] += dy @ K1m.T
    Ci, Co = K1m.shape
    dK2 = conv2d_backprop_filter_strided(x, dz, K2.shape[0], stride)
    dK1 = (x[:, ::stride, ::stride, :].reshape(-1, Ci).T @ dy.reshape(-1, Co))[None, None]
    return dx, [dK2, dz.sum(axis=(0, 1, 2)), dK1, dy.sum(axis=(0, 1, 2))]


@dataclass
class StagesSpec:
    """A multi-stage net: stages [(C, L, stride)] (stride 0: no transition),
    Euler identity blocks of one conv kind (NetSpec's kinds)."""
    stages: list = field(default_factory=lambda: [(16, 2, 0), (32, 2, 2), (64, 2, 2)])
    h: float = 1.0
    gamma: float = 0.0
    num_classes: int = 10
    H: int = 32
    W: int = 32
    Cin: int = 3
    subtract_mean: float | None = 127.5
    divide_by_stddev: float | None = 127.5
    kind: str = "3by3"
    antisymmetric: bool = True

    def block_spec(self, C):
        return NetSpec(C=C, L=0, h=self.h, gamma=self.gamma, kind=self.kind, antisymmetric=self.antisymmetric)

    def param_shapes(self):
        """asr_stages_config order: conv1 kernel/bias; per stage the transition
        (K2, b2, K1, b1) then per block [theta..., bias]; fc kernel/bias."""
        C0 = self.stages[0][0]
        s = [(3, 3, self.Cin, C0), (C0,)]
        Cp = C0
        for C, L, S in self.stages:
            if S:
                s += [(3, 3, Cp, C), (C,), (1, 1, Cp, C), (C,)]
            for _ in range(L):
                s += self.block_spec(C).theta_shapes() + [(C,)]
            Cp = C
        s += [(Cp, self.num_classes), (self.num_classes,)]
        return s

    def n_params(self):
        return int(sum(np.prod(x) for x in self.param_shapes()))


def stages_init_params(spec: StagesSpec, rng, dtype=np.float64, bias_std=0.0):
    """he_normal kernels (truncated, 2 sigma), biases zero or N(0, bias_std)."""
    out = []
    for shp in spec.param_shapes():
        if len(shp) == 1:
            out.append(np.zeros(shp, dtype) if bias_std == 0 else (rng.standard_normal(shp) * bias_std).astype(dtype))
        else:
            fan_in = int(np.prod(shp[:-1]))
            out.append(truncated_normal(rng, shp, math.sqrt(2.0 / fan_in), dtype))
    return out


def _block_W(spec: StagesSpec, C, theta):
    """(W, src, sign) of one block (src, sign None for the regular kind)."""
    if spec.kind == "regular":
        return np.asarray(theta[0]), None, None
    src, sign = _cached_map(C, spec.kind, spec.antisymmetric)
    return assemble_from_map(flatten(theta), C, src, sign, spec.gamma), src, sign


def stages_forward(spec: StagesSpec, params, images, dtype=np.float64, rnd=None, rnd_w=None):
    """rnd (optional): a rounding applied where a bf16 net (asr_stages_config
    dtype ASR_BF16) stores in bf16 -- the stem's output, every transition's and
    block's output, the blocks' assembled W -- so the restatement follows the
    bf16 executor's storage; everything else stays in `dtype`.
    rnd_w (optional): the blocks' W rounding instead of rnd, called as
    rnd_w(W, src, sign) with the block's parameter map (None, None for the
    regular kind): the executor's balanced bf16 pack (tests/helpers.py)."""
    r = rnd if rnd is not None else (lambda a: a)
    rw = rnd_w if rnd_w is not None else (lambda W, src, sign: r(W))
    ns = NetSpec(subtract_mean=spec.subtract_mean, divide_by_stddev=spec.divide_by_stddev)
    x0 = normalize_input(images, ns, dtype)
    z1 = conv2d_same(x0, params[0]) + params[1]
    x = r(np.maximum(z1, 0))
    i = 2
    ops = []  # per op: ("t", x_in, z, K2, K1, S) or ("b", x_in, z, W, C)
    for si, (C, L, S) in enumerate(spec.stages):
        if S:
            K2, b2, K1, b1 = params[i:i + 4]
            i += 4
            y, z = transition_fwd(x, K2, b2, K1, b1, S)
            ops.append(("t", x, z, K2, K1, S))
            x = r(y)
        nt = len(spec.block_spec(C).theta_shapes())
        for _ in range(L):
            theta, b = params[i:i + nt], params[i + nt]
            i += nt + 1
            W0, src, sign = _block_W(spec, C, theta)
            W = np.asarray(rw(W0, src, sign), np.float64) if (rnd is not None or rnd_w is not None) else W0
            y, z = euler_fwd(x, W, b, spec.h)
            ops.append(("b", x, z, W, C))
            x = r(y)
    fc_k, fc_b = params[i], params[i + 1]
    gap = x.mean(axis=(1, 2))
    probs = softmax(gap @ fc_k + fc_b)
    return probs, dict(x0=x0, z1=z1, ops=ops, xL=x, gap=gap, probs=probs, fc_k=fc_k, rnd=rnd)


def stages_backward(spec: StagesSpec, params, cache, onehot):
    """Gradients of the mean Keras CE loss, in StagesSpec.param_shapes order
    (with the forward's rnd applied to the chain gradient where the bf16
    executor stores it: after the head, every block and every transition)."""
    r = cache.get("rnd") or (lambda a: a)
    Nb = onehot.shape[0]
    dlogits = keras_cce_grad_logits(cache["probs"], onehot, 1.0 / Nb)
    d_fck = cache["gap"].T @ dlogits
    d_fcb = dlogits.sum(axis=0)
    xL = cache["xL"]
    dx = r(np.broadcast_to((dlogits @ cache["fc_k"].T)[:, None, None, :] / (xL.shape[1] * xL.shape[2]),
                           xL.shape).copy())
    back = []
    for op in reversed(cache["ops"]):
        if op[0] == "t":
            _, x_in, z, K2, K1, S = op
            dx, g = transition_bwd(dx, x_in, z, K2, K1, S)
            dx = r(dx)
            back.append(g)
        else:
            _, x_in, z, W, C = op
            bs = spec.block_spec(C)
            if bs.operator_antisymmetric():
                dx, dW, db = euler_bwd(dx, x_in, z, W, spec.h, spec.gamma)
            else:
                dx, dW, db = euler_bwd_generic(dx, x_in, z, W, spec.h)
            dx = r(dx)
            shapes = bs.theta_shapes()
            src, sign = _cached_map(C, spec.kind, spec.antisymmetric)
            ntheta = int(sum(np.prod(x) for x in shapes))
            back.append(unflatten(project_dW(dW, src, sign, ntheta), shapes) + [db])
    dz1 = dx * (cache["z1"] > 0)
    grads = [conv2d_backprop_filter(cache["x0"], dz1), dz1.sum(axis=(0, 1, 2))]
    for g in reversed(back):
        grads += list(g)
    return grads + [d_fck, d_fcb]
