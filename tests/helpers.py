"""Shared test utilities: bf16 rounding in numpy, mask decoding, tolerances."""
import numpy as np


def bf16_round(x):
    """Round float32 -> bfloat16 (RNE) and back, in numpy."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    u = a.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32).reshape(a.shape)


def decode_mask(mask_bytes, N, H, W, C):
    """Inverse of the relu-mask layout (include/asr.h): bit (pixel*C + o),
    LSB first, pixel = (n*H + y)*W + x.  Returns bool [N,H,W,C]."""
    b = np.asarray(mask_bytes).view(np.uint8)
    bits = np.unpackbits(b, bitorder="little")[: N * H * W * C]
    return bits.reshape(N, H, W, C).astype(bool)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def assert_close(got, want, rtol, atol=0.0, what=""):
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    err = np.abs(got - want)
    lim = atol + rtol * np.abs(want)
    bad = err > lim
    if bad.any():
        i = np.unravel_index(np.argmax(err - lim), err.shape)
        raise AssertionError(f"{what}: {bad.sum()} / {bad.size} elements outside tolerance "
                             f"(rtol={rtol}, atol={atol}); worst at {i}: got {got[i]!r} want {want[i]!r}")


def rel_l2(got, want):
    """||got - want||_2 / ||want||_2 over the flattened arrays."""
    got = np.asarray(got, np.float64).ravel()
    want = np.asarray(want, np.float64).ravel()
    return float(np.linalg.norm(got - want) / max(np.linalg.norm(want), 1e-30))


def grad_groups(spec, g):
    """(name, flat array) per gradient group in Keras weight order: conv1
    kernel and bias, per block its merged theta (all kernel variables) and
    bias, fc kernel and bias — the per-layer groups of the reference's
    gradient norms (training.py:385-409)."""
    nt = len(spec.theta_shapes())
    out = [("conv1/kernel", np.ravel(g[0])), ("conv1/bias", np.ravel(g[1]))]
    i = 2
    for b in range(spec.L):
        out.append((f"block{b}/theta", np.concatenate([np.ravel(a) for a in g[i:i + nt]])))
        out.append((f"block{b}/bias", np.ravel(g[i + nt])))
        i += nt + 1
    out += [("fc/kernel", np.ravel(g[i])), ("fc/bias", np.ravel(g[i + 1]))]
    return out


def assert_grad_tensors_max(spec, got, want, tol, report_only=False, groups=None):
    """Per-tensor bar inside the per-group one: every gradient tensor's
    max |got - want| <= tol x max |want| over the tensor's gradient group.
    A group's relative L2 dilutes a few wrong scalars (a zeroed channel of
    one theta variable) among thousands of kernel entries; this bar does
    not.  `groups`: [(name, [tensor indices])]; default: the network's
    (conv1, per block theta + bias, fc).  report_only: return the worst
    (name, ratio) instead of asserting."""
    if groups is None:
        nt = len(spec.theta_shapes())
        groups = [("conv1", [0, 1])]
        i = 2
        for b in range(spec.L):
            groups.append((f"block{b}", list(range(i, i + nt + 1))))
            i += nt + 1
        groups.append(("fc", [i, i + 1]))
    worst, bad = ("", 0.0), []
    for name, idx in groups:
        scale = max(float(np.abs(want[i]).max()) for i in idx)
        if scale == 0:
            continue
        for i in idx:
            r = float(np.abs(np.asarray(got[i], np.float64) - want[i]).max()) / scale
            if r > worst[1]:
                worst = (f"{name}/tensor{i} {np.shape(want[i])}", r)
            if not r <= tol:
                bad.append(f"{name}/tensor{i} {np.shape(want[i])}: {r:.3e}")
    if report_only:
        return worst
    assert not bad, f"per-tensor max|err| > {tol} x group max: " + "; ".join(bad[:12])
    return worst


def assert_grad_groups_rel_l2(spec, got, want, tol=2e-2):
    """bf16 network gradients vs the fp64 oracle: relative L2 <= tol per
    gradient group."""
    bad = []
    for (name, a), (_, b) in zip(grad_groups(spec, got), grad_groups(spec, want)):
        if np.linalg.norm(b) == 0:
            assert np.linalg.norm(a) == 0, name
            continue
        e = rel_l2(a, b)
        if not e <= tol:
            bad.append(f"{name}: rel-L2 {e:.3e}")
    assert not bad, "; ".join(bad)
