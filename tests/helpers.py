"""Shared test utilities: bf16 rounding in numpy, mask decoding, tolerances."""
import numpy as np


def bf16_round(x):
    """Round float32 -> bfloat16 (RNE) and back, in numpy."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    u = a.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32).reshape(a.shape)


def _pairs_antisymmetric(src, sign, C):
    """Every off-diagonal W[t][i][o] (i > o) and W[8-t][o][i] read the same
    theta with opposite signs (the 3by3 and general maps, either
    `antisymmetric` flag; not the regular kind)."""
    s = np.asarray(src).reshape(9, C, C)
    g = np.asarray(sign).reshape(9, C, C)
    i, o = np.triu_indices(C, 1)[::-1]  # i > o
    a, b = s[:, i, o], s[::-1][:, o, i]
    return bool(np.all(a >= 0) and np.all(a == b) and np.all(g[:, i, o] == -g[::-1][:, o, i]))


def w_bf16_balanced(W, src=None, sign=None):
    """The bf16 W of the executor's weight pack (asr_theta.hip,
    k_theta_to_w_pack_bal), bit-exact.  Maps whose off-diagonal entries come
    in antisymmetric pairs (W[t][i][o] = -W[8-t][o][i]) round each pair to one
    of its two bf16 neighbours, chosen so that every output channel's sum of
    rounding errors stays near zero: round-to-nearest perturbs each output
    channel by a fixed sum that every pixel of every image sees, and over a
    deep stack that coherent error dominates (tools/bf16_depth_emulate.py,
    DESIGN §3g).  Diagonal entries round to nearest and their errors (taps
    0..8, float32) start each channel's error sum e; the pairs are then
    visited in the round-robin order of the kernel (C-1 rounds of C/2 disjoint
    channel pairs); within a pair (o, i), D = e_o - e_i, and per tap 0..8 the
    upper neighbour iff D + (d_lo + d_hi) < 0, else the lower (a bf16 value
    stays), D += 2d; then e_o += S, e_i -= S for the pair's S = sum d, all in
    float32.  A map without the pairing (or src=None) rounds to nearest."""
    W32 = np.asarray(W, np.float32).reshape(3, 3, W.shape[2], W.shape[3])
    C = W32.shape[2]
    Q = bf16_round(W32).reshape(9, C, C).copy()
    if src is None or C % 2 or not _pairs_antisymmetric(src, sign, C):
        return Q.reshape(W32.shape)
    X = W32.reshape(9, C, C)
    err = np.zeros(C, np.float32)
    dg = np.arange(C)
    for t in range(9):  # the error sums start from the diagonal entries' (nearest) rounding
        err = err + (Q[t, dg, dg] - X[t, dg, dg])
    q = np.arange(1, C // 2)
    for r in range(C - 1):
        a = np.concatenate([[C - 1], (r + q) % (C - 1)])
        b = np.concatenate([[r], (r - q) % (C - 1)])
        o, i = np.minimum(a, b), np.maximum(a, b)
        eo, ei = err[o].copy(), err[i].copy()
        D, S = eo - ei, np.zeros_like(eo)
        for t in range(9):
            x = X[t, i, o]
            bits = x.view(np.uint32)
            exact = (bits & np.uint32(0xFFFF)) == 0
            dtz = (bits & np.uint32(0xFFFF0000)).view(np.float32) - x
            daw = ((bits & np.uint32(0xFFFF0000)) + np.uint32(0x10000)).view(np.float32) - x
            zero = np.float32(0)
            d_lo = np.where(exact, zero, np.where(x > 0, dtz, daw)).astype(np.float32)
            d_hi = np.where(exact, zero, np.where(x > 0, daw, dtz)).astype(np.float32)
            sd = np.where(exact, zero, dtz + daw).astype(np.float32)
            d = np.where(D + sd < 0, d_hi, d_lo).astype(np.float32)
            D = (D + np.float32(2) * d).astype(np.float32)
            S = (S + d).astype(np.float32)
            qv = (x + d).astype(np.float32)
            Q[t, i, o] = qv
            Q[8 - t, o, i] = -qv
        err[o], err[i] = eo + S, ei - S
    return Q.reshape(W32.shape)


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
