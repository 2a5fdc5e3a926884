"""The balanced bf16 rounding of the weight pack (asr_theta.hip,
k_theta_to_w_pack_bal), as restated by tests/helpers.py w_bf16_balanced: CPU
properties of the restatement, and a scalar re-derivation of the same greedy
rule it must equal bit for bit.  The GPU pack is checked against it in
tests/test_gpu_kernels.py (test_theta_to_w_bf16_pack_exact)."""
import numpy as np
import pytest

from helpers import bf16_round, w_bf16_balanced
from oracle import asr_oracle as O


def _w(C, kind, anti, gamma, seed):
    rng = np.random.default_rng(seed)
    src, sign = O.param_map(C, kind, 3, anti)
    n = int(src.max()) + 1
    th = (rng.standard_normal(n) * 0.2).astype(np.float32)
    return O.assemble_from_map(th.astype(np.float64), C, src, sign, gamma).astype(np.float32), src, sign


def _neighbours(x):
    """the bf16 values just below and above float32 x (equal if x is one)"""
    b = np.float32(x).view(np.uint32)
    tz = np.uint32(b & 0xFFFF0000).view(np.float32)
    aw = np.uint32((b & 0xFFFF0000) + 0x10000).view(np.float32)
    return (min(tz, aw), max(tz, aw)) if b & 0xFFFF else (x, x)


@pytest.mark.parametrize("C,kind,anti,gamma", [(16, "3by3", True, 0.0), (32, "3by3", True, -0.1),
                                               (64, "3by3", True, 0.0), (16, "general", True, 0.05),
                                               (16, "general", False, 0.0)])
def test_balanced_pack_properties(C, kind, anti, gamma):
    W, src, sign = _w(C, kind, anti, gamma, C)
    Q = w_bf16_balanced(W, src, sign)
    assert np.array_equal(bf16_round(Q), Q)  # bf16 values
    lo = np.vectorize(lambda v: _neighbours(v)[0])(W)
    hi = np.vectorize(lambda v: _neighbours(v)[1])(W)
    assert np.all((Q == lo) | (Q == hi))  # each entry one of its two bf16 neighbours
    i, o = np.triu_indices(C, 1)[::-1]
    Q9, W9 = Q.reshape(9, C, C), W.reshape(9, C, C)
    assert np.array_equal(Q9[:, i, o], -Q9[::-1][:, o, i])  # the pairs stay exactly antisymmetric
    assert np.array_equal(Q9[:, np.arange(C), np.arange(C)], bf16_round(W9[:, np.arange(C), np.arange(C)]))
    # every output channel's error sum: far below round-to-nearest's
    e_bal = np.abs((Q.astype(np.float64) - W).reshape(-1, C).sum(0))
    e_rn = np.abs((bf16_round(W).astype(np.float64) - W).reshape(-1, C).sum(0))
    ulp = np.abs(W).max() * 2.0 ** -8
    assert e_bal.max() <= 2 * ulp, (e_bal.max(), ulp)
    assert e_bal.mean() < 0.25 * e_rn.mean(), (e_bal.mean(), e_rn.mean())


def test_unpaired_map_rounds_to_nearest():
    """The regular kind (every entry its own variable) and src=None: round to nearest."""
    W = np.random.default_rng(0).standard_normal((3, 3, 16, 16)).astype(np.float32)
    assert np.array_equal(w_bf16_balanced(W), bf16_round(W))
    W3, src, sign = _w(16, "3by3", True, 0.0, 1)
    src2 = src.copy()
    src2[np.flatnonzero(src2 >= 0)[5]] = int(src.max()) + 1  # break one pair
    assert np.array_equal(w_bf16_balanced(W3, src2, sign), bf16_round(W3))


def test_vectorised_restatement_equals_scalar_greedy():
    """The same rule written pair by pair with float32 scalars: the round-robin
    order (round r: pair 0 = (C-1, r), pair k = ((r+k) % (C-1), (r-k) % (C-1))),
    taps 0..8 in a pair, upper neighbour iff D + (d_lo + d_hi) < 0 with
    D = e_o - e_i carried as D += 2d, the pair's sum S = sum d moving e_o and
    e_i after its last tap, the sums starting from the diagonal entries'
    nearest-rounding errors."""
    C = 16
    W, src, sign = _w(C, "3by3", True, -0.05, 7)
    Q = bf16_round(W).reshape(9, C, C).copy()
    X = W.reshape(9, C, C)
    e = [np.float32(0)] * C
    for c in range(C):
        for t in range(9):
            e[c] = np.float32(e[c] + np.float32(bf16_round(X[t, c, c])[()] - X[t, c, c]))
    for r in range(C - 1):
        for k in range(C // 2):
            a, b = (C - 1, r) if k == 0 else ((r + k) % (C - 1), (r - k) % (C - 1))
            o, i = min(a, b), max(a, b)
            D, S = np.float32(e[o] - e[i]), np.float32(0)
            for t in range(9):
                x = X[t, i, o]
                lo, hi = _neighbours(x)
                d = np.float32(0) if lo == hi else (np.float32(hi - x) if np.float32(
                    D + np.float32(np.float32(lo - x) + np.float32(hi - x))) < 0 else np.float32(lo - x))
                D, S = np.float32(D + np.float32(2 * d)), np.float32(S + d)
                q = np.float32(x + d)
                Q[t, i, o], Q[8 - t, o, i] = q, -q
            e[o], e[i] = np.float32(e[o] + S), np.float32(e[i] - S)
    assert np.array_equal(Q.reshape(W.shape).view(np.uint32), w_bf16_balanced(W, src, sign).view(np.uint32))
