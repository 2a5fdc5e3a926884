"""Shared test utilities: bf16 rounding in numpy, mask decoding, tolerances."""
import numpy as np


def bf16_round(x):
    """Round float32 -> bfloat16 (RNE) and back, in numpy."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    u = a.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32).reshape(a.shape)


def decode_mask(words, N, H, W, C):
    """Inverse of the mask layout (csrc/asr_common.h mask_base): returns bool
    [N,H,W,C] with bit (n,y,x,o) = word[((n*H+y)*PT + x//16)*OT + o//16)*4 + (o%16)%4]
    >> ((o%16)//4*16 + x%16)."""
    w = np.asarray(words).view(np.uint64)
    PT, OT = (W + 15) // 16, (C + 15) // 16
    n, y, x, o = np.meshgrid(np.arange(N), np.arange(H), np.arange(W), np.arange(C), indexing="ij")
    ol = o % 16
    idx = ((((n * H + y) * PT + x // 16) * OT + o // 16) * 4 + (ol % 4))
    bit = (ol // 4) * 16 + (x % 16)
    return ((w[idx] >> bit.astype(np.uint64)) & np.uint64(1)).astype(bool)


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
