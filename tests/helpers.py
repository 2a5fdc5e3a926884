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
