"""Development check of a forward-stack variant build that
is not bitwise equal to the per-block kernels: every layer of
asr_block_stack_forward against the oracle's Euler step on the variant's own
bf16 input of that layer (2^-8 relative + 4e-3 * max|ref|, as
tests/test_gpu_stack64.py), relu masks equal off the rounding boundary, and
the agreement with k_fwd3 (the per-block kernel of the same build).
usage: python tools/fwd_variant_check.py --lib build_abl_X.so"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402
from helpers import assert_close, bf16_round, decode_mask  # noqa: E402
from oracle import asr_oracle as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
a = ap.parse_args()
_lib.load(path=os.path.abspath(a.lib))
dev = rt.require_gpu()
C, H, W, h = 64, 32, 32, 8.0 / 30
for N, L, with_bias in ((1, 3, True), (5, 4, False), (300, 3, True), (512, 2, True)):
    rng = np.random.default_rng(N * 7 + L)
    pm = rt.param_map(C)
    th = np.concatenate([O.flatten(O.init_theta_3by3(C, rng, np.float64)) for _ in range(L)]).astype(np.float32)
    w = rt.theta_to_w(torch.from_numpy(th).to(dev), C, pm, 0.0, rt.ASR_BF16, layers=L)
    b = (rng.standard_normal((L, C)) * 0.1).astype(np.float32)
    bias = torch.from_numpy(b).to(dev) if with_bias else None
    x0 = torch.from_numpy(rng.standard_normal((N, H, W, C)).astype(np.float32)).to(dev).to(torch.bfloat16)
    ys, masks = rt.block_stack_forward(x0, w, bias, h)
    # against the per-block kernel of the same build, layer by layer on the stack's own inputs
    x = x0
    diff_y = diff_m = 0
    for l in range(L):
        m = torch.zeros(rt.mask_bytes(N, H, W, C), dtype=torch.uint8, device=dev)
        y = rt.conv_forward(rt.ASR_MODE_EULER, x, w[l:l + 1], bias[l].contiguous() if bias is not None else None, h, m)
        diff_y += int((y != ys[l]).sum())
        diff_m += int((m != masks[l]).sum())
        x = ys[l]
    src, sign = O.param_map(C)
    th2 = th.reshape(L, -1)
    pick = np.arange(N) if N <= 5 else np.array([0, N // 2, N - 1])
    xin = x0[pick].float().cpu().numpy().astype(np.float64)
    for l in range(L):
        Wl = bf16_round(O.assemble_from_map(th2[l].astype(np.float64), C, src, sign, 0.0)).astype(np.float64)
        z = O.conv2d_same(xin, Wl) + (b[l] if with_bias else 0.0)
        want = xin + h * np.maximum(z, 0)
        got = ys[l][pick].float().cpu().numpy()
        assert_close(got, want, rtol=2 ** -8, atol=4e-3 * np.abs(want).max(), what=f"N={N} layer {l}")
        mk = decode_mask(masks[l].cpu().numpy(), N, H, W, C)[pick]
        far = np.abs(z) > 1e-3 * np.abs(z).max()
        assert np.array_equal(mk[far], (z > 0)[far]), f"N={N} layer {l}: mask"
        xin = got.astype(np.float64)
    print(f"N={N} L={L} bias={with_bias}: oracle ok; vs per-block k_fwd3: {diff_y} y elements and {diff_m} mask "
          f"bytes differ (of {N * H * W * C * L})", flush=True)
print("fwd variant check ok")
