"""Development: where does the C=64 forward stack differ from per-block
k_fwd3 launches (rows, channel tiles, images), N and L from argv."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402
from oracle import asr_oracle as O  # noqa: E402

N, L = int(sys.argv[1]), int(sys.argv[2])
if len(sys.argv) > 3:
    _lib.load(path=os.path.abspath(sys.argv[3]))
C, H, W, h = 64, 32, 32, 8.0 / 30
rng = np.random.default_rng(N * 7 + L)
dev = rt.require_gpu()
pm = rt.param_map(C)
th = np.concatenate([O.flatten(O.init_theta_3by3(C, rng, np.float64)) for _ in range(L)]).astype(np.float32)
w = rt.theta_to_w(torch.from_numpy(th).to(dev), C, pm, 0.0, rt.ASR_BF16, layers=L)
b = (rng.standard_normal((L, C)) * 0.1).astype(np.float32)
bias = torch.from_numpy(b).to(dev)
x0 = torch.from_numpy(rng.standard_normal((N, H, W, C)).astype(np.float32)).to(dev).to(torch.bfloat16)
ys, masks = rt.block_stack_forward(x0, w, bias, h)
x = x0
for l in range(L):
    m = torch.zeros(rt.mask_bytes(N, H, W, C), dtype=torch.uint8, device=dev)
    y = rt.conv_forward(rt.ASR_MODE_EULER, x, w[l:l + 1], bias[l].contiguous(), h, m)
    d = (y.float() - ys[l].float()).abs().view(N, H, W, C).cpu()
    bad = d > 0
    print(f"layer {l}: {int(bad.sum())} differ, max {float(d.max()):.4g}")
    if bad.any():
        print("  images", torch.nonzero(bad.any(3).any(2).any(1)).flatten().tolist()[:20])
        print("  rows", torch.nonzero(bad.any(3).any(2).any(0)).flatten().tolist())
        print("  cols", torch.nonzero(bad.any(3).any(1).any(0)).flatten().tolist())
        print("  chans", torch.nonzero(bad.any(2).any(1).any(0)).flatten().tolist())
        for lo in range(L):
            if lo == l:
                continue
            yo = rt.conv_forward(rt.ASR_MODE_EULER, x, w[lo:lo + 1], bias[l].contiguous(), h,
                                 torch.zeros_like(m))
            yb = rt.conv_forward(rt.ASR_MODE_EULER, x, w[l:l + 1], bias[lo].contiguous(), h, torch.zeros_like(m))
            s = ys[l].view(N, H, W, C)
            print(f"  stale W of layer {lo} explains {int((yo.view(N, H, W, C) == s)[bad].sum())}; "
                  f"stale bias explains {int((yb.view(N, H, W, C) == s)[bad].sum())}")
    # float64 oracle on the layer's (shared) input: which side is off?
    src, sign = O.param_map(C)
    Wl = O.assemble_from_map(th.reshape(L, -1)[l].astype(np.float64), C, src, sign, 0.0)
    Wl = torch.from_numpy(Wl).to(torch.bfloat16).double().numpy()
    xin = x.double().cpu().numpy()
    want = xin + h * np.maximum(O.conv2d_same(xin, Wl) + b[l], 0)
    tol = 2 ** -8 * np.abs(want) + 4e-3 * np.abs(want).max()
    for name, got in (("per-block", y), ("stack", ys[l])):
        e = np.abs(got.double().cpu().numpy() - want)
        print(f"  {name} vs oracle: {int((e > tol).sum())} beyond tol, max err {e.max():.4g}")
    x = y
