"""Development: run one C=64 Euler forward (random operands, fixed seed) with
a given libasr build and save y and the relu mask, so that two kernel
variants can be compared bitwise (tools/fwddump.py --lib A --out a.npz; ...)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--out", required=True)
ap.add_argument("--N", type=int, default=300)
ap.add_argument("--mode", type=int, default=0)
a = ap.parse_args()
lib = _lib.load(path=a.lib)
dev = rt.require_gpu()
N, H, W, C = a.N, 32, 32, 64
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
pm = rt.param_map(C)
th = torch.randn(pm.n_theta, device=dev, generator=g) * 0.05
bias = torch.randn(C, device=dev, generator=g) * 0.1
w = rt.theta_to_w(th, C, pm, 0.0, rt.ASR_BF16)
y = torch.empty_like(x)
mask = torch.zeros(rt.mask_bytes(N, H, W, C), dtype=torch.uint8, device=dev)
s = torch.cuda.current_stream().cuda_stream
_lib.check(lib.asr_conv_forward(a.mode, x.data_ptr(), y.data_ptr(), mask.data_ptr() if a.mode == 0 else None,
                                w.data_ptr(), bias.data_ptr(), 8.0 / 30, N, H, W, C, rt.ASR_BF16, s))
torch.cuda.synchronize()
np.savez(a.out, y=y.view(torch.int16).cpu().numpy(), mask=mask.cpu().numpy())
print("saved", a.out)
