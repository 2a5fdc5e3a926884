"""Run the deep-stack C=16 path (asr_block_stack_forward + _backward, all L
blocks fused) at the C3 shape several times; used under rocprofv3
(--kernel-trace --stats, or --pmc passes)."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--N", type=int, default=1024)
ap.add_argument("--L", type=int, default=108)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--what", default="fwd,bwd")
ap.add_argument("--lib", default=None, help="development: another build of libasr (A/B timing)")
a = ap.parse_args()
lib = _lib.load(path=a.lib)
dev = rt.require_gpu()
N, L, C = a.N, a.L, 16
g = torch.Generator(device=dev).manual_seed(0)
pm = rt.param_map(C)
th = torch.randn(L * pm.n_theta, device=dev, generator=g) * 0.05
w = rt.theta_to_w(th, C, pm, 0.0, rt.ASR_BF16, layers=L)
bias = torch.randn(L, C, device=dev, generator=g) * 0.1
x0 = torch.randn(N, 32, 32, C, device=dev, generator=g).to(torch.bfloat16)
dyL = (torch.randn(N, 32, 32, C, device=dev, generator=g) * 0.1).to(torch.bfloat16)
h = 8.0 / L
ys, masks = rt.block_stack_forward(x0, w, bias, h)
whats = a.what.split(",")
for _ in range(a.reps):
    if "fwd" in whats:
        ys, masks = rt.block_stack_forward(x0, w, bias, h)
    if "bwd" in whats:
        dx0, dp = rt.block_stack_backward(dyL, x0, ys, masks, w, pm, h, 0.0)
torch.cuda.synchronize()
print("done")
