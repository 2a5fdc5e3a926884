"""Run one Euler block's kernels (fwd and/or fused bwd) at a bench shape many
times; used under rocprofv3 (--kernel-trace --stats, or --pmc passes)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--C", type=int, default=64)
ap.add_argument("--N", type=int, default=512)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--what", default="fwd,bwd")
ap.add_argument("--lib", default=None, help="development: another build of libasr (A/B timing)")
ap.add_argument("--stack", type=int, default=0, help="run L blocks through asr_block_stack_forward/backward instead")
a = ap.parse_args()
lib = _lib.load(path=a.lib)
dev = rt.require_gpu()
N, H, W, C = a.N, 32, 32, a.C
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
dy = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
y = torch.empty_like(x)
dx = torch.empty_like(x)
pm = rt.param_map(C)
th = torch.randn(pm.n_theta, device=dev, generator=g) * 0.05
bias = torch.zeros(C, device=dev)
w = rt.theta_to_w(th, C, pm, 0.0, rt.ASR_BF16)
mask = torch.zeros(rt.mask_bytes(N, H, W, C), dtype=torch.uint8, device=dev)
wsb = int(lib.asr_conv_backward_workspace_bytes(N, H, W, C, rt.ASR_BF16))
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
dth = torch.empty(pm.n_theta, device=dev)
db = torch.empty(C, device=dev)
_, tdst = pm.device(dev)
s = torch.cuda.current_stream().cuda_stream
whats = a.what.split(",")
if a.stack:  # the network's path: all L blocks in one forward and one backward launch
    L = a.stack
    w = rt.theta_to_w(torch.randn(L * pm.n_theta, device=dev, generator=g) * 0.05, C, pm, 0.0, rt.ASR_BF16, layers=L)
    biasL = torch.zeros(L, C, device=dev)
    for _ in range(a.reps):
        ys, masks = rt.block_stack_forward(x, w, biasL, 0.25)
        rt.block_stack_backward(dy, x, ys, masks, w, pm, 0.25, 0.0)
    torch.cuda.synchronize()
    print("done")
    sys.exit(0)
# one forward first: the backward reads its relu mask (random operands, ~half set)
_lib.check(lib.asr_conv_forward(0, x.data_ptr(), y.data_ptr(), mask.data_ptr(), w.data_ptr(), bias.data_ptr(),
                                0.25, N, H, W, C, 1, s))
for _ in range(a.reps):
    if "fwd" in whats:
        _lib.check(lib.asr_conv_forward(0, x.data_ptr(), y.data_ptr(), mask.data_ptr(), w.data_ptr(), bias.data_ptr(),
                                        0.25, N, H, W, C, 1, s))
    if "bwd" in whats:
        _lib.check(lib.asr_conv_backward(0, dy.data_ptr(), x.data_ptr(), mask.data_ptr(), w.data_ptr(),
                                         tdst.data_ptr(), pm.n_theta, 0.25, 0.0, N, H, W, C, 1, dx.data_ptr(),
                                         dth.data_ptr(), db.data_ptr(), None, ws.data_ptr(), wsb, s))
torch.cuda.synchronize()
print("done")
