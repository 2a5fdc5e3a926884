"""development: per-step timestamps of the fused C=16 backward (block 0:
dgrad wave 0, wgrad wave 4, staging wave 7) from a build with
-DASR_DEEP_TRACE=1 (tools/build_variants.sh e8 "-DASR_DEEP_TRACE=1").
usage: python tools/tracebench.py build_abl_e8.so [--N 1024 --L 108]"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--N", type=int, default=1024)
ap.add_argument("--L", type=int, default=108)
a = ap.parse_args()
path = os.path.abspath(a.lib)
_lib.load(path=path)
dev = rt.require_gpu()
N, L, C = a.N, a.L, 16
g = torch.Generator(device=dev).manual_seed(0)
pm = rt.param_map(C)
w = rt.theta_to_w(torch.randn(L * pm.n_theta, device=dev, generator=g) * 0.05, C, pm, 0.0, rt.ASR_BF16, layers=L)
bias = torch.randn(L, C, device=dev, generator=g) * 0.1
x0 = torch.randn(N, 32, 32, C, device=dev, generator=g).to(torch.bfloat16)
dyL = (torch.randn(N, 32, 32, C, device=dev, generator=g) * 0.1).to(torch.bfloat16)
h = 8.0 / L
ys, masks = rt.block_stack_forward(x0, w, bias, h)
for _ in range(3):
    rt.block_stack_backward(dyL, x0, ys, masks, w, pm, h, 0.0)
torch.cuda.synchronize()
lib = ctypes.CDLL(path)
buf = (ctypes.c_uint64 * (3 * 160 * 4))()
assert lib.asr_debug_deep16_trace(buf, ctypes.sizeof(buf)) == 0
tr4 = np.frombuffer(buf, np.uint64).reshape(3, 160, 4).astype(np.int64)
tr = tr4[:, :, :2]
t0 = tr[tr > 0].min()
names = ["dgrad0", "wgrad4", "stage7"]
print("step " + " ".join(f"{n + ' start':>13} {'busy':>6}" for n in names) + "   step_len")
for t in range(0, 60):
    row = []
    for r in range(3):
        s, e = tr[r, t]
        row.append(f"{s - t0:13d} {e - s:6d}" if s > 0 else " " * 20)
    nxt = tr[0, t + 1, 0] - tr[0, t, 0] if tr[0, t + 1, 0] > 0 and tr[0, t, 0] > 0 else 0
    print(f"{t:4d} " + " ".join(row) + f"   {nxt}")
for r in range(3):
    v = tr[r, 5:100]
    v = v[(v[:, 0] > 0)]
    print(names[r], "median busy", int(np.median(v[:, 1] - v[:, 0])))
s = tr[0, 5:100, 0]
s = s[s > 0]
print("median step", int(np.median(np.diff(s))))
v = tr4[2, 5:100]
v = v[v[:, 0] > 0]
print("stage7 median: start->written", int(np.median(v[:, 2] - v[:, 0])), " written->db done", int(np.median(v[:, 3] - v[:, 2])),
      " db done->x DMA landed", int(np.median(v[:, 1] - v[:, 3])))
