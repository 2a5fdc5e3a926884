"""development: per-band s_memtime stamps of workgroup 0 in the C=64 stack
kernels (k_fwd3_stack, k_bwd3_stack) and their in-kernel clock, from a build
with -DASR_BLK_TRACE=1 (tools/build_variants.sh tr "-DASR_BLK_TRACE=1").
The first 40 items cover the block switches of both kernels.
usage: python tools/stacktrace.py build_abl_tr.so [--N 512] [--L 30]"""
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
ap.add_argument("--N", type=int, default=512)
ap.add_argument("--L", type=int, default=30)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
path = os.path.abspath(a.lib)
_lib.load(path=path)
dev = rt.require_gpu()
N, C, L = a.N, 64, a.L
g = torch.Generator(device=dev).manual_seed(0)
pm = rt.param_map(C)
w = rt.theta_to_w(torch.randn(L * pm.n_theta, device=dev, generator=g) * 0.05, C, pm, 0.0, rt.ASR_BF16, layers=L)
bias = torch.zeros(L, C, device=dev)
x = torch.randn(N, 32, 32, C, device=dev, generator=g).to(torch.bfloat16)
dy = (torch.randn(N, 32, 32, C, device=dev, generator=g) * 0.1).to(torch.bfloat16)
for _ in range(a.reps):
    ys, masks = rt.block_stack_forward(x, w, bias, 0.25)
    rt.block_stack_backward(dy, x, ys, masks, w, pm, 0.25, 0.0)
torch.cuda.synchronize()
cl = ctypes.CDLL(path)
tb = (ctypes.c_uint64 * (2 * 2 * 40 * 8))()
cb = (ctypes.c_uint64 * (2 * 1024 * 4))()
assert cl.asr_debug_blk_trace(tb, ctypes.sizeof(tb), cb, ctypes.sizeof(cb)) == 0
tr = np.frombuffer(tb, np.uint64).reshape(2, 2, 40, 8).astype(np.int64)
ck = np.frombuffer(cb, np.uint64).reshape(2, 1024, 4).astype(np.int64)
for k, name in ((0, "k_fwd3_stack"), (1, "k_bwd3_stack")):
    c = ck[k]
    c = c[(c[:, 0] > 0) & (c[:, 2] > c[:, 0])]
    ghz = (c[:, 2] - c[:, 0]) / (c[:, 3] - c[:, 1]) * 0.1
    st, en = (c[:, 1] - c[:, 1].min()) / 100, (c[:, 3] - c[:, 1].min()) / 100
    print(f"{name}: workgroups {len(c)}, clock median {np.median(ghz):.3f} GHz; start us p100 {st.max():.1f}; "
          f"end us p0/p50/p100 {en.min():.1f}/{np.median(en):.1f}/{en.max():.1f}")


def rows(t, names, nslot):
    print("   item " + " ".join(f"{n:>9}" for n in names) + "      band")
    for i in range(40):
        if t[i, 0] == 0:
            break
        d = np.diff(t[i, :nslot])
        nxt = t[i + 1, 0] - t[i, 0] if i + 1 < 40 and t[i + 1, 0] > 0 else 0
        print(f"   {i:4d} " + " ".join(f"{v:9d}" for v in d) + f" {nxt:9d}")


print("k_fwd3_stack wave 0 (cycles):")
rows(tr[0, 0], ["barrier", "dma+copy", "conv", "epilogue"], 5)
print("k_bwd3_stack dgrad wave 0:")
rows(tr[1, 0], ["barrier", "conv", "epilogue", "halo"], 5)
print("k_bwd3_stack wgrad wave 4:")
rows(tr[1, 1], ["poll+bar", "issue", "mfma", "vmwait", "convert", "fold+slab"], 7)
