"""development: per-band timestamps of workgroup 0 and the in-kernel clock of
the C=64 band kernels (k_fwd3, k_bwd3) from a build with -DASR_BLK_TRACE=1
(tools/build_variants.sh tr "-DASR_BLK_TRACE=1").
usage: python tools/blktrace.py build_abl_tr.so [--N 512]"""
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
ap.add_argument("--reps", type=int, default=200)
a = ap.parse_args()
path = os.path.abspath(a.lib)
lib = _lib.load(path=path)
dev = rt.require_gpu()
N, H, W, C = a.N, 32, 32, 64
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
dy = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
y, dx = torch.empty_like(x), torch.empty_like(x)
pm = rt.param_map(C)
w = rt.theta_to_w(torch.randn(pm.n_theta, device=dev, generator=g) * 0.05, C, pm, 0.0, rt.ASR_BF16)
bias = torch.zeros(C, device=dev)
mask = torch.zeros(rt.mask_bytes(N, H, W, C), dtype=torch.uint8, device=dev)
wsb = int(lib.asr_conv_backward_workspace_bytes(N, H, W, C, rt.ASR_BF16))
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
dth, db = torch.empty(pm.n_theta, device=dev), torch.empty(C, device=dev)
_, tdst = pm.device(dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(a.reps):  # >= 2 s of back-to-back launches before the stamped ones
    _lib.check(lib.asr_conv_forward(0, x.data_ptr(), y.data_ptr(), mask.data_ptr(), w.data_ptr(), bias.data_ptr(),
                                    0.25, N, H, W, C, 1, s))
    _lib.check(lib.asr_conv_backward(0, dy.data_ptr(), x.data_ptr(), mask.data_ptr(), w.data_ptr(), tdst.data_ptr(),
                                     pm.n_theta, 0.25, 0.0, N, H, W, C, 1, dx.data_ptr(), dth.data_ptr(),
                                     db.data_ptr(), None, ws.data_ptr(), wsb, s))
torch.cuda.synchronize()
cl = ctypes.CDLL(path)
tb = (ctypes.c_uint64 * (2 * 2 * 40 * 6))()
cb = (ctypes.c_uint64 * (2 * 1024 * 4))()
assert cl.asr_debug_blk_trace(tb, ctypes.sizeof(tb), cb, ctypes.sizeof(cb)) == 0
tr = np.frombuffer(tb, np.uint64).reshape(2, 2, 40, 6).astype(np.int64)
ck = np.frombuffer(cb, np.uint64).reshape(2, 1024, 4).astype(np.int64)
for k, name in ((0, "k_fwd3"), (1, "k_bwd3")):
    c = ck[k]
    c = c[(c[:, 0] > 0) & (c[:, 2] > c[:, 0])]
    ghz = (c[:, 2] - c[:, 0]) / (c[:, 3] - c[:, 1]) * 0.1
    cyc = c[:, 2] - c[:, 0]
    print(f"{name}: workgroups {len(c)}, in-kernel clock median {np.median(ghz):.3f} GHz "
          f"(min {ghz.min():.3f}, max {ghz.max():.3f}); wave-0 cycles median {int(np.median(cyc))}, "
          f"max {int(cyc.max())}; wall median {np.median((c[:, 3] - c[:, 1]) / 100):.1f} us")
    st, en = (c[:, 1] - c[:, 1].min()) / 100, (c[:, 3] - c[:, 1].min()) / 100
    q = lambda v: " ".join(f"{x:.1f}" for x in np.percentile(v, [0, 10, 50, 90, 100]))  # noqa: E731
    print(f"   start us (p0 p10 p50 p90 p100): {q(st)};  end us: {q(en)};  span {en.max():.1f} us")


def phases(t, names):
    v = t[(t[:, 0] > 0)]
    v = v[1:-1] if len(v) > 3 else v
    d = np.diff(v[:, :len(names) + 1], axis=1)
    step = np.diff(v[:, 0])
    print("   " + "  ".join(f"{n}={int(np.median(d[:, i]))}" for i, n in enumerate(names)) +
          f"   band={int(np.median(step)) if len(step) else 0}")


print("k_fwd3 wave 0 (median cycles per band):")
phases(tr[0, 0, :, :5], ["barrier", "dma+copy", "conv", "epilogue"])
print("k_bwd3 dgrad wave 0:")
phases(tr[1, 0, :, :6], ["barrier", "mask+dma", "conv", "epilogue", "convert"])
print("k_bwd3 wgrad wave 4:")
phases(tr[1, 1, :, :5], ["barrier", "fold+xdma", "mfma", "halo+fold"])
# workgroup 0: cycles from its clock stamp to the first band, and from the last band to its end stamp
for k, role, last, name in ((0, 0, 4, "k_fwd3 wave 0"), (1, 0, 5, "k_bwd3 dgrad wave 0"), (1, 1, 4, "k_bwd3 wgrad wave 4")):
    t = tr[k, role]
    nbnd = int((t[:, 0] > 0).sum())
    if nbnd:
        pre = t[0, 0] - ck[k, 0, 0]
        post = ck[k, 0, 2] - t[nbnd - 1, last]
        print(f"{name}: {nbnd} bands; prologue {pre} cycles, after the last band {post} cycles, "
              f"first band {t[1, 0] - t[0, 0] if nbnd > 1 else 0}, last band {t[nbnd - 1, last] - t[nbnd - 1, 0]}")
