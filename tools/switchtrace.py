"""development: every workgroup's stamps at every block switch of the stacked
C=64 backward (k_bwd3_stack), in the bench's own composition (C2: N=512,
L=30, the network executor, in-launch fold on), from a trace build
(-DASR_BLK_TRACE=1: g_bswitch, asr_debug_blk_switch).  Per switch (the first
band of block l) and over all workgroups: the done[] poll wait of the wgrad
wave that polls, the wgrad wave's band-barrier wait after it, the dgrad
wave's barrier wait, and the spread of the workgroups' arrival at the switch
(s_memrealtime, one time base).  Cycles at the in-kernel clock.
usage: python tools/switchtrace.py build_abl_tr.so [--N 512] [--L 30] [--raw]"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402
from differential_equations_resnet_amd.netparams import init_net_params  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("--N", type=int, default=512)
ap.add_argument("--L", type=int, default=30)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--raw", action="store_true", help="also print every workgroup's row for the worst switch")
a = ap.parse_args()
path = os.path.abspath(a.lib)
_lib.load(path=path)
dev = rt.require_gpu()
N, C, L = a.N, 64, a.L
ex = rt.NetExecutor(N, 32, 32, 3, C, L, 10, 8.0 / L, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                    dtype="bfloat16", input_u8=True, device=dev)
params = torch.from_numpy(init_net_params(C, L, 3, 10, seed=0) * 0.5).to(dev)
rng = np.random.default_rng(7)
imgs = torch.from_numpy(rng.integers(0, 256, (N, 32, 32, 3), dtype=np.uint8)).to(dev)
tgt = torch.from_numpy(np.eye(10, dtype=np.float32)[rng.integers(0, 10, N)]).to(dev)
for _ in range(a.steps):
    ex.forward_backward(params, imgs, tgt)
torch.cuda.synchronize()
cl = ctypes.CDLL(path)
buf = (ctypes.c_uint64 * (256 * 128 * 7))()
assert cl.asr_debug_blk_switch(buf, ctypes.sizeof(buf)) == 0
sw = np.frombuffer(buf, np.uint64).reshape(256, 128, 7).astype(np.int64)
grid = int((sw[:, L - 1, 0] > 0).sum())
sw = sw[:grid, :L]
print(f"k_bwd3_stack block switches: {grid} workgroups, {L} blocks (block L-1 starts the launch; its first band "
      f"has no poll); cycles at the in-kernel clock, realtime in us")
t0 = sw[:, L - 1, 5].min()
print("  block   poll p50/p90/max    wgrad bar p50/p90/max   dgrad bar p50/p90/max   arrival spread us  "
      "block us (from the previous switch)")
worst, wv = None, -1
for l in range(L - 1, -1, -1):
    s = sw[:, l]
    poll = s[:, 1] - s[:, 0]
    wbar = s[:, 2] - s[:, 1]
    dbar = s[:, 4] - s[:, 3]
    arr = (s[:, 5] - t0) / 100.0
    dur = "" if l == L - 1 else f"{(np.median(s[:, 6]) - np.median(sw[:, l + 1, 6])) / 100.0:9.1f}"
    q = lambda v: f"{int(np.median(v)):6d} {int(np.percentile(v, 90)):6d} {int(v.max()):6d}"  # noqa: E731
    print(f"  {l:5d}  {q(poll)}   {q(wbar)}   {q(dbar)}   {arr.max() - arr.min():8.2f}   {dur}")
    tot = int((poll + wbar).max())
    if l < L - 1 and tot > wv:
        worst, wv = l, tot
print(f"worst switch: block {worst} (max poll + wgrad barrier {wv} cycles)")
sl = sw[:, :L - 1]  # the switches with a poll (blocks L-2 .. 0)
ov_w = (sl[:, :, 2] - sl[:, :, 0]).ravel()
ov_d = (sl[:, :, 4] - sl[:, :, 3]).ravel()
print(f"mean switch overhead over {sl.shape[1]} switches x {grid} workgroups: wgrad wave poll + barrier "
      f"{ov_w.mean():.0f} cycles (p50 {np.median(ov_w):.0f}, p99 {np.percentile(ov_w, 99):.0f}), dgrad wave barrier "
      f"{ov_d.mean():.0f} cycles (p50 {np.median(ov_d):.0f}, p99 {np.percentile(ov_d, 99):.0f})")
if a.raw and worst is not None:
    s = sw[:, worst]
    print("  wg   poll  wgrad_bar  dgrad_bar  arrival_us")
    for w in np.argsort(-(s[:, 1] - s[:, 0]))[:32]:
        print(f"  {w:3d} {s[w, 1] - s[w, 0]:6d} {s[w, 2] - s[w, 1]:10d} {s[w, 4] - s[w, 3]:10d} "
              f"{(s[w, 5] - t0) / 100.0:10.2f}")

# per-XCD pace (workgroup w on XCD w % 8 under the dispatcher's round-robin): the in-kernel clock
# (s_memtime / s_memrealtime over the workgroup's run) and its end time, both stack kernels
tb = (ctypes.c_uint64 * (2 * 2 * 40 * 8))()
cb = (ctypes.c_uint64 * (2 * 1024 * 4))()
assert cl.asr_debug_blk_trace(tb, ctypes.sizeof(tb), cb, ctypes.sizeof(cb)) == 0
ck = np.frombuffer(cb, np.uint64).reshape(2, 1024, 4).astype(np.int64)
for k, name in ((0, "k_fwd3_stack"), (1, "k_bwd3_stack")):
    c = ck[k]
    ok = (c[:, 0] > 0) & (c[:, 2] > c[:, 0])
    idx = np.nonzero(ok)[0]
    c = c[ok]
    ghz = (c[:, 2] - c[:, 0]) / (c[:, 3] - c[:, 1]) * 0.1
    end = (c[:, 3] - c[:, 1].min()) / 100.0
    dur = (c[:, 3] - c[:, 1]) / 100.0
    print(f"{name}: {len(c)} workgroups, end us p0/p50/p100 {end.min():.1f}/{np.median(end):.1f}/{end.max():.1f}; "
          f"per XCD (wg % 8): clock GHz / run us median / end us max")
    print("   " + "  ".join(f"x{x}: {np.median(ghz[idx % 8 == x]):.3f} / {np.median(dur[idx % 8 == x]):.1f} / "
                            f"{end[idx % 8 == x].max():.1f}" for x in range(8) if (idx % 8 == x).any()))
# the forward's two workgroups per CU: the first-dispatched half (blockIdx < grid/2) vs the second
c = ck[0]
ok = (c[:, 0] > 0) & (c[:, 2] > c[:, 0])
idx = np.nonzero(ok)[0]
dur = (c[ok][:, 3] - c[ok][:, 1]) / 100.0
half = len(idx) // 2
print(f"k_fwd3_stack run us, blockIdx < {half}: p50 {np.median(dur[idx < half]):.1f} max {dur[idx < half].max():.1f}; "
      f">= {half}: p50 {np.median(dur[idx >= half]):.1f} max {dur[idx >= half].max():.1f}")
