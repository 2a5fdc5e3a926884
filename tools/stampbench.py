"""Diagnostic: per-phase cycles of the fused backward from the stamp build.
  tools/build_variants.sh stamp "-DASR_STAMP_BUILD=1"
  python3 tools/stampbench.py $PWD/build_abl_stamp.so
Reads SHARES (the stamps' own waits slow the build), averaged over WGs and
interior bands."""
import ctypes as ct
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402

WHAT = os.environ.get("STAMP_WHAT", "bwd")
lib = _lib.load(path=sys.argv[1] if len(sys.argv) > 1 else None)
dev = rt.require_gpu()
N, H, W, C = 512, 32, 32, 64
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
dy = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
y = torch.empty_like(x)
dx = torch.empty_like(x)
pm = rt.param_map(C)
th = torch.randn(pm.n_theta, device=dev, generator=g) * 0.05
w = rt.theta_to_w(th, C, pm, 0.0, rt.ASR_BF16)
mask = torch.zeros(rt.mask_bytes(N, H, W, C), dtype=torch.uint8, device=dev)
wsb = int(lib.asr_conv_backward_workspace_bytes(N, H, W, C, rt.ASR_BF16))
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
dth = torch.empty(pm.n_theta, device=dev)
db = torch.empty(C, device=dev)
bias = torch.zeros(C, device=dev)
_, tdst = pm.device(dev)
s = torch.cuda.current_stream().cuda_stream
_lib.check(lib.asr_conv_forward(0, x.data_ptr(), y.data_ptr(), mask.data_ptr(), w.data_ptr(), bias.data_ptr(), 0.25,
                                N, H, W, C, 1, s))
for _ in range(3 if WHAT.startswith("bwd") else 0):
    _lib.check(lib.asr_conv_backward(0, dy.data_ptr(), x.data_ptr(), mask.data_ptr(), w.data_ptr(), tdst.data_ptr(),
                                     pm.n_theta, 0.25, 0.0, N, H, W, C, 1, dx.data_ptr(), dth.data_ptr(),
                                     db.data_ptr(), None, ws.data_ptr(), wsb, s))
for _ in range(3 if WHAT == "fwd" else 0):
    _lib.check(lib.asr_conv_forward(0, x.data_ptr(), y.data_ptr(), mask.data_ptr(), w.data_ptr(), bias.data_ptr(),
                                    0.25, N, H, W, C, 1, s))
torch.cuda.synchronize()
st = np.zeros((512, 2, 16, 8), dtype=np.uint64)
fn = lib.asr_debug_stamps
fn.restype = ct.c_int
fn.argtypes = [ct.c_void_p, ct.c_size_t]
assert fn(st.ctypes.data, st.nbytes) == 0
st = st.astype(np.int64)
grid = int((st[:, 0, 0, 0] != 0).sum())
if WHAT.startswith("bwd"):  # the forward (run first) stamps more WGs than the backward's persistent grid
    grid = min(grid, torch.cuda.get_device_properties(dev).multi_processor_count)
st = st[:grid]
if os.environ.get("STAMP_RAW"):
    for b in (4, 5):
        for role in (0, 1):
            print("raw wg0 band", b, "role", role, (st[0, role, b, :] - st[0, 0, b, 0]).tolist())
order = None
if WHAT == "fwd":
    names = {0: ["barrier_vm", "dma issue", "conv+epilogue hooks", "xres read", "loop"]}
    # bands 1..5 of WGs whose stamps are all present (the last band of a run exits early)
    ok = (st[:, 0, 1:7, :5] > 0).all(axis=(1, 2))
    st = st[ok]
elif WHAT == "bwd2":  # k_bwd2 slots: dgrad 0 1 2(conv0) 4(epi0) 3(conv1) 5(epi1) 6(staged next); wgrad 0 1 2 3
    names = {0: ["barrier_vm", "row0 conv+dma", "row0 epi", "row1 conv", "row1 epi", "stage next band", "loop"],
             1: ["barrier_vm", "x dma", "wgrad kk loop", "tail"]}
    order = {0: [0, 1, 2, 4, 3, 5, 6], 1: [0, 1, 2, 3]}
else:
    names = {0: ["barrier_vm", "convert", "barrier_lds", "row0 conv+dma", "row0 epi", "row1 conv+epi", "tail"],
             1: ["barrier_vm", "convert", "barrier_lds", "dma share", "wgrad kk loop", "tail"]}
nb = 16 if WHAT.startswith("bwd") else 8
for role in names:
    seg = []
    for b in range(1, nb - 2 if WHAT == "fwd" else nb - 1):  # the forward's last band exits before its stamps
        row = st[:, role, b, :]
        if order is not None:
            row = row[:, order[role]]
        nxt = st[:, role, b + 1, 0]
        k = len(names[role])
        d = [row[:, i + 1] - row[:, i] for i in range(k - 1)] + [nxt - row[:, k - 1]]
        seg.append(np.stack(d, 1))
    seg = np.concatenate(seg)
    tot = seg.sum(1).mean()
    print(f"{WHAT} role {role} ({['dgrad/fwd wave 0', 'wgrad wave 4'][role]}): band = {tot:.0f} cycles")
    for i, n in enumerate(names[role]):
        print(f"   {n:>16s} {seg[:, i].mean():8.0f}  {100 * seg[:, i].mean() / tot:5.1f}%")
