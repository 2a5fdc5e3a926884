"""development: what the round-5 r05k failure was (gpurun_out/test_r05k.log:
the bf16 general-kind stages net at h = 0.5, four consecutive scalar
gradients grad[1265..1268] at relative error exactly 1.000, i.e. zero on the
GPU where the fp64 oracle's were not).  Rebuilds that case (the test's
_stages_setup, N = 8, seed 0), names the layer / channel the four tensors
belong to, and prints per tensor the GPU gradient, the plain fp64 oracle's and
the bf16-storage oracle's, plus that channel's pre-activation z in both
oracles (max and the count of z > 0): a channel that is dead in the bf16
forward (z <= 0 at every pixel) has an exactly zero gradient, while the fp64
forward, a rounding away, still has a few live pixels.
usage: python tools/r05k_dead_channel.py [--h 0.5]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from helpers import bf16_round, w_bf16_balanced  # noqa: E402
from oracle import asr_oracle as O  # noqa: E402
from test_gpu_stages import KINDS, _stages_setup, _t  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--h", type=float, default=0.5)
ap.add_argument("--idx", type=int, nargs="*", default=[1264, 1265, 1266, 1267, 1268, 1073])
a = ap.parse_args()

from differential_equations_resnet_amd.runtime import StagesExecutor, require_gpu  # noqa: E402

require_gpu()
stages, kind, anti = [(32, 1, 0), (64, 2, 2), (64, 1, 2)], "general", False
spec, params, imgs, onehot = _stages_setup(stages, kind, anti, h=a.h, gamma=0.0, N=8)
ex = StagesExecutor(imgs.shape[0], spec.H, spec.W, 3, stages, 10, spec.h, spec.gamma, subtract_mean=127.5,
                    divide_by_stddev=127.5, input_u8=True, param_kind=KINDS[kind], antisymmetric=anti,
                    dtype="bfloat16")
flat = _t(O.flatten(params))
loss, grads = ex.forward_backward(flat, torch.from_numpy(imgs).cuda(), _t(onehot))
g_got = O.unflatten(grads.cpu().numpy().astype(np.float64), [p.shape for p in params])
probs, cache = O.stages_forward(spec, params, imgs)
g_plain = O.stages_backward(spec, params, cache, onehot)
probs_s, cache_s = O.stages_forward(spec, params, imgs, rnd=bf16_round, rnd_w=w_bf16_balanced)
g_store = O.stages_backward(spec, params, cache_s, onehot)
# round 5's executor rounded W to nearest (r05k ran that)
probs_n, cache_n = O.stages_forward(spec, params, imgs, rnd=bf16_round)
g_near = O.stages_backward(spec, params, cache_n, onehot)

# which block / output channel owns each tensor index (general kind, O.theta_shapes_general: per
# output o its diagonal-block scalars, then its [3,3,C-o-1,1] kernel; then the block's bias)
owner, i, bi = {}, 2, 0
for si, (C, L, S) in enumerate(spec.stages):
    if S:
        i += 4
    free = O._cs_free_positions(3, anti)
    for b in range(L):
        for o in range(C):
            for pos in free:
                owner[i] = (si, b, bi, o, f"centro_sym_{pos[0]}_{pos[1]}")
                i += 1
            if C - o - 1 > 0:
                owner[i] = (si, b, bi, o, f"input_kernels_for_output_kernel_{o}")
                i += 1
        i += 1  # bias
        bi += 1
ops = [op for op in cache["ops"] if op[0] == "b"]
ops_s = [op for op in cache_s["ops"] if op[0] == "b"]
ops_n = [op for op in cache_n["ops"] if op[0] == "b"]
for k in a.idx:
    si, b, bi, o, shp = owner[k]
    z, zs, zn = ops[bi][2][..., o], ops_s[bi][2][..., o], ops_n[bi][2][..., o]
    print(f"grad[{k}] {shp}: stage {si} block {b}, output channel {o}: GPU {float(np.ravel(g_got[k])[0]):+.3e}  "
          f"fp64 {float(np.ravel(g_plain[k])[0]):+.3e}  bf16-storage {float(np.ravel(g_store[k])[0]):+.3e}  "
          f"bf16-storage with W to nearest (round 5) {float(np.ravel(g_near[k])[0]):+.3e}  |  channel z max "
          f"(px > 0): fp64 {z.max():+.3e} ({int((z > 0).sum())}), bf16-storage {zs.max():+.3e} ({int((zs > 0).sum())}), "
          f"W to nearest {zn.max():+.3e} ({int((zn > 0).sum())})")
