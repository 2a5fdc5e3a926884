"""development: run-to-run determinism of the network step.  Runs one
NetExecutor's forward_backward `--reps` times on the same parameters and
images and reports, per run that differs from the first, the loss difference
and the gradient groups (stem, each block's theta / bias, head) that differ.
usage: python tools/determinism.py [--lib build.so] [--cfg c2] [--reps 8]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib, runtime as rt  # noqa: E402
from differential_equations_resnet_amd.netparams import init_net_params  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--cfg", default="c2")
ap.add_argument("--reps", type=int, default=8)
ap.add_argument("--variant", type=int, default=0)
a = ap.parse_args()
if a.lib:
    _lib.load(path=os.path.abspath(a.lib))
C, L, N, integ = {"c2": (64, 30, 512, "euler"), "c3_64": (64, 108, 1024, "euler"), "c5": (64, 30, 512, "rk2"),
                  "c3": (16, 108, 1024, "euler")}[a.cfg]
dev = torch.device("cuda")
params = torch.from_numpy(init_net_params(C, L, 3, 10, seed=0) * 0.5).to(dev)
rng = np.random.default_rng(7)
imgs = torch.from_numpy(rng.integers(0, 256, (N, 32, 32, 3), dtype=np.uint8)).to(dev)
tgt = torch.from_numpy(np.eye(10, dtype=np.float32)[rng.integers(0, 10, N)]).to(dev)
ex = rt.NetExecutor(N, 32, 32, 3, C, L, 10, 8.0 / L, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                    dtype="bfloat16", input_u8=True, device=dev, integrator=integ)
ex.variant = a.variant
for _ in range(2):  # warm (first calls build maps / workspaces)
    loss0, g0 = ex.forward_backward(params, imgs, tgt)
loss0, g0 = loss0.clone(), g0.clone()
# parameter layout: [conv1 kernel, conv1 bias, (theta, bias) per block, fc kernel, fc bias]
sizes = [27 * C, C]
nth = (params.numel() - 27 * C - C - 10 * C - 10) // L - C
for _ in range(L):
    sizes += [nth, C]
sizes += [10 * C, 10]
assert sum(sizes) == params.numel()
offs = np.cumsum([0] + sizes)
bad = 0
for r in range(a.reps):
    loss, g = ex.forward_backward(params, imgs, tgt)
    torch.cuda.synchronize()
    if torch.equal(loss, loss0) and torch.equal(g, g0):
        continue
    bad += 1
    d = (g - g0).abs()
    groups = []
    for i in range(len(sizes)):
        m = d[offs[i]:offs[i + 1]].max().item()
        if m > 0:
            name = "conv1" if i < 2 else ("fc" if i >= len(sizes) - 2 else f"block{(i - 2) // 2}")
            groups.append(f"{name}{'.b' if i % 2 else ''}:{m:.2e}")
    print(f"{a.cfg} rep {r}: loss diff {(loss - loss0).abs().item():.3e}; differing groups {len(groups)}: "
          f"{' '.join(groups[:4])} ... {' '.join(groups[-6:])}", flush=True)
print(f"{a.cfg} variant {a.variant}: {bad} of {a.reps} runs differ from the first", flush=True)
st = rt.stack_status() if hasattr(rt, "stack_status") else None
print("stack status", st)
