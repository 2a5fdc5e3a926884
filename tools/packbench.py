"""development: the bf16 weight pack (asr_theta_to_w, balanced rounding) timed
alone: L layers at C = 16 / 32 / 64, HIP events around `reps` launches.
usage: python tools/packbench.py [--lib build.so] [--L 30] [--reps 50]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from differential_equations_resnet_amd import _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib")
ap.add_argument("--L", type=int, default=30)
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
if a.lib:
    _lib.load(path=os.path.abspath(a.lib))
from differential_equations_resnet_amd import runtime as rt  # noqa: E402

rt.require_gpu()
for C in (16, 32, 64):
    pm = rt.param_map(C)
    th = torch.from_numpy((np.random.default_rng(C).standard_normal(a.L * pm.n_theta) * 0.1).astype(np.float32)).cuda()
    for _ in range(3):
        rt.theta_to_w(th, C, pm, 0.0, rt.ASR_BF16, layers=a.L)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        rt.theta_to_w(th, C, pm, 0.0, rt.ASR_BF16, layers=a.L)
    e1.record()
    torch.cuda.synchronize()
    print(f"{a.lib or 'in-tree'} C={C} L={a.L}: {e0.elapsed_time(e1) * 1e3 / a.reps:.1f} us per pack")
