"""development: same-process A/B of ASR_VARIANT_* arms of the network executor
at a bench config: whole training steps (fwd + bwd + Adam) alternating between
the arms, plus the in-step block kernel times (ASR_VARIANT_TIMED) of each arm.
usage: python tools/varab.py [--config c2] [--arms 0,256] [--rounds 6] [--steps 20]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from differential_equations_resnet_amd import runtime as rt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
ap.add_argument("--arms", default="0,256")
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
C, L, N, dtype_name, desc, integrator, mode = bench.CONFIGS[a.config]
dev = rt.require_gpu()
h = 8.0 / L
ex = rt.NetExecutor(N, 32, 32, 3, C, L, 10, h, 0.0, subtract_mean=127.5, divide_by_stddev=127.5, dtype=dtype_name,
                    input_u8=True, device=dev, integrator=integrator)
params = torch.from_numpy(bench.bench_params(C, L)).to(dev)
m, v = torch.zeros_like(params), torch.zeros_like(params)
rng = np.random.default_rng(1234)
imgs = torch.from_numpy(rng.integers(0, 256, (N, 32, 32, 3), dtype=np.uint8)).to(dev)
tgt = torch.from_numpy(np.eye(10, dtype=np.float32)[rng.integers(0, 10, N)]).to(dev)
arms = [int(x) for x in a.arms.split(",")]
step_no = [0]


def step():
    step_no[0] += 1
    loss, g = ex.forward_backward(params, imgs, tgt)
    rt.adam_update(params, g, m, v, 1e-4, 0.9, 0.999, 1e-7, step_no[0])


res = {arm: {"ms": [], "fwd": [], "bwd": []} for arm in arms}
for arm in arms:
    ex.variant = arm
    for _ in range(5):
        step()
torch.cuda.synchronize()
for r in range(a.rounds):
    for arm in arms:
        ex.variant = arm
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        res[arm]["ms"].append((time.perf_counter() - t0) / a.steps * 1e3)
        ex.variant = arm | rt.ASR_VARIANT_TIMED
        step()
        kt = ex.kernel_times()
        res[arm]["fwd"].append(kt["fwd"])
        res[arm]["bwd"].append(kt["bwd"])
for arm in arms:
    d = res[arm]
    print(f"arm {arm}: ms/step {np.median(d['ms']):.4f} (min {min(d['ms']):.4f}) images/s {N / np.median(d['ms']) * 1e3:.0f}"
          f"  fwd {np.median(d['fwd']):.1f} us  bwd {np.median(d['bwd']):.1f} us  all ms {[round(x, 4) for x in d['ms']]}",
          flush=True)
print("degraded hand-offs:", rt.stack_status(reset=True))
