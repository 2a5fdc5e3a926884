"""development: is a config's training step host-bound?  Times the host side
of each step (the asr_*_forward_backward call + Adam enqueue, no sync) and
the device side (HIP events on the stream around the step), for the bench's
own composition.  usage: python tools/hostgap.py [--config he32_bf16] [--steps 50]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from differential_equations_resnet_amd import runtime as rt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="he32_bf16")
ap.add_argument("--steps", type=int, default=50)
a = ap.parse_args()
dev = rt.require_gpu()
stages, N, dtype, _ = bench.STAGE_CONFIGS[a.config]
L = sum(l for _, l, _ in stages)
ex = rt.StagesExecutor(N, 32, 32, 3, stages, 10, 8.0 / L, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                       input_u8=True, device=dev, dtype=dtype)
params = torch.from_numpy(bench.stages_params(stages)).to(dev)
m, v = torch.zeros_like(params), torch.zeros_like(params)
rng = np.random.default_rng(0)
imgs = torch.from_numpy(rng.integers(0, 256, (N, 32, 32, 3), dtype=np.uint8)).to(dev)
tgt = torch.from_numpy(np.eye(10, dtype=np.float32)[rng.integers(0, 10, N)]).to(dev)


def step(k):
    loss, grads = ex.forward_backward(params, imgs, tgt)
    rt.adam_update(params, grads, m, v, 1e-3, 0.9, 0.999, 1e-7, k, 1.0)


for k in range(5):
    step(k + 1)
torch.cuda.synchronize()
host, dev_ms = [], []
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
t_all = time.perf_counter()
for k in range(a.steps):
    evs[k][0].record()
    t0 = time.perf_counter()
    step(k + 6)
    host.append((time.perf_counter() - t0) * 1e6)
    evs[k][1].record()
torch.cuda.synchronize()
wall = (time.perf_counter() - t_all) / a.steps * 1e6
dev_ms = [e0.elapsed_time(e1) * 1e3 for e0, e1 in evs]
print(f"{a.config}: wall {wall:.1f} us/step; host enqueue p50 {np.median(host):.1f} us (min {min(host):.1f}, "
      f"max {max(host):.1f}); device step (events) p50 {np.median(dev_ms):.1f} us")
# the same steps queued back to back with one sync: the device-only rate
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for k in range(a.steps):
    step(k + 100)
e1.record()
torch.cuda.synchronize()
print(f"{a.config}: {a.steps} steps back to back: {e0.elapsed_time(e1) * 1e3 / a.steps:.1f} us/step (device clock)")
