"""development: one training step (fwd + bwd + Adam) captured in a HIP graph
(torch.cuda.CUDAGraph over the libasr launches on the capture stream) vs the
eager step, for the launch-bound small-batch configs.  Prints images/s of
both and checks that a replay gives the eager step's gradients bit for bit.
usage: python tools/graphbench.py [--config he32|c1] [--steps 50]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
from differential_equations_resnet_amd import runtime as rt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="he32")
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    dev = rt.require_gpu()
    if a.config in bench.STAGE_CONFIGS:
        stages, N, dt, _ = bench.STAGE_CONFIGS[a.config]
        L = sum(l for _, l, _ in stages)
        ex = rt.StagesExecutor(N, 32, 32, 3, stages, 10, 8.0 / L, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                               input_u8=True, device=dev, dtype=dt)
        params = torch.from_numpy(bench.stages_params(stages)).to(dev)
    else:
        C, L, N, dtype, _, integ, _ = bench.CONFIGS[a.config]
        ex = rt.NetExecutor(N, 32, 32, 3, C, L, 10, 8.0 / L, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                            dtype=dtype, input_u8=True, device=dev, integrator=integ)
        params = torch.from_numpy(bench.bench_params(C, L)).to(dev)
    rng = np.random.default_rng(0)
    images = torch.from_numpy(rng.integers(0, 256, (N, 32, 32, 3), dtype=np.uint8)).to(dev)
    targets = torch.from_numpy(np.eye(10, dtype=np.float32)[rng.integers(0, 10, N)]).to(dev)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    step_t = torch.ones(1, dtype=torch.int64)

    def step(k):
        ex.forward_backward(params, images, targets)
        rt.adam_update(params, ex.grads, m, v, 1e-3, 0.9, 0.999, 1e-7, k, 1.0)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            fn(k + 1)
        torch.cuda.synchronize()
        return N * a.steps / (time.perf_counter() - t0)
    for k in range(3):
        step(k + 1)
    eager = timed(step)
    # capture (Adam's step count is a host scalar baked into the graph: fixed lr_t, fine for timing)
    p0 = params.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step(5)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step(5)
    # parity: eager step vs replay from the same parameters
    params.copy_(p0)
    ex.forward_backward(params, images, targets)
    ge = ex.grads.clone()
    params.copy_(p0)
    g.replay()
    torch.cuda.synchronize()
    same = torch.equal(ge, ex.grads)
    graph = timed(lambda k: g.replay())
    print(f"{a.config}: eager {eager:.1f} images/s, graph {graph:.1f} images/s ({graph / eager:.3f}x); "
          f"replay grads bitwise equal to eager: {same}")


if __name__ == "__main__":
    main()
