#!/usr/bin/env python3
"""Headline benchmark: CIFAR-10 images/sec of one full training step
(forward + backward + Adam) of the antisymmetric ResNet on MI355X.

Workload (BASELINE.json configs[1], the metric's config): antisym-ResNet-32 —
get_single_block_resnet_build_function(kernel_type='antisymmetric',
num_stages=2, blocks_per_stage=[30], filters_per_block=[64], strides=[(1,1)],
subtract_mean=127.5, divide_by_stddev=127.5, num_classes=10), h = 8/30,
batch 512 per GPU, bf16 activations with fp32 accumulation and fp32
parameters/Adam.  Synthetic uniform uint8 images and random one-hot labels
(no dataset on the box), random-init weights of that architecture.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]

N > 1 is launched by torch.distributed.run, one process per GPU; the batch is
sharded by rank (512 per GPU, weak scaling) and the fp32 gradient buffer is
all-reduced with RCCL (backend "nccl") before the replicated Adam update.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "CIFAR-10 images/sec (fwd+bwd) antisym-ResNet-32 @ batch 512; 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (spec)
F32_PEAK_TFLOPS = 157.3

CONFIGS = {
    # name: (C, L, per-GPU batch, dtype, description, integrator)
    "c2": (64, 30, 512, "bfloat16", "antisym-ResNet-32 (C=64, 30 Euler blocks) batch 512/GPU bf16", "euler"),
    "c2_16": (16, 30, 512, "bfloat16", "antisym-ResNet-32 (C=16, 30 Euler blocks) batch 512/GPU bf16", "euler"),
    "c1": (16, 18, 128, "float32", "antisym-ResNet-20 (C=16, 18 Euler blocks) batch 128 fp32", "euler"),
    "c3": (16, 108, 1024, "bfloat16", "antisym-ResNet-110 (C=16, 108 Euler blocks) batch 1024 bf16", "euler"),
    "c3_64": (64, 108, 1024, "bfloat16", "antisym-ResNet-110 (C=64, 108 Euler blocks) batch 1024 bf16", "euler"),
    "c5": (64, 30, 512, "bfloat16", "antisym-ResNet-32 (C=64, 30 RK2 midpoint blocks) batch 512/GPU bf16", "rk2"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--block-reps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=16)
    ap.add_argument("--cpu-steps", type=int, default=2)
    return ap.parse_args()


def block_roofline(rt, lib, C, N, dtype_name, reps, h, integrator="euler"):
    """Time one block (fwd + full bwd) at the workload shape with HIP events
    on the launch stream; return per-launch averages.

    Algorithmic bytes: Euler block 5·P·s (fwd: read x, write y;
    bwd: read dy, read x, write dx).  RK2 block 12·P·s, the minimum of its
    two-stage composition with the midpoint stored: fwd read x, write xm,
    read xm, read x, write y; bwd stage 2 read dy, read xm, write g; stage 1
    read g, read x, read dy, write dx."""
    import torch
    from differential_equations_resnet_amd import _lib
    dev = torch.device("cuda")
    H = W = 32
    dt = rt.dtype_code(dtype_name)
    tdt = rt.torch_dtype(dt)
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(N, H, W, C, device=dev, generator=g).to(tdt)
    dy = torch.randn(N, H, W, C, device=dev, generator=g).to(tdt)
    y = torch.empty_like(x)
    dx = torch.empty_like(x)
    pm = rt.param_map(C)
    th = torch.randn(pm.n_theta, device=dev, generator=g) * 0.05
    bias = torch.zeros(C, device=dev)
    w = rt.theta_to_w(th, C, pm, 0.0, dt)
    mask = torch.zeros(rt.mask_bytes(N, H, W, C), dtype=torch.uint8, device=dev)
    ws_bytes = int(lib.asr_conv_backward_workspace_bytes(N, H, W, C, dt))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    dth = torch.empty(pm.n_theta, device=dev)
    db = torch.empty(C, device=dev)
    w_src, theta_dst = pm.device(dev)
    s = torch.cuda.current_stream().cuda_stream

    def fwd():
        _lib.check(lib.asr_conv_forward(0, x.data_ptr(), y.data_ptr(), mask.data_ptr(), w.data_ptr(),
                                        bias.data_ptr(), h, N, H, W, C, dt, s), "fwd")

    def bwd():
        _lib.check(lib.asr_conv_backward(0, dy.data_ptr(), x.data_ptr(), mask.data_ptr(), w.data_ptr(),
                                         theta_dst.data_ptr(), pm.n_theta, h, 0.0, N, H, W, C, dt, dx.data_ptr(),
                                         dth.data_ptr(), db.data_ptr(), None, ws.data_ptr(), ws_bytes, s), "bwd")

    if integrator == "rk2":
        xm = torch.empty_like(x)
        mask2 = torch.zeros_like(mask)
        ws_bytes = int(lib.asr_rk2_backward_workspace_bytes(N, H, W, C, dt))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)

        def fwd():  # noqa: F811
            _lib.check(lib.asr_rk2_forward(x.data_ptr(), xm.data_ptr(), y.data_ptr(), mask.data_ptr(),
                                           mask2.data_ptr(), w.data_ptr(), bias.data_ptr(), h, N, H, W, C, dt, s),
                       "rk2 fwd")

        def bwd():  # noqa: F811
            _lib.check(lib.asr_rk2_backward(dy.data_ptr(), x.data_ptr(), xm.data_ptr(), mask.data_ptr(),
                                            mask2.data_ptr(), w.data_ptr(), theta_dst.data_ptr(), pm.n_theta, h, 0.0,
                                            N, H, W, C, dt, dx.data_ptr(), dth.data_ptr(), db.data_ptr(), None,
                                            ws.data_ptr(), ws_bytes, s), "rk2 bwd")

    for _ in range(10):
        fwd()
        bwd()
    torch.cuda.synchronize()
    def timed(fn):
        # one event pair around `reps` back-to-back launches: the per-launch
        # average then matches rocprofv3's kernel durations (events between
        # every launch would add their own serialisation gaps)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    tf = timed(fwd)
    tb = timed(bwd)
    t_blk = timed(lambda: (fwd(), bwd()))
    esz = 2 if dt == rt.ASR_BF16 else 4
    P = N * H * W * C
    stages = 2 if integrator == "rk2" else 1
    bytes_alg = (12 if stages == 2 else 5) * P * esz  # see the docstring
    flops = stages * 3 * 2 * 9 * C * C * N * H * W
    return dict(t_fwd=tf, t_bwd=tb, t=t_blk, bytes=bytes_alg, flops=flops)


def cpu_baseline(C, L, h, batch, steps):
    """The oracle's op-by-op PyTorch-CPU restatement of the reference TF graph
    (oracle/torch_cpu_ref.py), timed on this box's host cores."""
    import torch
    from oracle import asr_oracle as O
    from oracle.torch_cpu_ref import RefNet
    cores = min(16, os.cpu_count() or 1)
    torch.set_num_threads(cores)
    spec = O.NetSpec(C=C, L=L, h=h)
    rng = np.random.default_rng(0)
    params = O.init_params(spec, rng, np.float32)
    net = RefNet(params, C, L, h)
    imgs = rng.integers(0, 256, (batch, 32, 32, 3)).astype(np.uint8)
    onehot = np.eye(10, dtype=np.float32)[rng.integers(0, 10, batch)]
    net.train_step(imgs, onehot)  # warm-up (allocations, oneDNN primitive creation)
    t0 = time.perf_counter()
    for _ in range(steps):
        net.train_step(imgs, onehot)
    dt = time.perf_counter() - t0
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(batch * steps / dt, 3), "unit": "images/s", "cores": cores, "kind": "port",
            "sample": f"{steps} training steps (fwd+bwd+Adam) of the same model (C={C}, {L} blocks) at batch {batch}, "
                      f"fp32, torch-CPU op-by-op restatement of the reference TF graph (per-step slice/neg/concat "
                      f"kernel assembly); {dt:.1f} s on {cores} threads of {cpu}"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from differential_equations_resnet_amd import _lib, runtime as rt
    from differential_equations_resnet_amd.netparams import init_net_params

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    dev = rt.require_gpu()
    lib = _lib.load()

    C, L, N, dtype_name, desc, integrator = CONFIGS[args.config]
    h = 8.0 / L  # final_time 8 (experiments_antisymmetric_resnet_v6.ipynb cell 1)
    ex = rt.NetExecutor(N, 32, 32, 3, C, L, 10, h, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                        dtype=dtype_name, input_u8=True, device=dev, integrator=integrator)
    params = torch.from_numpy(init_net_params(C, L, 3, 10, seed=0)).to(dev)
    if world > 1:
        dist.broadcast(params, 0)
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    rng = np.random.default_rng(1234 + rank)
    images = torch.from_numpy(rng.integers(0, 256, (N, 32, 32, 3), dtype=np.uint8)).to(dev)
    targets = torch.from_numpy(np.eye(10, dtype=np.float32)[rng.integers(0, 10, N)]).to(dev)
    step_no = [0]

    def step():
        loss, grads = ex.forward_backward(params, images, targets)
        if world > 1:
            dist.all_reduce(grads)
        step_no[0] += 1
        rt.adam_update(params, grads, m, v, args.lr, 0.9, 0.999, 1e-7, step_no[0], 1.0 / world)
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.item())
    value = N * world * args.steps / elapsed

    roof = None
    cpu = None
    if rank == 0:
        rb = block_roofline(rt, lib, C, N, dtype_name, args.block_reps, h, integrator)
        achieved = rb["bytes"] / rb["t"] / 1e9
        tflops = rb["flops"] / rb["t"] / 1e12
        peak_tf = BF16_PEAK_TFLOPS if dtype_name == "bfloat16" else F32_PEAK_TFLOPS
        traffic = None
        tpath = os.path.join(HERE, "profiles", f"traffic_{args.config}.json")
        if os.path.exists(tpath):
            with open(tpath) as f:
                traffic = json.load(f).get("hbm_bytes_per_block")
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": ("RK2 block fwd+bwd (2x blk::k_fwd_pipe, blk::k_bwd2 stage 2 + blk::k_bwd2<XT> stage 1 on one slab set, k_reduce_slabs, k_project)"
                           if integrator == "rk2" else
                           "Euler block fwd+bwd (blk::k_fwd_pipe, blk::k_bwd2 fused dgrad+wgrad, k_reduce_slabs, "
                           "k_project)"),
                "algorithmic_bytes": rb["bytes"], "avg_us": round(rb["t"] * 1e6, 2),
                "avg_us_fwd": round(rb["t_fwd"] * 1e6, 2), "avg_us_bwd": round(rb["t_bwd"] * 1e6, 2),
                "mfma_tflops": round(tflops, 1), "mfma_frac": round(tflops / peak_tf, 4)}
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(C, L, h, args.cpu_batch, args.cpu_steps) if integrator == "euler" else None
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if dtype_name == "bfloat16" else "f32",
            "data": "synthetic (uniform uint8 32x32x3 images, random one-hot labels; random-init weights)",
            "config": {"workload": desc + "; train step = fwd + bwd + Adam", "global_batch": N * world,
                       "per_gpu_batch": N, "channels": C, "blocks": L, "integrator": integrator, "h": round(h, 6),
                       "parallelism": f"dp{world}", "final_loss": round(final_loss, 4)},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
