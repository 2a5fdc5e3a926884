#!/usr/bin/env python3
"""Headline benchmark: CIFAR-10 images/sec of one full training step
(forward + backward + Adam) of the antisymmetric ResNet on MI355X.

Workload (BASELINE.json configs[1], the metric's config): antisym-ResNet-32 —
get_single_block_resnet_build_function(kernel_type='antisymmetric',
num_stages=2, blocks_per_stage=[30], filters_per_block=[64], strides=[(1,1)],
subtract_mean=127.5, divide_by_stddev=127.5, num_classes=10), h = 8/30,
batch 512 per GPU, bf16 activations with fp32 accumulation and fp32
parameters/Adam.  Synthetic data (no dataset on the box): 8 batches of
uniform uint8 images with random labels, resident in HBM and cycled.
Weights: the reference initialisation (he_normal, truncated-normal thetas,
zero biases) with the block thetas scaled by 0.5 and the fc kernel by 0.1, so
that the timed steps are NOT in the saturated-softmax regime (at the plain
reference init this 30-block net starts at loss 13 with |logits| ~ 50 and
the Keras clip zeroes the gradient of most images; the line reports the
loss and the fraction of images with a live gradient, and fails below 0.9).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2]

--config c2_eval times the forward pass alone (the metric's model in
evaluation: asr_net_forward on the forward-only workspace, probabilities of
512 images per step; reference: Training._evaluate, training/training.py:670-706).

The line's `roofline` is measured on the timed step's own kernels: after the
timed region, --timed-steps more steps run with ASR_VARIANT_TIMED, which
records HIP events on the launch stream around the block launches inside
asr_net_forward_backward (the single k_fwd3_stack / k_bwd3_stack launches at
C2); their averages give `avg_us` and `frac`.  The random-operand timing of
the same kernels through the stack ABI is kept as `random_operand_leg`.

--gpus N > 1 without WORLD_SIZE in the environment re-launches this script
under torch.distributed.run (N processes, one per GPU) before touching the
GPU; with WORLD_SIZE set (the driver's own torchrun launch) each rank takes
512 images per step (weak scaling), the fp32 gradient buffer is all-reduced
through asr_dist_allreduce_sum (RCCL over xGMI) and Adam runs replicated.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "CIFAR-10 images/sec (fwd+bwd) antisym-ResNet-32 @ batch 512; 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (spec)
F32_PEAK_TFLOPS = 157.3
THETA_SCALE, FC_SCALE = 0.5, 0.1  # bench init (see the module docstring)
N_BATCHES = 8

CONFIGS = {
    # name: (C, L, per-GPU batch, dtype, description, integrator, mode)
    "c2": (64, 30, 512, "bfloat16", "antisym-ResNet-32 (C=64, 30 Euler blocks) batch 512/GPU bf16", "euler", "train"),
    "c2_eval": (64, 30, 512, "bfloat16", "antisym-ResNet-32 (C=64, 30 Euler blocks) batch 512/GPU bf16, forward only "
                "(evaluation)", "euler", "eval"),
    "c2_16": (16, 30, 512, "bfloat16", "antisym-ResNet-32 (C=16, 30 Euler blocks) batch 512/GPU bf16", "euler", "train"),
    "c1": (16, 18, 128, "float32", "antisym-ResNet-20 (C=16, 18 Euler blocks) batch 128 fp32", "euler", "train"),
    "c3": (16, 108, 1024, "bfloat16", "antisym-ResNet-110 (C=16, 108 Euler blocks) batch 1024 bf16", "euler", "train"),
    "c3_64": (64, 108, 1024, "bfloat16", "antisym-ResNet-110 (C=64, 108 Euler blocks) batch 1024 bf16", "euler",
              "train"),
    "c5": (64, 30, 512, "bfloat16", "antisym-ResNet-32 (C=64, 30 RK2 midpoint blocks) batch 512/GPU bf16", "rk2",
           "train"),
    "c2_f32": (64, 30, 512, "float32", "antisym-ResNet-32 (C=64, 30 Euler blocks) batch 512/GPU fp32 (the reference's "
               "precision, fp32 MFMA)", "euler", "train"),
    # the notebooks' trained model: 64 blocks x 16 filters, h = 8/64, batch 32 (experiments_antisymmetric_resnet_v6.ipynb
    # cells 1, 5, 9, :30-45, :107-135, :353-389) and its batch-1 predict (_v7.ipynb cells 19-25, :571-672)
    "v6": (16, 64, 32, "bfloat16", "antisym 64 blocks x 16 filters (v6 notebook model), batch 32 bf16", "euler",
           "train"),
    "v6_f32": (16, 64, 32, "float32", "antisym 64 blocks x 16 filters (v6 notebook model), batch 32 fp32", "euler",
               "train"),
    "v7_predict": (16, 64, 1, "bfloat16", "antisym 64 blocks x 16 filters, Model.predict of ONE image (v7 notebook "
                   "speed test), bf16", "euler", "eval"),
}
# multi-stage nets (asr_stages_*): name -> (stages [(C, L, transition stride)], per-GPU batch, dtype, description)
HE32 = ("He-style antisym-ResNet-32 (num_stages=4, blocks [10,10,10] at 32^2 x 16, 16^2 x 32, 8^2 x 64, stride-2 "
        "single_layer_conv_block transitions, tfkeras_resnets.py:575-593)")
STAGE_CONFIGS = {
    "he32": ([(16, 10, 0), (32, 9, 2), (64, 9, 2)], 128, "float32", HE32 + " batch 128/GPU fp32"),
    "he32_bf16": ([(16, 10, 0), (32, 9, 2), (64, 9, 2)], 512, "bfloat16",
                  HE32 + " batch 512/GPU bf16 (bf16 activations; identity blocks and their weight gradients on bf16 "
                         "MFMA with fp32 accumulation, the 32^2 x 16 stage's forward with bf16 hi + lo weights; fp32 "
                         "parameters, gradients and Adam; stem, transition and head weights fp32)"),
}
# the reference's own measurements of the same metric (TF 1.12, fp32, one NVIDIA GPU)
REFERENCE = {
    "v6": (46.7, "images/s", "training 1.46 it/s x 32, experiments_antisymmetric_resnet_v6.ipynb:362"),
    "v6_f32": (46.7, "images/s", "training 1.46 it/s x 32, experiments_antisymmetric_resnet_v6.ipynb:362"),
    "v7_predict": (5.02, "images/s", "batch-1 predict 0.1993 s/image, experiments_antisymmetric_resnet_v7.ipynb:650-651"),
}
METRICS = {
    "v6": "CIFAR-10 images/sec (fwd+bwd) antisym 64x16 (v6 notebook model) @ batch 32; 1 GPU",
    "v6_f32": "CIFAR-10 images/sec (fwd+bwd) antisym 64x16 (v6 notebook model) @ batch 32 fp32; 1 GPU",
    "v7_predict": "batch-1 Model.predict images/sec (1 / latency) antisym 64x16; 1 GPU",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS) + sorted(STAGE_CONFIGS))
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--block-reps", type=int, default=50)
    ap.add_argument("--timed-steps", type=int, default=10,
                    help="instrumented steps after the timed region: in-step kernel times for the roofline")
    ap.add_argument("--share-device", action="store_true",
                    help="test only: every rank on cuda:0 with its own RCCL host id (multi-rank rehearsal on one GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-random-leg", action="store_true",
                    help="skip the random-operand leg (profiling passes of the network's own kernels only)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every CPU this process may run on")
    ap.add_argument("--lib", default=None, help="development A/B only: load this libasr build instead of the in-tree one")
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """Re-run this script as N ranks under torch.distributed.run; the parent
    never touches the GPU and only relays the children's exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def bench_params(C, L):
    from differential_equations_resnet_amd.netparams import init_net_params, net_param_shapes
    flat = init_net_params(C, L, 3, 10, seed=0)
    sizes = [int(np.prod(s)) for s in net_param_shapes(C, L, 3, 10)]
    nt = 4 + C - 1  # theta arrays per block
    off = sizes[0] + sizes[1]
    for _ in range(L):
        n = sum(sizes[2:2 + nt])
        flat[off:off + n] *= THETA_SCALE
        off += n + C
    flat[off:off + C * 10] *= FC_SCALE
    return flat


def block_roofline(rt, lib, C, N, dtype_name, reps, h, integrator="euler"):
    """Time one block's kernels at the workload shape on random operands with
    HIP events on the launch stream (torch's current stream, which every
    libasr call here launches on); per-launch averages.

    Algorithmic bytes: Euler block 5·P·s (fwd: read x, write y;
    bwd: read dy, read x, write dx), forward 2·P·s, backward 3·P·s.  RK2 block
    12·P·s, the minimum of its two-stage composition with the midpoint stored:
    fwd read x, write xm, read xm, read x, write y; bwd stage 2 read dy, read
    xm, write g; stage 1 read g, read x, read dy, write dx."""
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

    def cs():  # the launch stream: torch's current one (a capture stream inside timed())
        return torch.cuda.current_stream().cuda_stream

    def fwd():
        _lib.check(lib.asr_conv_forward(0, x.data_ptr(), y.data_ptr(), mask.data_ptr(), w.data_ptr(),
                                        bias.data_ptr(), h, N, H, W, C, dt, cs()), "fwd")

    def bwd_kernel():  # dx only: the fused dgrad + wgrad kernel alone (no slab reduction / projection)
        _lib.check(lib.asr_conv_backward(0, dy.data_ptr(), x.data_ptr(), mask.data_ptr(), w.data_ptr(),
                                         theta_dst.data_ptr(), pm.n_theta, h, 0.0, N, H, W, C, dt, dx.data_ptr(),
                                         None, None, None, ws.data_ptr(), ws_bytes, cs()), "bwd")

    def bwd():
        _lib.check(lib.asr_conv_backward(0, dy.data_ptr(), x.data_ptr(), mask.data_ptr(), w.data_ptr(),
                                         theta_dst.data_ptr(), pm.n_theta, h, 0.0, N, H, W, C, dt, dx.data_ptr(),
                                         dth.data_ptr(), db.data_ptr(), None, ws.data_ptr(), ws_bytes, cs()), "bwd")

    if integrator == "rk2":
        xm = torch.empty_like(x)
        mask2 = torch.zeros_like(mask)
        ws_bytes = int(lib.asr_rk2_backward_workspace_bytes(N, H, W, C, dt))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)

        def fwd():  # noqa: F811
            _lib.check(lib.asr_rk2_forward(x.data_ptr(), xm.data_ptr(), y.data_ptr(), mask.data_ptr(),
                                           mask2.data_ptr(), w.data_ptr(), bias.data_ptr(), h, N, H, W, C, dt, cs()),
                       "rk2 fwd")

        def bwd():  # noqa: F811
            _lib.check(lib.asr_rk2_backward(dy.data_ptr(), x.data_ptr(), xm.data_ptr(), mask.data_ptr(),
                                            mask2.data_ptr(), w.data_ptr(), theta_dst.data_ptr(), pm.n_theta, h, 0.0,
                                            N, H, W, C, dt, dx.data_ptr(), dth.data_ptr(), db.data_ptr(), None,
                                            ws.data_ptr(), ws_bytes, cs()), "rk2 bwd")
        bwd_kernel = None

    for _ in range(10):
        fwd()
        bwd()
    torch.cuda.synchronize()
    timing_mode = [None]

    def timed(fn):
        # `reps` back-to-back launches captured in one HIP graph and replayed
        # between two events on the replay stream: per-launch averages without
        # the Python/ctypes launch path (at ~40 us per kernel that path, not the
        # GPU, would set the pace); eager launches if capture is unavailable
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        try:
            gr = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                fn()
            torch.cuda.current_stream().wait_stream(side)
            with torch.cuda.graph(gr):
                for _ in range(reps):
                    fn()
            gr.replay()
            torch.cuda.synchronize()
            e0.record()
            gr.replay()
            e1.record()
            torch.cuda.synchronize()
            timing_mode[0] = "hip graph of %d launches, events around the replay" % reps
        except Exception as ex:  # noqa: BLE001
            timing_mode[0] = "eager launches (graph capture failed: %s)" % type(ex).__name__
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    tf = timed(fwd)
    tbk = timed(bwd_kernel) if bwd_kernel is not None else None
    tb = timed(bwd)
    t_blk = timed(lambda: (fwd(), bwd()))
    esz = 2 if dt == rt.ASR_BF16 else 4
    P = N * H * W * C
    stages = 2 if integrator == "rk2" else 1
    bytes_alg = (12 if stages == 2 else 5) * P * esz  # see the docstring
    flops = stages * 3 * 2 * 9 * C * C * N * H * W
    # per pass: Euler fwd 2 (x, y), bwd 3 (dy, x, dx); RK2 fwd 5, bwd 7 (docstring)
    fb, bb = (5, 7) if stages == 2 else (2, 3)
    return dict(t_fwd=tf, t_bwd_kernel=tbk, t_bwd=tb, t=t_blk, bytes=bytes_alg, flops=flops,
                bytes_fwd=fb * P * esz, bytes_bwd=bb * P * esz, timing=timing_mode[0])


def stack_roofline(rt, N, L, reps, h, C=16, rk2=False):
    """The network's block path at the workload shape: all L Euler blocks in
    one forward and one backward launch (C=16: asr_deep16.hip, every image
    resident in LDS; C=64: k_fwd3_stack / k_bwd3_stack, whole images per
    workgroup), through asr_block_stack_forward / _backward, timed on random
    operands with HIP events on the launch stream (torch's current stream).

    Algorithmic bytes per image.  C=16, extended to the fused
    stack: forward reads x_0 and writes every x_l and its relu mask (the
    backward needs them): s·P + L·(s·P + P/8); backward reads every x_l and
    mask, dL/dx_L, and writes dx_0: L·(s·P + P/8) + 2·s·P (P = 32·32·16, s = 2 B).
    C=64: the survey's per-block unit 5·P·s (forward x, y; backward dy, x, dx),
    times L: x_l is re-read from HBM by every block there.  RK2 (config 5,
    asr_rk2_stack_forward / _backward): the RK2 block unit 12·P·s (forward 5
    passes: x, x_mid written and read, x again as the residual, y; backward 7)."""
    import torch
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    pm = rt.param_map(C)
    w = rt.theta_to_w(torch.randn(L * pm.n_theta, device=dev, generator=g) * 0.05, C, pm, 0.0, rt.ASR_BF16,
                      layers=L)
    bias = torch.randn(L, C, device=dev, generator=g) * 0.1
    x0 = torch.randn(N, 32, 32, C, device=dev, generator=g).to(torch.bfloat16)
    dyL = (torch.randn(N, 32, 32, C, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    from differential_equations_resnet_amd import _lib
    P = 32 * 32 * C
    mb = rt.mask_bytes(N, 32, 32, C)
    xs = torch.empty((L + 1, N, 32, 32, C), dtype=torch.bfloat16, device=dev)  # x_0, .., x_L: one stack
    xs[0].copy_(x0)
    masks = torch.empty((L, mb), dtype=torch.uint8, device=dev)
    wsb = int(_lib.load().asr_block_stack_backward_workspace_bytes(N, 32, 32, C, L, rt.ASR_BF16))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    dx0 = torch.empty_like(x0)
    dparams = torch.empty(L, pm.n_theta + C, dtype=torch.float32, device=dev)
    _, theta_dst = pm.device(dev)
    s = torch.cuda.current_stream().cuda_stream
    per = w[0].numel()

    if rk2:
        xm = torch.empty((L, N, 32, 32, C), dtype=torch.bfloat16, device=dev)
        masks2 = torch.empty((L, mb), dtype=torch.uint8, device=dev)
        wsb = int(_lib.load().asr_rk2_stack_backward_workspace_bytes(N, 32, 32, C, L, rt.ASR_BF16))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)

        def fwd():  # x_1 .. x_L behind x_0, the L x_mid and both masks of every block
            _lib.call("asr_rk2_stack_forward", xs[0].data_ptr(), xs[1].data_ptr(), xm.data_ptr(), N * P,
                      masks.data_ptr(), masks2.data_ptr(), mb, w.data_ptr(), per, bias.data_ptr(), C, float(h), N, 32,
                      32, C, L, rt.ASR_BF16, s)

        def bwd():
            _lib.call("asr_rk2_stack_backward", dyL.data_ptr(), xs.data_ptr(), xm.data_ptr(), N * P,
                      masks.data_ptr(), masks2.data_ptr(), mb, w.data_ptr(), per, theta_dst.data_ptr(), pm.n_theta,
                      float(h), 0.0, N, 32, 32, C, L, rt.ASR_BF16, dx0.data_ptr(), dparams.data_ptr(), ws.data_ptr(),
                      wsb, s)
    else:
        def fwd():  # writes x_1 .. x_L behind x_0 and the L masks
            _lib.call("asr_block_stack_forward", xs[0].data_ptr(), xs[1].data_ptr(), N * P, masks.data_ptr(), mb,
                      w.data_ptr(), per, bias.data_ptr(), C, float(h), N, 32, 32, C, L, rt.ASR_BF16, 1, s)

        def bwd():  # incl. the slab reduction and projection onto theta
            _lib.call("asr_block_stack_backward", dyL.data_ptr(), xs.data_ptr(), N * P, masks.data_ptr(), mb,
                      w.data_ptr(), per, theta_dst.data_ptr(), pm.n_theta, float(h), 0.0, N, 32, 32, C, L,
                      rt.ASR_BF16, dx0.data_ptr(), dparams.data_ptr(), ws.data_ptr(), wsb, s)

    fwd()
    bwd()
    torch.cuda.synchronize()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    tf = timed(fwd)
    tb = timed(bwd)
    if C == 16:
        act = L * (2 * P + P // 8)
        bytes_fwd, bytes_bwd = N * (2 * P + act), N * (act + 4 * P)
    elif rk2:
        bytes_fwd, bytes_bwd = N * L * 5 * 2 * P, N * L * 7 * 2 * P
    else:
        bytes_fwd, bytes_bwd = N * L * 2 * 2 * P, N * L * 3 * 2 * P
    flops = (2 if rk2 else 1) * 3 * 2 * 9 * C * C * 32 * 32 * N * L
    return dict(t_fwd=tf, t_bwd=tb, t=tf + tb, bytes=bytes_fwd + bytes_bwd, flops=flops, bytes_fwd=bytes_fwd,
                bytes_bwd=bytes_bwd)


def cpu_baseline(threads, c1_only=False):
    """The oracle's PyTorch-CPU restatements of the reference TF graph
    (oracle/torch_cpu_ref.py), timed on this box's host cores: the metric's
    workload (C2: C=64, 30 blocks, batch 512) with the reference's op-by-op
    kernel assembly (the headline value) and with the vectorised assembly, and
    BASELINE config C1 (C=16, 18 blocks, batch 128).  One untimed step (oneDNN
    primitive creation), then whole training steps (fwd + bwd + Adam)."""
    import torch
    from oracle import asr_oracle as O
    from oracle.torch_cpu_ref import RefNet
    torch.set_num_threads(threads)
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass

    def run(C, L, batch, steps, assembly):
        spec = O.NetSpec(C=C, L=L, h=8.0 / L)
        rng = np.random.default_rng(0)
        net = RefNet(O.init_params(spec, rng, np.float32), C, L, 8.0 / L, assembly=assembly)
        imgs = rng.integers(0, 256, (batch, 32, 32, 3)).astype(np.uint8)
        onehot = np.eye(10, dtype=np.float32)[rng.integers(0, 10, batch)]
        net.train_step(imgs, onehot)
        t0 = time.perf_counter()
        for _ in range(steps):
            net.train_step(imgs, onehot)
        dt = time.perf_counter() - t0
        print(f"bench: cpu baseline C={C} L={L} batch {batch} ({assembly}): {batch * steps / dt:.2f} images/s",
              file=sys.stderr, flush=True)
        return round(batch * steps / dt, 3), dt

    if c1_only:  # --config c1: BASELINE C1 itself
        c1, t1 = run(16, 18, 128, 4, "reference")
        return {"value": c1, "unit": "images/s", "cores": threads, "kind": "port",
                "sample": f"4 training steps (fwd+bwd+Adam) of BASELINE C1 (C=16, 18 blocks, batch 128, fp32) in the "
                          f"torch-CPU op-by-op restatement of the reference TF graph, after 1 untimed step; "
                          f"{t1:.1f} s on {threads} threads of {cpu}"}
    c2, t2 = run(64, 30, 512, 1, "reference")
    c2v, t2v = run(64, 30, 512, 1, "vectorised")
    c1, t1 = run(16, 18, 128, 2, "reference")
    return {"value": c2, "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"1 training step (fwd+bwd+Adam) of the metric's model (C=64, 30 blocks, batch 512, fp32) in "
                      f"the torch-CPU op-by-op restatement of the reference TF graph (per-step slice/neg/concat "
                      f"kernel assembly), after 1 untimed step; {t2:.1f} s on {threads} threads of {cpu}",
            "vectorised_assembly": {"value": c2v, "unit": "images/s", "seconds": round(t2v, 2),
                                    "sample": "same, W = P - P* + gamma*I as one gather per block"},
            "c1": {"value": c1, "unit": "images/s", "seconds": round(t1, 2),
                   "sample": "BASELINE C1: C=16, 18 blocks, batch 128, fp32, op-by-op assembly, 2 steps"}}


def host_threads() -> int:
    """CPUs this process may use: its affinity set, capped by a cgroup CPU
    quota when one is set (the GPU box shows the whole machine's CPUs)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return n


def traffic_record(config):
    """HBM traffic per block from the committed rocprofv3 PMC summary
    (profiles/traffic_<config>.json, written by tools/traffic.py from
    separate FETCH_SIZE / WRITE_SIZE passes with the gfx950 x2 read
    correction) — labelled with its round tag; null if none."""
    path = os.path.join(HERE, "profiles", f"traffic_{config}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_block"), f"profiles/traffic_{config}.json ({d.get('round', '?')})"


def co_bound(config, flops, bytes_blk, t_blk, train, dtype_name):
    """The MFMA side of the co-bound, at the clock the chip holds: the held
    clock of the block kernels comes from the committed PMC pass over the same
    bench command (profiles/clock_<config>.json, tools/clock.py:
    GRBM_GUI_ACTIVE / 8 XCDs / kernel time, time-weighted over the forward and
    backward kernels).  mfma_frac_held_clock = achieved FLOP/s / (1024 SIMDs x
    FLOP/clk/SIMD x that clock); hbm_frac_at_mfma_ceiling = the HBM fraction
    these algorithmic bytes would reach if the MFMA pipes were busy 100 % of
    that time (the ceiling of `frac` for this FLOP count).  None without the
    file or for an fp32 line."""
    path = os.path.join(HERE, "profiles", f"clock_{config}.json")
    if dtype_name != "bfloat16" or not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    ghz = d.get("clock_ghz_train" if train else "clock_ghz_fwd")
    if not ghz:
        return None
    flop_per_clk = 1024 * 1024  # 1024 SIMDs x 1024 bf16 FLOP/clk (v_mfma_f32_16x16x32_bf16: 16384 FLOP / 16 clk)
    peak = flop_per_clk * ghz * 1e9
    t_mfma = flops / peak
    return {"mfma_frac_held_clock": round(flops / t_blk / peak, 4), "held_clock_ghz": round(ghz, 3),
            "mfma_peak_held_clock_tflops": round(peak / 1e12, 1),
            "hbm_frac_at_mfma_ceiling": round(bytes_blk / t_mfma / 1e9 / HBM_PEAK_GBS, 4),
            "clock_source": f"profiles/clock_{config}.json ({d.get('round', '?')})"}


def algorithmic_bytes(C, L, N, esz, integrator, deep):
    """Per-step algorithmic bytes of the blocks' forward and backward (SURVEY
    §8d; see stack_roofline / block_roofline for the per-config units)."""
    P = 32 * 32 * C
    if deep:  # C=16 fused stack: every x_l and mask written once and read once
        act = L * (esz * P + P // 8)
        return N * (esz * P + act), N * (act + 2 * esz * P)
    if integrator == "rk2":
        return N * L * 5 * esz * P, N * L * 7 * esz * P
    return N * L * 2 * esz * P, N * L * 3 * esz * P


def cpu_eval_baseline(threads):
    """Forward-only CPU baseline for --config c2_eval: the oracle's PyTorch-CPU
    op-by-op restatement (oracle/torch_cpu_ref.py) evaluating the metric's
    model on 512 images (no autograd), after one untimed pass."""
    import torch
    from oracle import asr_oracle as O
    from oracle.torch_cpu_ref import RefNet
    torch.set_num_threads(threads)
    spec = O.NetSpec(C=64, L=30, h=8.0 / 30)
    rng = np.random.default_rng(0)
    net = RefNet(O.init_params(spec, rng, np.float32), 64, 30, 8.0 / 30)
    imgs = rng.integers(0, 256, (512, 32, 32, 3)).astype(np.uint8)
    with torch.no_grad():
        net.forward(imgs)
        t0 = time.perf_counter()
        net.forward(imgs)
        dt = time.perf_counter() - t0
    return {"value": round(512 / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"1 forward pass of the metric's model (C=64, 30 blocks, batch 512, fp32) in the torch-CPU "
                      f"op-by-op restatement of the reference TF graph, after 1 untimed pass; {dt:.1f} s"}


def cpu_stages_baseline(threads, stages, flat, h, images=256):
    """CPU baseline of a multi-stage net (--config he32 / he32_bf16): the
    oracle's numpy restatement of the reference graph (oracle.asr_oracle
    stages_forward / stages_backward: tfkeras_resnets.py:547-597 with the
    single_layer_conv_block transitions, :204-269) in float32 on a bounded
    sample of `images` images, forward + backward (no Adam: elementwise,
    <1 % of a step), after one untimed pass."""
    import threadpoolctl
    from oracle import asr_oracle as O
    spec = O.StagesSpec(stages=[tuple(s) for s in stages], h=h)
    shapes = spec.param_shapes()
    params, o = [], 0
    for shp in shapes:
        k = int(np.prod(shp))
        params.append(flat[o:o + k].reshape(shp).astype(np.float32))
        o += k
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (images, 32, 32, 3)).astype(np.uint8)
    onehot = np.eye(10, dtype=np.float32)[rng.integers(0, 10, images)]
    with threadpoolctl.threadpool_limits(threads):
        def one():
            probs, cache = O.stages_forward(spec, params, imgs, dtype=np.float32)
            O.stages_backward(spec, params, cache, onehot)
        one()
        t0 = time.perf_counter()
        one()
        dt = time.perf_counter() - t0
    return {"value": round(images / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"1 forward + backward of {images} images in the oracle's numpy float32 restatement of the "
                      f"reference graph (stages_forward / stages_backward), after 1 untimed pass; {dt:.1f} s on "
                      f"{threads} threads (BLAS)"}


def stages_params(stages, num_classes=10, seed=0):
    """Flat parameters in the asr_stages_config order: he_normal (2-sigma
    truncated) kernels, zero biases, block thetas x THETA_SCALE and the fc
    kernel x FC_SCALE (as bench_params)."""
    from differential_equations_resnet_amd import runtime as rt
    rng = np.random.default_rng(seed)

    def he(shape, fan_in, scale=1.0):
        return (np.clip(rng.standard_normal(shape), -2, 2) * np.sqrt(2.0 / fan_in) * scale).astype(np.float32)
    out = [he(3 * 3 * 3 * stages[0][0], 27), np.zeros(stages[0][0], np.float32)]
    Cp = stages[0][0]
    for C, L, S in stages:
        if S:
            out += [he(9 * Cp * C, 9 * Cp), np.zeros(C, np.float32), he(Cp * C, Cp), np.zeros(C, np.float32)]
        for _ in range(L):
            out += [he(rt.theta_count(C), 9 * C, THETA_SCALE), np.zeros(C, np.float32)]
        Cp = C
    out += [he(Cp * num_classes, Cp, FC_SCALE), np.zeros(num_classes, np.float32)]
    return np.concatenate(out)


def stages_main(args):
    """--config he32 / he32_bf16: one training step (fwd + bwd + Adam) of a multi-stage
    net on the asr_stages_* executor, same timing contract as main()."""
    import torch
    from differential_equations_resnet_amd import _lib, distributed, runtime as rt
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    if args.lib:
        _lib.load(path=os.path.abspath(args.lib))
    dev = rt.require_gpu()
    distributed.init_from_env(device=dev)
    stages, N, dtype, desc = STAGE_CONFIGS[args.config]
    L = sum(l for _, l, _ in stages)
    h = 8.0 / L
    ex = rt.StagesExecutor(N, 32, 32, 3, stages, 10, h, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                           input_u8=True, device=dev, dtype=dtype)
    params = torch.from_numpy(stages_params(stages)).to(dev)
    assert params.numel() == ex.n_params
    distributed.broadcast_params(params, 0)
    m, v = torch.zeros_like(params), torch.zeros_like(params)
    rng = np.random.default_rng(1234 + rank)
    batches = [(torch.from_numpy(rng.integers(0, 256, (N, 32, 32, 3), dtype=np.uint8)).to(dev),
                torch.from_numpy(np.eye(10, dtype=np.float32)[rng.integers(0, 10, N)]).to(dev))
               for _ in range(N_BATCHES)]
    k = [0]

    def step():
        images, targets = batches[k[0] % N_BATCHES]
        k[0] += 1
        loss, grads = ex.forward_backward(params, images, targets)
        distributed.allreduce_grads(grads)
        rt.adam_update(params, grads, m, v, args.lr, 0.9, 0.999, 1e-7, k[0], 1.0 / world)
        return loss
    first = None
    for i in range(args.warmup):
        out = step()
        if i == 0:
            first = float(out.item())
    distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    distributed.barrier()
    torch.cuda.synchronize()
    elapsed = distributed.max_over_ranks(time.perf_counter() - t0)
    value = N * world * args.steps / elapsed
    if rank == 0:
        # conv FLOPs per image, forward: stem, transitions (3x3 + 1x1), identity blocks; train = 3x forward
        fl, Hc, Cp = 2 * 9 * 3 * stages[0][0] * 32 * 32, 32, stages[0][0]
        for C, Lb, S in stages:
            if S:
                Hc = -(-Hc // S)
                fl += 2 * 10 * Cp * C * Hc * Hc
            fl += Lb * 2 * 9 * C * C * Hc * Hc
            Cp = C
        tflops = 3 * fl * N * world / (elapsed / args.steps) / 1e12 / world
        peak = BF16_PEAK_TFLOPS if dtype == "bfloat16" else F32_PEAK_TFLOPS
        out_line = {
            "metric": f"CIFAR-10 images/sec (fwd+bwd) {desc}; {world} GPU", "value": round(value, 1),
            "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16" if dtype == "bfloat16" else "f32",
            "data": f"synthetic ({N_BATCHES} HBM-resident batches of uniform uint8 32x32x3 images, random one-hot "
                    f"labels; he_normal init, thetas x{THETA_SCALE}, fc x{FC_SCALE})",
            "config": {"workload": desc + "; train step = fwd + bwd + Adam (asr_stages_forward_backward)",
                       "global_batch": N * world, "per_gpu_batch": N, "stages": stages, "h": round(h, 6),
                       "parallelism": f"dp{world}", "initial_loss": round(first, 4) if first is not None else None,
                       "final_loss": round(float(out.item()), 4)},
            "roofline": {"bound": "mfma", "achieved": round(tflops, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(tflops / peak, 4), "traffic": None,
                         "kernel": "whole step per GPU (conv FLOPs 3 x forward / step time; all kernels incl. "
                                   "stem, head, reductions, Adam)"},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out_line["cpu_baseline"] = cpu_stages_baseline(args.cpu_threads or host_threads(), stages,
                                                           params.cpu().numpy(), h)
        print(json.dumps(out_line), flush=True)
    distributed.shutdown()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if args.config in STAGE_CONFIGS:
        return stages_main(args)

    import torch
    from differential_equations_resnet_amd import _lib, distributed, runtime as rt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if args.share_device:  # test only: all ranks on one device, RCCL told they are on different hosts
        local = 0
        os.environ["NCCL_HOSTID"] = f"asr-bench-rank-{rank}"
    torch.cuda.set_device(local)
    if args.lib:
        _lib.load(path=os.path.abspath(args.lib))
    dev = rt.require_gpu()
    distributed.init_from_env(device=dev)  # RCCL communicator through asr_dist_init (world > 1)
    lib = _lib.load()

    C, L, N, dtype_name, desc, integrator, mode = CONFIGS[args.config]
    train = mode == "train"
    h = 8.0 / L  # final_time 8 (experiments_antisymmetric_resnet_v6.ipynb cell 1)
    ex = rt.NetExecutor(N, 32, 32, 3, C, L, 10, h, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                        dtype=dtype_name, input_u8=True, device=dev, integrator=integrator, inference=not train)
    # ranks sharing one device (test only) cannot keep both stacked backward grids resident: their
    # in-launch slab hand-offs degrade (bounded waits, the flagged blocks reduced after the launch;
    # counted in degraded_handoffs) -- slower, the same gradients
    base_variant = 0
    ex.variant = base_variant
    if train:
        rt.stack_status(reset=True)
    params = torch.from_numpy(bench_params(C, L)).to(dev)
    distributed.broadcast_params(params, 0)
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    rng = np.random.default_rng(1234 + rank)
    batches = []
    for _ in range(N_BATCHES):
        labels = rng.integers(0, 10, N)
        batches.append((torch.from_numpy(rng.integers(0, 256, (N, 32, 32, 3), dtype=np.uint8)).to(dev),
                        torch.from_numpy(np.eye(10, dtype=np.float32)[labels]).to(dev), torch.from_numpy(labels)))
    step_no = [0]

    def step():
        images, targets, _ = batches[step_no[0] % N_BATCHES]
        step_no[0] += 1
        if not train:  # evaluation: the softmax outputs of the batch
            return ex.forward(params, images)
        loss, grads = ex.forward_backward(params, images, targets, want_probs=True)
        distributed.allreduce_grads(grads)
        rt.adam_update(params, grads, m, v, args.lr, 0.9, 0.999, 1e-7, step_no[0], 1.0 / world)
        return loss

    def live_fraction():
        """Images of the last step whose target probability lies inside the
        Keras clip range (their loss gradient is not clipped to zero)."""
        labels = batches[(step_no[0] - 1) % N_BATCHES][2].numpy()
        p = ex.probs.cpu().numpy()[np.arange(N), labels]
        return float(((p > 1e-7) & (p < 1 - 1e-7)).mean())

    initial_loss = None
    for i in range(args.warmup):
        out = step()
        if i == 0 and train:
            initial_loss = float(out.item())
    distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = distributed.max_over_ranks(elapsed)
    value = N * world * args.steps / elapsed
    final_loss = float(out.item()) if train else None
    live = -distributed.max_over_ranks(-live_fraction()) if train else None  # min over ranks
    if train:
        ex.check_status()  # blocking: every launch completed

    # the timed step's own block kernels: events inside instrumented steps (all ranks take part)
    ex.variant = rt.ASR_VARIANT_TIMED | base_variant
    kts = []
    for _ in range(max(1, args.timed_steps)):
        step()
        kts.append(ex.kernel_times())
    ex.variant = base_variant
    degraded = None
    if train:
        ex.check_status()
        degraded = rt.stack_status(reset=True)  # hand-offs of the timed + instrumented steps that degraded

    if rank == 0:
        def avg(key):
            vals = [k[key] for k in kts if k[key] is not None]
            return sum(vals) / len(vals) * 1e-6 if vals else None
        t_fwd, t_bwd, t_red = avg("fwd"), avg("bwd"), avg("bwd_reduce")
        esz = 2 if dtype_name == "bfloat16" else 4
        deep = dtype_name == "bfloat16" and C == 16 and integrator == "euler"
        stacked = dtype_name == "bfloat16" and C == 64
        b_fwd, b_bwd = algorithmic_bytes(C, L, N, esz, integrator, deep)
        stages = 2 if integrator == "rk2" else 1
        fl_fwd = stages * 2 * 9 * C * C * 32 * 32 * N * L
        if train:
            t_blk, bytes_blk, flops = t_fwd + t_bwd, b_fwd + b_bwd, 3 * fl_fwd
        else:
            t_blk, bytes_blk, flops = t_fwd, b_fwd, fl_fwd
        achieved = bytes_blk / t_blk / 1e9
        tflops = flops / t_blk / 1e12
        peak_tf = BF16_PEAK_TFLOPS if dtype_name == "bfloat16" else F32_PEAK_TFLOPS
        traffic, traffic_src = traffic_record(args.config)
        if deep:
            kname = ("fused stack of all L Euler blocks: deep::k_fwd16_fused (forward), deep::k_bwd16_fused "
                     "(backward)")
        elif stacked and integrator == "rk2":
            kname = "all L RK2 blocks (2L stages) in one launch each: blk::k_fwd3_stack<RK2>, blk::k_bwd3_stack<RK2>"
        elif stacked:
            kname = ("all L Euler blocks in one launch each: blk::k_fwd3_stack (forward), blk::k_bwd3_stack "
                     "(backward, pass 1 of the slab reduction in-launch)")
        elif dtype_name == "float32":
            kname = ("the per-block fp32 MFMA kernels of every block (asr_conv_f32.hip: k_conv32 forward / dgrad, "
                     "k_wgrad32; v_mfma_f32_16x16x4_f32)")
        else:
            kname = "the per-block kernels of every block"
        if not train:
            kname = ("all L Euler blocks in one launch: blk::k_fwd3_stack over two ping-pong activation slots, "
                     "no relu masks (forward only)" if stacked else kname + " (forward only)")
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": kname,
                "timing": (f"HIP events on the launch stream around the block launches inside "
                           f"{'asr_net_forward_backward' if train else 'asr_net_forward'} (ASR_VARIANT_TIMED), "
                           f"averaged over {len(kts)} instrumented steps after the timed region; the "
                           f"post-launch slab reductions and projection are excluded (kernels.bwd_reduce)"),
                "operands": "the timed step's own (network activations of the synthetic batches)",
                "algorithmic_bytes": bytes_blk, "avg_us": round(t_blk * 1e6, 2),
                "mfma_tflops": round(tflops, 1), "mfma_frac": round(tflops / peak_tf, 4),
                "kernels": {"fwd": {"avg_us": round(t_fwd * 1e6, 2), "algorithmic_bytes": b_fwd,
                                    "frac": round(b_fwd / t_fwd / 1e9 / HBM_PEAK_GBS, 4)}}}
        if dtype_name == "float32":
            # fp32 blocks sit far right of the fp32 ridge (157 TF / 8 TB/s = 20 FLOP/B; C=16: 43, C=64: 173):
            # the bound is the fp32 MFMA pipe (v_mfma_f32_16x16x4_f32 = the fp32 vector rate)
            roof.update({"bound": "mfma", "achieved": round(tflops, 2), "peak": F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tflops / F32_PEAK_TFLOPS, 4), "hbm_gbs": round(achieved, 1),
                         "hbm_frac": round(achieved / HBM_PEAK_GBS, 4)})
        if train:
            roof["kernels"]["bwd"] = {"avg_us": round(t_bwd * 1e6, 2), "algorithmic_bytes": b_bwd,
                                      "frac": round(b_bwd / t_bwd / 1e9 / HBM_PEAK_GBS, 4)}
            if t_red is not None:
                roof["kernels"]["bwd_reduce"] = {"avg_us": round(t_red * 1e6, 2)}
            # secondary: the same kernels through the layer/stack ABI on random operands
            if args.no_random_leg:
                rb = None
            elif stacked or deep:
                rb = stack_roofline(rt, N, L, max(2, args.block_reps // 10), h, C, rk2=integrator == "rk2")
            else:
                rb = block_roofline(rt, lib, C, N, dtype_name, args.block_reps, h, integrator)
            if rb is not None:
                roof["random_operand_leg"] = {
                    "avg_us": round(rb["t"] * 1e6, 2), "algorithmic_bytes": rb["bytes"],
                    "frac": round(rb["bytes"] / rb["t"] / 1e9 / HBM_PEAK_GBS, 4),
                    "fwd_us": round(rb["t_fwd"] * 1e6, 2), "bwd_with_reduction_us": round(rb["t_bwd"] * 1e6, 2),
                    "operands": f"random (x, dy ~ N(0,1) in {'bf16' if dtype_name == 'bfloat16' else 'fp32'}, "
                                f"theta ~ N(0, 0.05^2)) through the stack / layer ABI"}
        co = co_bound(args.config, flops, bytes_blk, t_blk, train, dtype_name)
        if co:
            roof.update(co)
        cpu = None
        if world == 1 and not args.no_cpu_baseline and integrator == "euler":
            threads = args.cpu_threads or host_threads()
            if args.config == "c2":
                cpu = cpu_baseline(threads)
            elif args.config == "c1":
                cpu = cpu_baseline(threads, c1_only=True)
            elif args.config == "c2_eval":
                cpu = cpu_eval_baseline(threads)
        ref = REFERENCE.get(args.config)
        out = {
            "metric": METRICS.get(args.config, (METRIC if train else METRIC.replace("(fwd+bwd)", "(forward only, "
                                                                                 "evaluation)"))
                                  if args.config in ("c2", "c2_eval") else
                                  f"CIFAR-10 images/sec ({'fwd+bwd' if train else 'forward only'}) {desc}; {world} GPU"),
            "value": round(value, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(value / ref[0], 1) if ref else None,
            "dtype": "bf16" if dtype_name == "bfloat16" else "f32",
            "data": f"synthetic ({N_BATCHES} HBM-resident batches of uniform uint8 32x32x3 images with random one-hot "
                    f"labels, cycled; reference init with block thetas x{THETA_SCALE} and fc kernel x{FC_SCALE})",
            "config": {"workload": desc + ("; train step = fwd + bwd + Adam" if train else "; step = forward of the "
                                           "batch (probabilities)"),
                       "global_batch": N * world, "per_gpu_batch": N, "channels": C, "blocks": L,
                       "integrator": integrator, "h": round(h, 6), "parallelism": f"dp{world}",
                       "collective": "asr_dist_allreduce_sum (RCCL)" if world > 1 and train else None,
                       "initial_loss": None if initial_loss is None else round(initial_loss, 4),
                       "final_loss": None if final_loss is None else round(final_loss, 4),
                       "live_gradient_fraction": None if live is None else round(live, 4),
                       "degraded_handoffs": degraded},
            "roofline": roof, "cpu_baseline": cpu,
        }
        if ref:
            out["baseline"] = {"value": ref[0], "unit": ref[1], "source": ref[2],
                               "hardware": "one NVIDIA GPU, TensorFlow 1.12, fp32 (BASELINE.md §1)"}
        print(json.dumps(out), flush=True)
    distributed.shutdown()
    if live is not None and live < 0.9:
        print(f"bench: only {live:.3f} of the images have a live loss gradient (saturated softmax)", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
