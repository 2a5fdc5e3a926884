"""One rank of the data-parallel GPU tests (tests/test_gpu_distributed.py),
launched by torch.distributed.run: the native executor's forward+backward on
this rank's slice of a fixed global batch, the gradient all-reduce through
the package's distributed layer (backend from argv), one Adam step with
grad_scale 1/world; results to <outdir>/r<rank>.npz.

usage: python -m torch.distributed.run --nproc-per-node 2 ... tests/dp_worker.py OUTDIR BACKEND [CASE]
BACKEND: "gloo", "rccl" (asr_dist_*), or "user_nccl" (the caller initialised
torch.distributed with nccl before the package's init_from_env).

CASE "small" (default): fp32, C=16, L=2, 4 images per rank (the per-block
fp32 kernels).  CASE "c2": BASELINE C4's per-rank composition at a reduced
depth: bf16, C=64, L=3, 192 images per rank, so every rank runs the stacked
kernels (k_fwd3_stack / k_bwd3_stack, several images per workgroup, the
in-launch slab fold: the production variant 0) before the all-reduce.  Both
ranks share the box's one device, so their two stacked-backward grids cannot
both be resident: the in-launch hand-off then degrades (bounded waits, the
flagged blocks reduced after the launch; the count is saved as `degraded`),
which must not change the gradients.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = {  # C, L, per-rank batch B, h, activation dtype
    "small": (16, 2, 4, 0.5, "float32"),
    "c2": (64, 3, 192, 8.0 / 30, "bfloat16"),
}
C, L, B, H, DTYPE = CASES["small"]


def use_case(name):
    global C, L, B, H, DTYPE
    C, L, B, H, DTYPE = CASES[name]


def global_batch(world):
    rng = np.random.default_rng(21)
    imgs = rng.integers(0, 256, (B * world, 32, 32, 3)).astype(np.uint8)
    onehot = np.eye(10, dtype=np.float32)[rng.integers(0, 10, B * world)]
    return imgs, onehot


def params0(seed):
    from differential_equations_resnet_amd.netparams import init_net_params
    return init_net_params(C, L, 3, 10, seed=seed, bias_std=0.05)


def main():
    outdir, backend = sys.argv[1], sys.argv[2]
    use_case(sys.argv[3] if len(sys.argv) > 3 else "small")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if backend in ("rccl", "user_nccl") and os.environ.get("ASR_TEST_SPLIT_HOSTID"):
        # two ranks on ONE device: RCCL refuses a duplicate GPU within a host,
        # so each rank claims its own host id and the ranks talk over sockets
        os.environ["NCCL_HOSTID"] = f"asr-dp-test-{rank}"
    import torch
    from differential_equations_resnet_amd import distributed, runtime as rt
    torch.cuda.set_device(0)
    dev = rt.require_gpu()
    if backend == "user_nccl":
        # the caller owns an nccl default group; the package adds a gloo group
        # for its host-side control plane and leaves the device collectives
        # to the default group
        torch.distributed.init_process_group("nccl", rank=rank, world_size=world)
        distributed.init_from_env(device=dev)
        assert distributed.device_backend() is None
    else:
        distributed.init_from_env(backend=backend, device=dev)
        assert distributed.device_backend() == backend
    assert distributed.world_size() == world
    params = torch.from_numpy(params0(100 + rank)).to(dev)  # differs per rank until the broadcast
    distributed.broadcast_params(params, 0)
    imgs, onehot = global_batch(world)
    sl = slice(rank * B, (rank + 1) * B)
    ex = rt.NetExecutor(B, 32, 32, 3, C, L, 10, H, 0.0, subtract_mean=127.5, divide_by_stddev=127.5,
                        dtype=DTYPE, input_u8=True, device=dev)
    # the production composition (variant 0, in-launch slab fold): ranks sharing one
    # device degrade the hand-off gracefully (rt.stack_status counts it)
    rt.stack_status(reset=True)
    loss, grads = ex.forward_backward(params, torch.from_numpy(imgs[sl]).to(dev), torch.from_numpy(onehot[sl]).to(dev))
    p_before = params.cpu().numpy()
    distributed.allreduce_grads(grads)
    m = torch.zeros_like(params)
    v = torch.zeros_like(params)
    rt.adam_update(params, grads, m, v, 1e-3, 0.9, 0.999, 1e-7, 1, 1.0 / world)
    distributed.barrier()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), g=grads.cpu().numpy(), p0=p_before, p1=params.cpu().numpy(),
             loss=loss.cpu().numpy(), t=distributed.max_over_ranks(1.0 + rank), degraded=rt.stack_status(reset=True))
    distributed.shutdown()


if __name__ == "__main__":
    main()
