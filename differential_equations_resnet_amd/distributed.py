"""Data parallelism over torch.distributed: one process per GPU, RCCL
("nccl" backend on ROCm) between GPUs over xGMI, gloo for CPU tests.

The path shards by image (no BatchNorm, batch-mean loss), so
the only exchange is one all-reduce of the flat fp32 gradient buffer per
step (all dtheta, dbias, conv1 and fc gradients: 2.2 MB at C=64, L=30).  It is
a single bucket on purpose: at that size an xGMI ring is latency-bound, and
the backward of the last block finishes ~3 ms after the first gradient is
ready, so there is nothing to overlap finer buckets with that one launch
does not already hide.  Adam then runs replicated with grad_scale 1/world.
"""
from __future__ import annotations

import os

__all__ = ["init_from_env", "is_initialized", "rank", "world_size", "broadcast_params", "allreduce_grads",
           "max_over_ranks", "shutdown"]


def _dist():
    import torch.distributed as dist
    return dist


def is_initialized() -> bool:
    d = _dist()
    return d.is_available() and d.is_initialized()


def rank() -> int:
    return _dist().get_rank() if is_initialized() else 0


def world_size() -> int:
    return _dist().get_world_size() if is_initialized() else 1


def init_from_env(backend: str | None = None, device=None):
    """Initialise from RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (as set
    by torch.distributed.run); backend defaults to "nccl" (RCCL) when a
    device is given, else gloo.  No-op for WORLD_SIZE 1."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 or is_initialized():
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = backend or ("nccl" if device is not None else "gloo")
    kw = {}
    if backend == "nccl" and device is not None:
        kw["device_id"] = torch.device(device)
    _dist().init_process_group(backend, rank=int(os.environ["RANK"]), world_size=world, **kw)


def broadcast_params(params, src: int = 0):
    if is_initialized() and world_size() > 1:
        _dist().broadcast(params, src)


def allreduce_grads(grads):
    """Sum the flat gradient buffer over ranks in place; the optimizer
    applies the 1/world mean (asr_adam_update's grad_scale)."""
    if is_initialized() and world_size() > 1:
        _dist().all_reduce(grads)
    return grads


def max_over_ranks(value: float, device=None) -> float:
    import torch
    if not (is_initialized() and world_size() > 1):
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    _dist().all_reduce(t, op=_dist().ReduceOp.MAX)
    return float(t.item())


def shutdown():
    if is_initialized():
        _dist().barrier()
        _dist().destroy_process_group()
