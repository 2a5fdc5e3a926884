"""Data parallelism: one process per GPU, the gradient exchange on RCCL over
xGMI through libasr's C ABI (asr_dist_*), torch.distributed/gloo only as the
host control plane (rendezvous, barriers, host scalars).

The path shards by image (no BatchNorm, batch-mean loss), so
the only exchange is one all-reduce of the flat fp32 gradient buffer per
step (all dtheta, dbias, conv1 and fc gradients: 2.2 MB at C=64, L=30) plus
one broadcast of the initial parameters.  It is a single bucket on purpose:
at that size an xGMI ring is latency-bound (≈25 µs of bandwidth term on
7 × 153 GB/s links against a multi-ms step), so finer buckets overlapped
with the backward would buy nothing a single launch does not.  Adam then
runs replicated with grad_scale 1/world.

Device collective backends:
  "rccl" (default with a GPU): asr_dist_unique_id on rank 0, the 128-byte id
          broadcast over the gloo control plane, asr_dist_init on every rank;
          asr_dist_allreduce_sum / asr_dist_broadcast on the current stream.
  "gloo": torch.distributed over gloo for the device tensors too — CPU tests
          and the 2-ranks-on-one-GPU test (RCCL refuses two ranks on one
          device).
The reference has no counterpart (it is single-device,
experiments_antisymmetric_resnet_v6.ipynb:361).
"""
from __future__ import annotations

import os

__all__ = ["init_from_env", "is_initialized", "rank", "world_size", "device_backend", "broadcast_params",
           "allreduce_grads", "max_over_ranks", "barrier", "shutdown"]

_state = {"backend": None, "ctrl": None, "owns_default": False}


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


def device_backend() -> str | None:
    """'rccl', 'gloo' or None (single process)."""
    return _state["backend"]


def init_from_env(backend: str | None = None, device=None):
    """Initialise from RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (as set
    by torch.distributed.run).  backend: "rccl" (default when `device` is a
    GPU device) or "gloo".  No-op for WORLD_SIZE 1."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if is_initialized():
        # The caller made the default group.  The control plane all-reduces
        # host float64 tensors, so it needs a gloo group of its own when the
        # default one is nccl (collective: every rank calls this).
        if _dist().get_backend() != "gloo" and _state["ctrl"] is None:
            _state["ctrl"] = _dist().new_group(backend="gloo")
        return
    if world <= 1:
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    on_gpu = device is not None and torch.device(device).type == "cuda"
    backend = backend or ("rccl" if on_gpu else "gloo")
    if backend not in ("rccl", "gloo"):
        raise ValueError(f"unknown device collective backend {backend!r} ('rccl' or 'gloo')")
    r = int(os.environ["RANK"])
    _dist().init_process_group("gloo", rank=r, world_size=world)  # host control plane
    _state["owns_default"] = True  # shutdown() may tear the default group down
    if backend == "rccl":
        if not on_gpu:
            raise ValueError("the rccl backend needs a GPU device")
        from . import _lib
        uid = torch.zeros(_lib.ASR_DIST_UNIQUE_ID_BYTES, dtype=torch.uint8)
        if r == 0:
            _lib.call("asr_dist_unique_id", uid.data_ptr())
        _dist().broadcast(uid, 0)
        _lib.call("asr_dist_init", r, world, uid.data_ptr())
    _state["backend"] = backend


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def _dtype_code(t):
    import torch
    from . import _lib
    if t.dtype == torch.float32:
        return _lib.ASR_F32
    if t.dtype == torch.bfloat16:
        return _lib.ASR_BF16
    raise ValueError(f"collectives take float32 or bfloat16 buffers, not {t.dtype}")


def _rccl_check(t, what):
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError(f"{what}: RCCL buffers must be contiguous device tensors")


def broadcast_params(params, src: int = 0):
    if not (is_initialized() and world_size() > 1):
        return
    if _state["backend"] == "rccl":
        from . import _lib
        _rccl_check(params, "broadcast_params")
        _lib.call("asr_dist_broadcast", params.data_ptr(), params.numel(), _dtype_code(params), int(src), _stream())
    else:
        _dist().broadcast(params, src)


def allreduce_grads(grads):
    """Sum the flat gradient buffer over ranks in place; the optimizer
    applies the 1/world mean (asr_adam_update's grad_scale)."""
    if not (is_initialized() and world_size() > 1):
        return grads
    if _state["backend"] == "rccl":
        from . import _lib
        _rccl_check(grads, "allreduce_grads")
        _lib.call("asr_dist_allreduce_sum", grads.data_ptr(), grads.numel(), _dtype_code(grads), _stream())
    else:
        _dist().all_reduce(grads)
    return grads


def max_over_ranks(value: float, device=None) -> float:
    """Max of a host scalar over ranks (control plane)."""
    import torch
    if not (is_initialized() and world_size() > 1):
        return float(value)
    t = torch.tensor([value], dtype=torch.float64)
    _dist().all_reduce(t, op=_dist().ReduceOp.MAX, group=_state["ctrl"])
    return float(t.item())


def sum_over_ranks(values):
    """Elementwise sum of a host float vector over ranks (control plane)."""
    import torch
    t = torch.tensor(list(values), dtype=torch.float64)
    if is_initialized() and world_size() > 1:
        _dist().all_reduce(t, group=_state["ctrl"])
    return t.tolist()


def barrier(device_sync: bool = True):
    """Host barrier over ranks, with this rank's device work drained first."""
    import torch
    if device_sync and torch.cuda.is_available():
        torch.cuda.synchronize()
    if is_initialized() and world_size() > 1:
        _dist().barrier()


def shutdown():
    """Finalise the RCCL communicator and destroy the groups this package
    created: the default group only when init_from_env made it (a caller that
    owns its default group keeps it; only the gloo control group goes)."""
    if is_initialized():
        _dist().barrier()
        if _state["backend"] == "rccl":
            from . import _lib
            _lib.call("asr_dist_finalize")
        if _state["owns_default"]:
            _dist().destroy_process_group()
        elif _state["ctrl"] is not None:
            _dist().destroy_process_group(_state["ctrl"])
    _state["backend"] = None
    _state["ctrl"] = None
    _state["owns_default"] = False
