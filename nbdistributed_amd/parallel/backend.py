"""Data-plane bring-up: device binding and the ``rccl`` process-group backend.

Reference: ``worker.py:128-151`` sets RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*, binds
``torch.cuda.set_device(gpu_id or rank % n)`` and calls ``init_process_group("nccl" | "gloo")``;
the NCCL communicator is then created lazily by the first collective a user types.

MI355X-native version:

* ``"rccl"`` is registered as a first-class backend name (stock torch rejects it: SURVEY §0.1).
  On ROCm, torch's ProcessGroupNCCL *is* RCCL, so the creator builds a ProcessGroupNCCL with our
  options.  Collective streams use NORMAL priority: measured on MI355X (ROCm 7, GPT-2 small
  bf16 DDP step, benchmarks/ddp_compare.py), high-priority RCCL streams doubled the step time
  (55 ms vs 26 ms) — opt in with NBD_RCCL_HIGH_PRIORITY=1.
* The communicator is initialised eagerly during ``%dist_init`` with one tiny all-reduce, so the
  first collective inside a cell does not pay ncclCommInitRank (topology discovery + xGMI ring
  setup) — that cost moves to worker bring-up, where it belongs.
* Device binding uses ``HIP_VISIBLE_DEVICES`` ordering prepared by the launcher, so
  ``LOCAL_RANK`` == local device index == this rank's slot; libraries that read LOCAL_RANK
  (accelerate, reference bug D-12) pick the right GPU.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

_REGISTERED = False


def register_rccl_backend() -> bool:
    """Register ``backend="rccl"`` with torch.distributed (idempotent).  Returns False when this
    torch build has no ProcessGroupNCCL (CPU-only builds)."""
    global _REGISTERED
    if _REGISTERED:
        return True
    import torch.distributed as dist

    try:
        from torch.distributed import ProcessGroupNCCL
    except ImportError:
        return False

    high_prio = os.environ.get("NBD_RCCL_HIGH_PRIORITY", "0") not in ("0", "false", "False")

    def _create_rccl(store, rank, world_size, timeout):
        opts = ProcessGroupNCCL.Options(is_high_priority_stream=high_prio)
        if timeout is not None:
            opts._timeout = timeout
        return ProcessGroupNCCL(store, rank, world_size, opts)

    if "rccl" not in dist.Backend.backend_list:
        dist.Backend.register_backend("rccl", _create_rccl, devices=["cuda"])
    _REGISTERED = True
    return True


def resolve_backend(requested: Optional[str], cuda_available: bool) -> str:
    req = (requested or "auto").lower()
    if req == "auto":
        return "rccl" if cuda_available else "gloo"
    if req in ("rccl", "nccl") and not cuda_available:
        raise RuntimeError(f"backend {req!r} requested but no GPU is visible to this worker")
    return req


def rccl_version() -> Optional[str]:
    try:
        import torch

        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return None


def bind_device(local_index: Optional[int]):
    """Bind this process to its GPU; returns the torch.device (cpu when no GPU)."""
    import torch

    if torch.cuda.is_available() and local_index is not None:
        n = torch.cuda.device_count()
        idx = local_index % n if n else 0
        torch.cuda.set_device(idx)
        return torch.device("cuda", idx)
    return torch.device("cpu")


def init_data_plane(backend: str, rank: int, world_size: int, device, timeout_s: Optional[float] = None,
                    eager: bool = True, init_method: Optional[str] = None):
    """init_process_group + eager communicator creation.  Returns the default group."""
    import torch
    import torch.distributed as dist

    if backend == "rccl":
        if not register_rccl_backend():
            raise RuntimeError("this torch build has no ProcessGroupNCCL/RCCL")
    kw = {}
    if timeout_s:
        kw["timeout"] = datetime.timedelta(seconds=timeout_s)
    if backend in ("nccl", "rccl") and device is not None and device.type == "cuda":
        # bound device (both names are RCCL here): torch creates the communicator eagerly on it
        # (ProcessGroupNCCL.eager_connect_single_device) and every later device-less call —
        # a cell's plain dist.barrier(), new_group splits — uses it instead of guessing.  A bare
        # torch.device("cuda") means the current device (torch wants an index).
        kw["device_id"] = device if device.index is not None else torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group(backend=backend, rank=rank, world_size=world_size,
                            init_method=init_method or "env://", **kw)
    if eager:
        t = torch.zeros(1, device=device if device is not None else "cpu")
        dist.all_reduce(t)
        if device is not None and device.type == "cuda":
            torch.cuda.synchronize(device)
    return dist.group.WORLD


def abort_process_group() -> bool:
    """Abort the default group's communicators so ranks blocked in a collective unblock
    (used by the interrupt watchdog).  Returns True if something was aborted."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return False
    try:
        from torch.distributed.distributed_c10d import _abort_process_group

        _abort_process_group()
        return True
    except Exception:
        pass
    try:
        pg = dist.group.WORLD
        be = pg._get_backend(torch.device("cuda"))
        be.abort()
        return True
    except Exception:
        return False
