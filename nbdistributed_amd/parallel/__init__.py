"""Data-plane helpers: the ``rccl`` backend, DDP with fused HIP bucket kernels, collectives."""
from .backend import abort_process_group, init_data_plane, rccl_version, register_rccl_backend, resolve_backend

__all__ = ["abort_process_group", "init_data_plane", "rccl_version", "register_rccl_backend", "resolve_backend",
           "DistributedDataParallel", "bf16_compress_hook", "allreduce_hook", "broadcast_params", "broadcast_tensors"]


def __getattr__(name):
    if name in ("DistributedDataParallel", "bf16_compress_hook", "allreduce_hook", "broadcast_params",
                "broadcast_tensors"):
        from . import ddp

        return getattr(ddp, name)
    raise AttributeError(name)
