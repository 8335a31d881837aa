"""Data-plane helpers: the ``rccl`` backend, DDP with fused HIP bucket kernels, tensor parallelism
(``parallel.tensor``), Ulysses sequence parallelism (``parallel.sequence``), expert parallelism (``parallel.expert``),
pipeline parallelism (``parallel.pipeline``),
ring-attention context parallelism (``parallel.context``)."""
from .backend import abort_process_group, init_data_plane, rccl_version, register_rccl_backend, resolve_backend

__all__ = ["abort_process_group", "init_data_plane", "rccl_version", "register_rccl_backend", "resolve_backend",
           "DistributedDataParallel", "bf16_compress_hook", "allreduce_hook", "broadcast_params", "broadcast_tensors",
           "tensor", "sequence", "expert", "pipeline", "pipeline_step", "MoE", "parallelize_gpt2", "parallelize_llama", "ColumnParallelLinear", "RowParallelLinear", "ulysses_attention", "context", "ring_attention", "mesh", "ParallelMesh", "p2p", "batch_isend_irecv"]


def __getattr__(name):
    if name in ("DistributedDataParallel", "bf16_compress_hook", "allreduce_hook", "broadcast_params",
                "broadcast_tensors"):
        from . import ddp

        return getattr(ddp, name)
    if name == "batch_isend_irecv":
        from . import p2p

        return p2p.batch_isend_irecv
    if name in ("tensor", "sequence", "expert", "pipeline", "context", "mesh", "p2p"):
        import importlib

        return importlib.import_module(f".{name}", __name__)
    if name in ("parallelize_gpt2", "parallelize_llama", "ColumnParallelLinear", "RowParallelLinear"):
        from . import tensor

        return getattr(tensor, name)
    if name == "pipeline_step":
        from . import pipeline

        return pipeline.pipeline_step
    if name == "MoE":
        from . import expert

        return expert.MoE
    if name == "ulysses_attention":
        from . import sequence

        return sequence.ulysses_attention
    if name == "ParallelMesh":
        from . import mesh

        return mesh.ParallelMesh
    if name == "ring_attention":
        from . import context

        return context.ring_attention
    raise AttributeError(name)
