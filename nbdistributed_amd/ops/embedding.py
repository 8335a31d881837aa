"""Embedding with a counting-sort weight gradient (K10): graph-safe, padding-robust."""
from __future__ import annotations

from ._lib import _require


_EmbFn = None

def _emb_fn():
    global _EmbFn
    if _EmbFn is None:
        import torch

        class _Embedding(torch.autograd.Function):
            @staticmethod
            def forward(ctx, idx, weight):
                ctx.save_for_backward(idx)
                ctx.V = weight.shape[0]
                return torch.nn.functional.embedding(idx, weight)

            @staticmethod
            def backward(ctx, dy):
                (idx,) = ctx.saved_tensors
                C = dy.shape[-1]
                dy2 = dy.reshape(-1, C)
                dy2 = dy2 if dy2.is_contiguous() else dy2.contiguous()
                return None, torch.ops.nbd.embedding_bwd(dy2, idx.reshape(-1).contiguous(), ctx.V)

        _EmbFn = _Embedding
    return _EmbFn

def embedding(idx, weight):
    """``F.embedding`` whose weight gradient comes from the HIP counting-sort kernels
    (``csrc/kernels/embed.hip``): deterministic launch shapes and caching-allocator memory only,
    so a step containing it can be captured in a HIP graph (torch's sort/unique path cannot)."""
    import torch

    C = weight.shape[-1]
    if (weight.is_cuda and idx.dtype == torch.int64 and C % 4 == 0 and C <= 4096 and weight.requires_grad
            and weight.dtype in (torch.bfloat16, torch.float16, torch.float32)):
        _require()
        return _emb_fn().apply(idx, weight)
    return torch.nn.functional.embedding(idx, weight)
