"""Embedding with a counting-sort weight gradient (K10): graph-safe, padding-robust."""
from __future__ import annotations

import os

from ._lib import _require

# NBD_FUSED_EMBED=0: token and position lookups as two gathers + an add (A/B)
FUSED_EMBED = os.environ.get("NBD_FUSED_EMBED", "1") != "0"


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

_TokPosFn = None


def _tokpos_fn():
    global _TokPosFn
    if _TokPosFn is None:
        import torch

        class _TokPos(torch.autograd.Function):
            @staticmethod
            def forward(ctx, idx, wte, pos, wpe):
                ctx.save_for_backward(idx, pos)
                ctx.shapes = (wte.shape[0], wpe.shape[0])
                return torch.ops.nbd.embedding_tokpos(idx, wte, pos, wpe)

            @staticmethod
            def backward(ctx, dy):
                idx, pos = ctx.saved_tensors
                V, P = ctx.shapes
                C = dy.shape[-1]
                dy2 = dy.reshape(-1, C)
                dy2 = dy2 if dy2.is_contiguous() else dy2.contiguous()
                d_wte = torch.ops.nbd.embedding_bwd(dy2, idx.reshape(-1), V) if ctx.needs_input_grad[1] else None
                d_wpe = None
                if ctx.needs_input_grad[3]:
                    # positions repeat every T rows: sum the batch first (fp32), then place the T
                    # rows (unique positions: index_add_ without collisions — deterministic)
                    T = pos.numel()
                    s = dy2.view(-1, T, C).sum(0, dtype=torch.float32)
                    d_wpe = torch.zeros(P, C, dtype=torch.float32, device=dy.device).index_add_(0, pos, s).to(dy.dtype)
                return None, d_wte, None, d_wpe

        _TokPosFn = _TokPos
    return _TokPosFn


def embedding_tok_pos(idx, wte, pos, wpe):
    """``F.embedding(idx, wte) + F.embedding(pos, wpe)`` (GPT-2's input: token + learned position
    embeddings, ``idx`` [..., T], ``pos`` [T] of unique positions) in one HIP pass on the GPU; the
    backward sums the batch for the position table and uses the counting-sort kernels for the
    token table."""
    import torch

    C = wte.shape[-1]
    if (FUSED_EMBED and wte.is_cuda and idx.dtype == torch.int64 and pos.dtype == torch.int64 and C % 8 == 0 and C <= 4096
            and wte.dtype == wpe.dtype and wte.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and idx.shape[-1] == pos.numel() and pos.dim() == 1):
        _require()
        return _tokpos_fn().apply(idx.contiguous(), wte, pos.contiguous(), wpe)
    return embedding(idx, wte) + embedding(pos, wpe)


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
