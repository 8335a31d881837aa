"""Flash attention (K7): forward + FA2 backward, causal or not, grouped-query heads."""
from __future__ import annotations

from typing import Optional

from ._lib import _require


_AttnFns = None

def _attn_fns():
    global _AttnFns
    if _AttnFns is not None:
        return _AttnFns
    import torch

    def _ok_view(t):
        return t.stride(-1) == 1 and all(st % 8 == 0 for st in t.stride()[:-1]) and t.data_ptr() % 16 == 0

    def _fix(t):
        return t if _ok_view(t) else t.contiguous()

    class _FlashAttention(torch.autograd.Function):
        @staticmethod
        def forward(ctx, q, k, v, causal, scale):
            q, k, v = _fix(q), _fix(k), _fix(v)
            o, lse = torch.ops.nbd.attn_fwd(q, k, v, causal, scale, None, None)
            ctx.save_for_backward(q, k, v, o, lse)
            ctx.causal, ctx.scale = causal, scale
            return o

        @staticmethod
        def backward(ctx, do):
            q, k, v, o, lse = ctx.saved_tensors
            B, H, T, D = q.shape
            Hkv = k.shape[1]
            dq = torch.empty(B, T, H, D, dtype=q.dtype, device=q.device).transpose(1, 2)
            dkv = torch.empty(B, T, 2, Hkv, D, dtype=q.dtype, device=q.device)
            dk, dv = dkv[:, :, 0].transpose(1, 2), dkv[:, :, 1].transpose(1, 2)
            torch.ops.nbd.attn_bwd(_fix(do), q, k, v, o, lse, ctx.causal, ctx.scale, dq, dk, dv, None, None)
            return dq, dk, dv, None, None

    def _split(qkv, H, Hkv):
        B, T, W = qkv.shape
        D = W // (H + 2 * Hkv)
        q = qkv[:, :, : H * D].view(B, T, H, D).transpose(1, 2)
        k = qkv[:, :, H * D:(H + Hkv) * D].view(B, T, Hkv, D).transpose(1, 2)
        v = qkv[:, :, (H + Hkv) * D:].view(B, T, Hkv, D).transpose(1, 2)
        return q, k, v

    class _FlashAttentionQKV(torch.autograd.Function):
        """[B, T, (H + 2·Hkv)·D] packed projection in, [B, T, H·D] out; the backward writes the
        packed gradient directly (no split/cat, no transposes).  Hkv < H: grouped-query attention."""

        @staticmethod
        def forward(ctx, qkv, n_head, n_kv, causal, scale, cos, sin):
            B, T, _ = qkv.shape
            q, k, v = _split(qkv, n_head, n_kv)
            o, lse = torch.ops.nbd.attn_fwd(q, k, v, causal, scale, cos, sin)
            ctx.save_for_backward(qkv, o, lse)
            ctx.n_head, ctx.n_kv, ctx.causal, ctx.scale = n_head, n_kv, causal, scale
            ctx.rope = (cos, sin)  # constant tables (no gradient), kept by reference
            return o.transpose(1, 2).reshape(B, T, -1)  # o is stored [B, T, H, D]: a view

        @staticmethod
        def backward(ctx, dy):
            qkv, o, lse = ctx.saved_tensors
            cos, sin = ctx.rope
            B, T, _ = qkv.shape
            q, k, v = _split(qkv, ctx.n_head, ctx.n_kv)
            dy = dy if dy.is_contiguous() else dy.contiguous()
            dqkv = torch.empty_like(qkv, memory_format=torch.contiguous_format)
            dq, dk, dv = _split(dqkv, ctx.n_head, ctx.n_kv)
            do = dy.view(B, T, ctx.n_head, -1).transpose(1, 2)
            torch.ops.nbd.attn_bwd(do, q, k, v, o, lse, ctx.causal, ctx.scale, dq, dk, dv, cos, sin)
            return dqkv, None, None, None, None, None, None

    _AttnFns = (_FlashAttention, _FlashAttentionQKV)
    return _AttnFns

def flash_supported(q) -> bool:
    """The HIP kernels cover bf16, head dim 64, T a multiple of 128 (GPT-2's shapes)."""
    import torch

    return (q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] == 64 and q.shape[-2] % 128 == 0
            and q.shape[-2] >= 128)

def flash_attention(q, k, v, causal: bool = False, scale: Optional[float] = None):
    """softmax(q·kᵀ·scale [+ causal mask])·v for [B, H, T, D] tensors — the HIP flash kernels
    (``csrc/kernels/attn.hip``) where :func:`flash_supported`, else PyTorch SDPA."""
    import torch.nn.functional as F

    sc = float(scale) if scale is not None else q.shape[-1] ** -0.5
    gqa = k.shape[1] != q.shape[1]
    if (flash_supported(q) and k.shape == v.shape and q.shape[0] == k.shape[0] and q.shape[2:] == k.shape[2:]
            and q.shape[1] % k.shape[1] == 0 and k.dtype == v.dtype == q.dtype):
        _require()
        return _attn_fns()[0].apply(q, k, v, bool(causal), sc)
    return F.scaled_dot_product_attention(q, k, v, is_causal=causal, scale=sc, enable_gqa=gqa)

def attention_qkv(qkv, n_head: int, causal: bool = True, scale: Optional[float] = None,
                  n_kv_head: Optional[int] = None, rope=None):
    """Multi-head attention straight from a packed [B, T, (H + 2·Hkv)·D] projection (GPT-2's
    ``c_attn`` output, or a fused Llama q|k|v projection) to [B, T, H·D].  ``n_kv_head`` < ``n_head``
    is grouped-query attention.  ``rope=(cos, sin)`` (tables from ``rope_tables``) applies rotary
    embeddings to q and k — inside the attention kernels on the HIP path."""
    import torch
    import torch.nn.functional as F

    B, T, W = qkv.shape
    Hkv = n_kv_head or n_head
    D = W // (n_head + 2 * Hkv)
    sc = float(scale) if scale is not None else D ** -0.5
    if (qkv.is_cuda and qkv.dtype == torch.bfloat16 and D == 64 and T % 128 == 0 and qkv.stride(-1) == 1
            and qkv.stride(1) % 8 == 0 and qkv.stride(0) % 8 == 0 and qkv.data_ptr() % 16 == 0
            and n_head % Hkv == 0):
        _require()
        cos, sin = rope if rope is not None else (None, None)
        from .gemm import _native

        if _native():  # the C++ autograd node (csrc/kernels/autograd.hip)
            return torch.ops.nbd.attn_qkv_ag(qkv, int(n_head), int(Hkv), bool(causal), sc, cos, sin)
        return _attn_fns()[1].apply(qkv, int(n_head), int(Hkv), bool(causal), sc, cos, sin)
    if rope is not None:
        from .llama import rope_

        qkv = rope_(qkv if qkv.is_contiguous() else qkv.contiguous(), rope[0], rope[1], n_head + Hkv, D)
    q = qkv[:, :, : n_head * D].view(B, T, n_head, D).transpose(1, 2)
    k = qkv[:, :, n_head * D:(n_head + Hkv) * D].view(B, T, Hkv, D).transpose(1, 2)
    v = qkv[:, :, (n_head + Hkv) * D:].view(B, T, Hkv, D).transpose(1, 2)
    y = F.scaled_dot_product_attention(q, k, v, is_causal=causal, scale=sc, enable_gqa=Hkv != n_head)
    return y.transpose(1, 2).reshape(B, T, n_head * D)
