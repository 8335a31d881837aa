"""Llama-family elementwise kernels (K11): rotary embedding in place, fused SwiGLU."""
from __future__ import annotations

from ._lib import _require


_LlamaFns = None

def _llama_fns():
    global _LlamaFns
    if _LlamaFns is not None:
        return _LlamaFns
    import torch

    def _c(t):
        return t if t.is_contiguous() else t.contiguous()

    class _RMSNorm(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, eps):
            y, _, rstd = torch.ops.nbd.rms_fwd(x, None, w, eps)
            ctx.save_for_backward(x, w, rstd)
            return y

        @staticmethod
        def backward(ctx, dy):
            x, w, rstd = ctx.saved_tensors
            dx, dw = torch.ops.nbd.rms_bwd(x, _c(dy), None, w, rstd)
            return dx, dw, None

    class _AddRMSNorm(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, delta, w, eps):
            y, s, rstd = torch.ops.nbd.rms_fwd(x, delta, w, eps)
            ctx.save_for_backward(s, w, rstd)
            return s, y

        @staticmethod
        def backward(ctx, ds, dy):
            s, w, rstd = ctx.saved_tensors
            if dy is None:
                return ds, ds, None, None
            dx, dw = torch.ops.nbd.rms_bwd(s, _c(dy), None if ds is None else _c(ds), w, rstd)
            return dx, dx, dw, None

    class _Rope(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, cos, sin, n_rot, head_dim):
            torch.ops.nbd.rope_(x, cos, sin, n_rot, head_dim, False)
            ctx.mark_dirty(x)
            ctx.save_for_backward(cos, sin)
            ctx.n_rot, ctx.head_dim = n_rot, head_dim
            return x

        @staticmethod
        def backward(ctx, g):
            cos, sin = ctx.saved_tensors
            g = g.contiguous().clone()  # never rotate a gradient buffer someone else may hold
            torch.ops.nbd.rope_(g, cos, sin, ctx.n_rot, ctx.head_dim, True)
            return g, None, None, None, None

    class _SwiGLU(torch.autograd.Function):
        @staticmethod
        def forward(ctx, gu):
            ctx.save_for_backward(gu)
            return torch.ops.nbd.swiglu_fwd(gu)

        @staticmethod
        def backward(ctx, d):
            (gu,) = ctx.saved_tensors
            return torch.ops.nbd.swiglu_bwd(gu, _c(d))

    _LlamaFns = (_RMSNorm, _AddRMSNorm, _Rope, _SwiGLU)
    return _LlamaFns

def rope_tables(T: int, head_dim: int, theta: float, device, scaling=None) -> tuple:
    """cos/sin [T, head_dim/2] float32 for :func:`rope_` (HF default rope; ``scaling`` = Llama 3.x
    frequency scaling {factor, low_freq_factor, high_freq_factor, original_max_position_embeddings})."""
    import math

    import torch

    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float32, device=device) / head_dim))
    if scaling is not None:  # long wavelengths slowed by `factor`, short kept, a smooth blend between
        f, lo, hi = scaling["factor"], scaling["low_freq_factor"], scaling["high_freq_factor"]
        ctx = scaling["original_max_position_embeddings"]
        wavelen = 2 * math.pi / inv
        scaled = torch.where(wavelen > ctx / lo, inv / f, inv)
        smooth = (ctx / wavelen - lo) / (hi - lo)
        blended = (1 - smooth) * scaled / f + smooth * scaled
        medium = (wavelen >= ctx / hi) & (wavelen <= ctx / lo)
        inv = torch.where(medium, blended, scaled)
    f = torch.outer(torch.arange(T, dtype=torch.float32, device=device), inv)
    return f.cos().contiguous(), f.sin().contiguous()

def rope_(x, cos, sin, n_rot: int, head_dim: int):
    """Rotary embedding in place on the first ``n_rot`` heads of each row of a packed
    [B, T, H_total·head_dim] projection (HF rotate_half convention).  Returns ``x``."""
    import torch

    if x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and head_dim % 8 == 0 and x.is_contiguous():
        _require()
        return _llama_fns()[2].apply(x, cos, sin, int(n_rot), int(head_dim))
    B, T, W = x.shape
    half = head_dim // 2
    r = x[:, :, : n_rot * head_dim].view(B, T, n_rot, head_dim)
    a, b = r[..., :half].float(), r[..., half:].float()
    c, s_ = cos[:T, None, :], sin[:T, None, :]
    rot = torch.cat([a * c - b * s_, b * c + a * s_], -1).to(x.dtype).view(B, T, n_rot * head_dim)
    return torch.cat([rot, x[:, :, n_rot * head_dim:]], -1)

def swiglu(gu):
    """``silu(g) · u`` for a fused [..., 2I] gate|up projection (HIP fwd/bwd on GPU)."""
    import torch
    import torch.nn.functional as F

    I2 = gu.shape[-1]
    if gu.is_cuda and I2 % 16 == 0 and gu.dtype in (torch.bfloat16, torch.float16, torch.float32):
        _require()
        return _llama_fns()[3].apply(gu if gu.is_contiguous() else gu.contiguous())
    g, u = gu[..., : I2 // 2], gu[..., I2 // 2:]
    return F.silu(g) * u
