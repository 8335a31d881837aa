"""LayerNorm / RMSNorm with fused residual adds, bias-gradient column sums, Linear (K8, K9, K11)."""
from __future__ import annotations

import os

from ._lib import _require
from .gemm import _native
from .llama import _llama_fns


_NormFns = None

def _norm_fns():
    global _NormFns
    if _NormFns is not None:
        return _NormFns
    import torch

    def _c(t):
        return t if t.is_contiguous() else t.contiguous()

    class _LayerNorm(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, b, eps):
            y, _, mean, rstd = torch.ops.nbd.ln_fwd(x, None, w, b, eps)
            ctx.save_for_backward(x, w, mean, rstd)
            return y

        @staticmethod
        def backward(ctx, dy):
            x, w, mean, rstd = ctx.saved_tensors
            dx, dw, db = torch.ops.nbd.ln_bwd(x, _c(dy), None, w, mean, rstd)
            return dx, dw, db, None

    class _AddLayerNorm(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, delta, w, b, eps):
            y, s, mean, rstd = torch.ops.nbd.ln_fwd(x, delta, w, b, eps)
            ctx.save_for_backward(s, w, mean, rstd)
            return s, y

        @staticmethod
        def backward(ctx, ds, dy):
            s, w, mean, rstd = ctx.saved_tensors
            if dy is None:
                return ds, ds, None, None, None
            dx, dw, db = torch.ops.nbd.ln_bwd(s, _c(dy), None if ds is None else _c(ds), w, mean, rstd)
            return dx, dx, dw, db, None

    class _Linear(torch.autograd.Function):
        """F.linear forward (hipBLASLt, bias fused in the epilogue); backward with the two GEMMs
        and the bias gradient from the HIP column-sum kernel."""

        @staticmethod
        def forward(ctx, x, w, b):
            ctx.save_for_backward(x, w)
            ctx.has_bias = b is not None
            return torch.nn.functional.linear(x, w, b)

        @staticmethod
        def backward(ctx, dy):
            x, w = ctx.saved_tensors
            dy2 = _c(dy).view(-1, dy.shape[-1])
            dx = dw = db = None
            if ctx.needs_input_grad[0]:
                dx = (dy2 @ w).view(x.shape)
            if ctx.needs_input_grad[1]:
                dw = dy2.t() @ _c(x).view(-1, x.shape[-1])
            if ctx.has_bias and ctx.needs_input_grad[2]:
                db = torch.ops.nbd.colsum(dy2, w.dtype)
            return dx, dw, db

    _NormFns = (_LayerNorm, _AddLayerNorm, _Linear)
    return _NormFns

def _norm_ok(x, C: int) -> bool:
    import torch

    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and C % 8 == 0 and C <= 2048
            and not torch.is_autocast_enabled())

def layer_norm(x, weight, bias, eps: float = 1e-5):
    """LayerNorm over the last dim (HIP kernels on GPU; ``F.layer_norm`` otherwise)."""
    import torch
    import torch.nn.functional as F

    C = x.shape[-1]
    if _norm_ok(x, C) and weight is not None and bias is not None and weight.dtype == x.dtype:
        _require()
        if _native():
            return torch.ops.nbd.layer_norm_ag(x if x.is_contiguous() else x.contiguous(), weight, bias, float(eps))
        return _norm_fns()[0].apply(x if x.is_contiguous() else x.contiguous(), weight, bias, float(eps))
    return F.layer_norm(x, (C,), weight, bias, eps)

def add_layer_norm(x, delta, weight, bias, eps: float = 1e-5):
    """``s = x + delta; return s, LayerNorm(s)`` — the residual add and the norm in one HIP pass
    (and their backward in one pass: dx includes the residual stream's gradient)."""
    import torch
    import torch.nn.functional as F

    C = x.shape[-1]
    if (_norm_ok(x, C) and weight is not None and bias is not None and weight.dtype == x.dtype
            and delta.dtype == x.dtype and delta.shape == x.shape):
        _require()
        x, delta = (x if x.is_contiguous() else x.contiguous()), (delta if delta.is_contiguous() else delta.contiguous())
        if _native():
            return torch.ops.nbd.add_layer_norm_ag(x, delta, weight, bias, float(eps))
        return _norm_fns()[1].apply(x, delta, weight, bias, float(eps))
    s = x + delta
    return s, F.layer_norm(s, (C,), weight, bias, eps)

def linear(x, weight, bias=None):
    """``F.linear`` whose backward computes the bias gradient with the HIP column-sum kernel."""
    import torch.nn.functional as F

    import torch

    if (bias is not None and x.is_cuda and weight.shape[0] % 8 == 0 and x.dtype == weight.dtype == bias.dtype
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and not torch.is_autocast_enabled()):
        _require()
        return _norm_fns()[2].apply(x, weight, bias)
    return F.linear(x, weight, bias)

def colsum(x, dtype=None):
    """Σ over all rows of ``x`` [..., C] (fp32 accumulation), as ``dtype`` (default x.dtype)."""
    import torch

    C = x.shape[-1]
    if x.is_cuda and C % 8 == 0:
        _require()
        return torch.ops.nbd.colsum(x if x.is_contiguous() else x.contiguous(), dtype or x.dtype)
    return x.reshape(-1, C).float().sum(0).to(dtype or x.dtype)

def _rms_ok(x, w) -> bool:
    import torch

    C = x.shape[-1]
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and C % 8 == 0 and C <= 2048
            and w.dtype == x.dtype and not torch.is_autocast_enabled())

def rms_norm(x, weight, eps: float = 1e-6):
    """RMSNorm over the last dim: ``x · rsqrt(mean(x²) + eps) · weight`` (HIP on GPU)."""
    import torch

    if _rms_ok(x, weight):
        _require()
        if _native():
            return torch.ops.nbd.rms_norm_ag(x if x.is_contiguous() else x.contiguous(), weight, float(eps))
        return _llama_fns()[0].apply(x if x.is_contiguous() else x.contiguous(), weight, float(eps))
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * weight

def add_rms_norm(x, delta, weight, eps: float = 1e-6):
    """``s = x + delta; return s, RMSNorm(s)`` in one HIP pass (and one for the backward)."""
    if _rms_ok(x, weight) and delta.dtype == x.dtype and delta.shape == x.shape:
        _require()
        x, delta = (x if x.is_contiguous() else x.contiguous()), (delta if delta.is_contiguous() else delta.contiguous())
        if _native():
            import torch

            return torch.ops.nbd.add_rms_norm_ag(x, delta, weight, float(eps))
        return _llama_fns()[1].apply(x, delta, weight, float(eps))
    s = x + delta
    return s, rms_norm(s, weight, eps)


# the fused token embedding + first RMSNorm (NBD_EMBED_RMS=0: the two ops, A/B)
_EMBED_RMS = os.environ.get("NBD_EMBED_RMS", "1") != "0"


def embed_rms_norm(ids, table, weight, eps: float = 1e-6):
    """``x = F.embedding(ids, table); return x, rms_norm(x, weight)`` — a Llama model's input: one
    HIP pass forward (the gathered rows stored as the residual stream beside their norm) and, in
    backward, one norm pass that also adds the residual stream's gradient, then the table's
    gradient straight into its DDP bucket slice (``csrc/kernels/autograd.hip`` EmbedRMSFn).
    Same bits as the two separate ops."""
    import torch

    from .embedding import _poll_ids, embedding

    C = table.shape[-1]
    if (_EMBED_RMS and table.is_cuda and _native() and ids.dtype == torch.int64 and table.dim() == 2
            and table.dtype == weight.dtype and table.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and C % 4 == 0 and C <= 2048 and table.is_contiguous() and not torch.is_autocast_enabled()):
        _require()
        return torch.ops.nbd.embed_rms_norm_ag(ids if ids.is_contiguous() else ids.contiguous(), table, weight,
                                               float(eps), _poll_ids(table.device))
    x = embedding(ids, table)
    return x, rms_norm(x, weight, eps)


def tokpos_layer_norm(idx, wte, pos, wpe, vocab: int, weight, bias, eps: float = 1e-5):
    """``x = embedding_tok_pos(idx, wte, pos, wpe, vocab); return x, layer_norm(x, weight, bias)`` —
    GPT-2's input and its first LayerNorm in one HIP pass, their backward in one norm pass (the
    residual stream's gradient added there) plus the two tables' gradients, each into its DDP
    bucket slice (``csrc/kernels/autograd.hip`` TokPosLNFn).  Same bits forward as the two ops.
    ``NBD_EMBED_RMS=0`` also turns this fusion off (A/B)."""
    import torch

    from .embedding import FUSED_EMBED, _poll_ids, embedding_tok_pos

    C = wte.shape[-1]
    if (_EMBED_RMS and FUSED_EMBED and wte.is_cuda and _native() and idx.dtype == torch.int64
            and pos.dtype == torch.int64 and pos.dim() == 1 and idx.shape[-1] == pos.numel() and wte.dim() == 2
            and wte.dtype == wpe.dtype == weight.dtype == bias.dtype and wte.dtype in (torch.bfloat16, torch.float16)
            and C % 8 == 0 and C <= 2048 and wte.is_contiguous() and wpe.is_contiguous()
            and not torch.is_autocast_enabled()):
        _require()
        return torch.ops.nbd.tokpos_layer_norm_ag(idx.contiguous(), wte, pos.contiguous(), wpe, weight, bias,
                                                  int(vocab), float(eps), _poll_ids(wte.device))
    x = embedding_tok_pos(idx, wte, pos, wpe, vocab)
    return x, layer_norm(x, weight, bias, eps)

