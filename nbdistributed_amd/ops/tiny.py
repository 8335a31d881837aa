"""Linear layers with a tiny output dimension on the GPU: ``csrc/kernels/tiny.hip``.

A classifier head (SmolLM2's ``score``: 576 -> 2 labels on 16 pooled rows,
``/root/reference/00_accelerate.ipynb`` exec 22 builds it through
``AutoModelForSequenceClassification``) is a handful of dot products.  Tiled GEMMs pad it to a
64-wide tile (the hand-written ones need 64-granular shapes; hipBLASLt ran three ``Cijk``
launches per notebook step for it); here the forward is one launch (a wave per output) and the
backward one launch (dx, dW and db together).  bf16 in, fp32 accumulation in a fixed order,
bf16 out.  Anything else (CPU, other dtypes, N > 64) goes through ``F.linear``.
"""
from __future__ import annotations

import os

from ._lib import _require

# NBD_LINEAR_TINY=0: the library path (F.linear) for A/B measurements
ENABLED = os.environ.get("NBD_LINEAR_TINY", "1") != "0"
MAX_N = 64
MAX_M = 4096  # dW loops over the rows in one thread per (n, 8 k): fine for heads, not for token-wide M


def shape_ok(x, n: int, k: int) -> bool:
    """x [..., k] bf16 on the GPU times a [n, k] bf16 weight fits the kernels."""
    import torch

    return bool(ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and 1 <= n <= MAX_N and x.shape[-1] == k
                and k % 8 == 0 and x.numel() // max(1, k) <= MAX_M)


def supported(x, weight, bias=None) -> bool:
    import torch

    return bool(weight.dim() == 2 and weight.dtype == torch.bfloat16 and shape_ok(x, weight.shape[0], weight.shape[1])
                and (bias is None or (bias.dtype == torch.bfloat16 and bias.numel() == weight.shape[0])))


_Fn = None


def _fn():
    global _Fn
    if _Fn is not None:
        return _Fn
    import torch

    def _c(t):
        return t if t.is_contiguous() and t.data_ptr() % 16 == 0 else t.contiguous()

    class _LinearTiny(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, b):
            x2 = _c(x.reshape(-1, x.shape[-1]))
            w2 = _c(w)
            ctx.save_for_backward(x2, w2)
            ctx.xshape = x.shape
            ctx.has_b = b is not None
            y = torch.ops.nbd.linear_tiny(x2, w2, b.contiguous() if b is not None else None)
            return y.view(*x.shape[:-1], w.shape[0])

        @staticmethod
        def backward(ctx, dy):
            x2, w2 = ctx.saved_tensors
            dy2 = _c(dy.reshape(-1, dy.shape[-1]).to(torch.bfloat16))
            nx, nw, nb = ctx.needs_input_grad
            dx, dw, db = torch.ops.nbd.linear_tiny_bwd(dy2, x2, w2, bool(nx), bool(nw), bool(nb and ctx.has_b))
            return (dx.view(ctx.xshape) if nx else None, dw if nw else None, db if nb and ctx.has_b else None)

    _Fn = _LinearTiny
    return _Fn


def linear_tiny(x, weight, bias=None):
    """``F.linear(x, weight, bias)`` for ``weight`` [N <= 64, K] on the HIP tiny-linear kernels
    (bf16 GPU tensors, K % 8 == 0, at most 4096 rows); ``F.linear`` otherwise."""
    if supported(x, weight, bias):
        _require()
        return _fn().apply(x, weight, bias)
    import torch.nn.functional as F

    return F.linear(x, weight, bias)


# ---- the sequence-classification tail, fused (pooled row -> score -> mean cross-entropy) ------
_SeqFn = None
MAX_ROWS = 64


def seqcls_ok(h, weight, labels) -> bool:
    """h [B, T, C] bf16 (GPU, contiguous), ``weight`` [N, C] bf16, integer ``labels`` [B]: fits
    ``nbd::seqcls_head`` (B <= 64, N <= 64, B·N <= 1024, C % 8 == 0)."""
    import torch

    return bool(ENABLED and h.is_cuda and h.dim() == 3 and h.dtype == torch.bfloat16 and weight.dim() == 2
                and weight.dtype == torch.bfloat16 and weight.shape[1] == h.shape[2] and h.shape[2] % 8 == 0
                and 1 <= h.shape[0] <= MAX_ROWS and 1 <= weight.shape[0] <= MAX_N
                and h.shape[0] * weight.shape[0] <= 1024 and labels is not None
                and labels.dtype in (torch.int64, torch.int32) and labels.numel() == h.shape[0])


def _seq_fn():
    global _SeqFn
    if _SeqFn is not None:
        return _SeqFn
    import torch

    class _SeqClsHead(torch.autograd.Function):
        @staticmethod
        def forward(ctx, h, last, w, labels, ignore_index):
            h = h if h.is_contiguous() and h.data_ptr() % 16 == 0 else h.contiguous()
            w2 = w if w.is_contiguous() and w.data_ptr() % 16 == 0 else w.contiguous()
            loss, logits, dl = torch.ops.nbd.seqcls_head(h, last, w2, labels, int(ignore_index))
            ctx.save_for_backward(h, last, w2, dl)
            ctx.set_materialize_grads(False)  # an unused output's gradient arrives as None, not a zero fill
            ctx.param = w if isinstance(w, torch.nn.Parameter) else None
            return loss, logits

        @staticmethod
        def backward(ctx, g_loss, g_logits):
            from . import graddst

            h, last, w2, dl = ctx.saved_tensors
            need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[2]
            if not (need_h or need_w):
                return None, None, None, None, None
            g = (g_loss.float().reshape(1) if g_loss is not None
                 else torch.zeros(1, dtype=torch.float32, device=h.device))
            glog = g_logits.to(torch.bfloat16).contiguous() if g_logits is not None else None
            dst, acc = graddst.claim(ctx.param) if need_w and ctx.param is not None else (None, False)
            if dst is not None and (dst.dtype != torch.bfloat16 or dst.shape != w2.shape or not dst.is_contiguous()):
                raise RuntimeError("seqcls_head: unexpected DDP gradient slice for the score weight")
            dh, dw = torch.ops.nbd.seqcls_head_bwd(h, last, w2, dl, g, glog, dst, acc)
            if dst is not None:
                dw = graddst.hand_back(ctx.param, dst, acc)
            return (dh if need_h else None), None, (dw if need_w else None), None, None

    _SeqFn = _SeqClsHead
    return _SeqFn


def seqcls_head_loss(h, last, weight, labels, ignore_index: int = -100):
    """(loss, logits) of a sequence classifier's tail — ``pooled = h[b, last[b]]``, ``logits =
    pooled·weightᵀ`` (bf16, as ``F.linear``), ``loss = F.cross_entropy(logits.float(), labels)``
    (mean over rows whose label is not ``ignore_index``) — in one HIP launch forward and one
    backward (``csrc/kernels/tiny.hip`` seqcls); the caller checks ``seqcls_ok`` first."""
    _require()
    return _seq_fn().apply(h, last.reshape(-1).long().contiguous(), weight, labels.reshape(-1).long().contiguous(),
                           int(ignore_index))
