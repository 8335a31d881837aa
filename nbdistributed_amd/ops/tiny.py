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
