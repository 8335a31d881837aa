"""Fused large-vocabulary softmax cross-entropy (K6)."""
from __future__ import annotations

from ._lib import _require


_XentFn = None

def _xent_fn():
    global _XentFn
    if _XentFn is not None:
        return _XentFn
    import torch

    class _FusedCrossEntropy(torch.autograd.Function):
        @staticmethod
        def forward(ctx, logits, target, ignore_index, reduction, inplace_backward):
            loss_rows, lse = torch.ops.nbd.xent_fwd(logits, target, ignore_index)
            if reduction == "mean":
                denom = (target != ignore_index).sum()
                loss = loss_rows.sum() / denom  # 0/0 = nan when every row is ignored, as torch
            else:
                denom = torch.ones((), dtype=torch.int64, device=logits.device)
                loss = loss_rows.sum()
            ctx.save_for_backward(logits, target, lse, denom)
            ctx.ignore_index = ignore_index
            ctx.inplace = inplace_backward
            return loss

        @staticmethod
        def backward(ctx, grad):
            logits, target, lse, denom = ctx.saved_tensors
            scale = (grad.float() / denom).reshape(1)
            dlogits = logits if ctx.inplace else torch.empty_like(logits)
            torch.ops.nbd.xent_bwd(logits, target, lse, scale, ctx.ignore_index, dlogits)
            return dlogits, None, None, None, None

    _XentFn = _FusedCrossEntropy
    return _XentFn

def cross_entropy(logits, target, ignore_index: int = -100, reduction: str = "mean", inplace_backward: bool = False):
    """Softmax cross-entropy of ``logits`` [N, V] (any float dtype) against int64 ``target`` [N]
    — ``F.cross_entropy(logits.float(), target)`` semantics (mean over non-ignored rows, or sum)
    without materialising fp32 logits: one fused HIP pass forward (per-row logsumexp), one pass
    backward writing dlogits in the logits' dtype (``csrc/kernels/xent.hip``).
    ``inplace_backward=True`` writes the gradient over the logits storage (use when nothing reads
    the logits after the loss — saves a [N, V] allocation)."""
    import torch
    import torch.nn.functional as F

    if reduction not in ("mean", "sum"):
        raise ValueError("cross_entropy: reduction must be 'mean' or 'sum'")
    if not logits.is_cuda:
        return F.cross_entropy(logits.float(), target, ignore_index=ignore_index, reduction=reduction)
    _require()
    if logits.stride(-1) != 1:
        logits = logits.contiguous()
    return _xent_fn().apply(logits, target.contiguous().long(), int(ignore_index), reduction, bool(inplace_backward))
