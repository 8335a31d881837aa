"""Gradient destinations (``csrc/kernels/graddst.{h,cpp}``): DDP registers, per parameter, the
bucket slice that is its gradient's home; backward nodes write their weight-gradient GEMM straight
into it (accumulating in the GEMM epilogue when ``.grad`` already is that slice), so the bucket
needs no flatten copy before its all-reduce and gradient accumulation needs no separate adds.

The C++ autograd nodes (``autograd.hip``) use the registry directly; these helpers serve the
Python ``autograd.Function``s on the hot path (the LM head in ``ops/loss.py``, the token
embedding in ``ops/embedding.py``)."""
from __future__ import annotations

from typing import Optional, Tuple

from ._lib import _require


def register(param, dst) -> None:
    """Make ``dst`` (contiguous, ``param``'s shape / dtype / device) the home of ``param``'s
    gradient; ``dst=None`` removes the registration."""
    import torch

    _require()
    torch.ops.nbd.set_grad_dest(param, dst)


def new_pass() -> None:
    """Start a backward pass: each destination may be handed out once per pass."""
    import torch

    torch.ops.nbd.grad_dest_new_pass()


def count() -> int:
    import torch

    return int(torch.ops.nbd.grad_dest_count())


def claim(param) -> Tuple[Optional["torch.Tensor"], bool]:  # noqa: F821
    """(destination, accumulate) for a gradient of ``param`` about to be computed, or (None,
    False): allocate as usual."""
    import torch

    if not param.is_cuda:
        return None, False
    d, acc = torch.ops.nbd.grad_dest_claim(param)
    return (d, bool(acc)) if d.numel() else (None, False)


def hand_back(param, dst, acc: bool):
    """The tensor a backward returns for a gradient written into ``dst`` (claimed with ``acc``):
    a fresh view that AccumulateGrad installs as ``.grad`` without a copy."""
    if acc:
        param.grad = None  # AccumulateGrad steals only while .grad is unset; dst holds the sum
    return dst.view(dst.shape)


def defer_enable(on: bool) -> None:
    """Queue the split-K reduces of weight gradients written into their slices (graddst.h
    ``defer``) instead of launching one per Linear; ``defer_flush`` issues them in one launch."""
    import torch

    _require()
    torch.ops.nbd.grad_defer_enable(bool(on))


def defer_flush() -> None:
    """Issue every queued weight-gradient reduce (one launch, on the stream they were queued on)."""
    import torch

    torch.ops.nbd.grad_defer_flush()


def defer_pending() -> int:
    import torch

    return int(torch.ops.nbd.grad_defer_pending())


def join(param):
    """The destination if another node already wrote ``param``'s gradient there in this pass
    (it is still on its way to AccumulateGrad): add into it and return no gradient."""
    import torch

    if not param.is_cuda:
        return None
    d = torch.ops.nbd.grad_dest_join(param)
    return d if d.numel() else None
