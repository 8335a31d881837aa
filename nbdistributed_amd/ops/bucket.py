"""Gradient-bucket kernels (K1-K3): flatten/unflatten with fused cast + scale, local pre-reduce.

CPU tensors use the PyTorch reference implementations (the GPU numerics tests' oracle)."""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from ._lib import _require


def plan_offsets(numels: Sequence[int], align: int = 64) -> Tuple[List[int], int]:
    """Bucket layout: each tensor starts at a multiple of ``align`` elements (128 B for bf16,
    256 B for fp32) so every tensor takes the kernels' 16-B vector path.  Returns (offsets,
    total numel)."""
    offs = []
    pos = 0
    for n in numels:
        offs.append(pos)
        pos += (int(n) + align - 1) // align * align
    return offs, pos


# ---------------------------------------------------------------- reference implementations

def _ref_flatten(tensors, bucket, offsets, scale, accumulate=False):
    for t, o in zip(tensors, offsets):
        n = t.numel()
        v = t.reshape(-1).float() * scale
        if accumulate:
            v = v + bucket[o:o + n].float()
        bucket[o:o + n].copy_(v.to(bucket.dtype))

def _ref_unflatten(bucket, tensors, offsets, scale, accumulate):
    for t, o in zip(tensors, offsets):
        n = t.numel()
        v = bucket[o:o + n].float() * scale
        if accumulate:
            v = v + t.reshape(-1).float()
        t.view(-1).copy_(v.to(t.dtype))

def _ref_prereduce(inputs, out, scale):
    acc = inputs[0].reshape(-1).float().clone()
    for x in inputs[1:]:
        acc += x.reshape(-1).float()
    out.view(-1).copy_((acc * scale).to(out.dtype))

def bucket_flatten(tensors: Sequence, bucket=None, offsets: Optional[Sequence[int]] = None, dtype=None,
                   scale: float = 1.0, align: int = 64, accumulate: bool = False):
    """Copy ``tensors`` into one flat ``bucket`` (allocated if None), casting to the bucket's dtype
    and multiplying by ``scale``; ``accumulate``: add into the bucket's contents instead (fp32 math,
    one rounding — the local pre-reduce of micro-batch gradients).  Returns (bucket, offsets)."""
    import torch

    tensors = list(tensors)
    if offsets is None:
        offsets, total = plan_offsets([t.numel() for t in tensors], align)
    elif bucket is None:  # (the no_sync pre-reduce passes both: no per-tensor Python loop on its path)
        total = max((o + t.numel() for o, t in zip(offsets, tensors)), default=0)
    if bucket is None:
        dev = tensors[0].device if tensors else "cpu"
        bucket = torch.zeros(total, dtype=dtype or (tensors[0].dtype if tensors else torch.float32), device=dev)
    if not tensors:
        return bucket, list(offsets)
    flat = [t if t.is_contiguous() else t.contiguous() for t in tensors]
    if bucket.is_cuda:
        _require()
        torch.ops.nbd.bucket_flatten(flat, bucket, list(offsets), float(scale), bool(accumulate))
    else:
        _ref_flatten(flat, bucket, offsets, scale, accumulate)
    return bucket, list(offsets)

def bucket_unflatten(bucket, tensors: Sequence, offsets: Sequence[int], scale: float = 1.0,
                     accumulate: bool = False) -> None:
    """Scatter ``bucket`` back into ``tensors`` (in place), times ``scale``, cast to each
    tensor's dtype, optionally accumulating (``t += scale * bucket[...]``)."""
    import torch

    tensors = list(tensors)
    if not tensors:
        return
    for t in tensors:
        if not t.is_contiguous():
            raise ValueError("bucket_unflatten targets must be contiguous")
    if bucket.is_cuda:
        _require()
        torch.ops.nbd.bucket_unflatten(bucket, tensors, list(offsets), float(scale), bool(accumulate))
    else:
        _ref_unflatten(bucket, tensors, offsets, scale, accumulate)

def prereduce_into_bucket(tensors: Sequence, bucket, offsets: Sequence[int], scale: float = 1.0) -> None:
    """K3 in its multi-tensor form: ``bucket[slice_i] += scale * tensors[i]`` for every i, fp32
    accumulation, one launch per <= 256 tensors.  DDP's ``no_sync`` path sums each micro-batch's
    gradients into their bucket with it (``parallel/ddp.py``), so the last micro-batch's bucket is
    the locally pre-reduced gradient and no per-parameter autograd adds run."""
    bucket_flatten(tensors, bucket, offsets, scale=scale, accumulate=True)


def local_prereduce(inputs: Sequence, out=None, scale: float = 1.0, dtype=None):
    """``out = scale * Σ inputs`` with fp32 accumulation.  Returns ``out``."""
    import torch

    inputs = [x if x.is_contiguous() else x.contiguous() for x in inputs]
    if not inputs:
        raise ValueError("local_prereduce needs at least one input")
    if out is None:
        out = torch.empty_like(inputs[0], dtype=dtype or inputs[0].dtype)
    if out.is_cuda:
        _require()
        if len(inputs) > 16:
            partials = []
            for i in range(0, len(inputs), 16):
                p = torch.empty(out.shape, dtype=torch.float32, device=out.device)
                torch.ops.nbd.local_prereduce(inputs[i:i + 16], p, 1.0)
                partials.append(p)
            return local_prereduce(partials, out, scale)
        torch.ops.nbd.local_prereduce(inputs, out, float(scale))
    else:
        _ref_prereduce(inputs, out, scale)
    return out
