"""Sequence parallelism: Ulysses all-to-all attention over an SP group.

The reference has no long-context support ("Any SP/CP would be user code calling
``dist.all_to_all`` … inside cells").  Here it is a library call.  Every rank holds a contiguous
chunk of the sequence (``T / n`` tokens) for all heads; one all-to-all turns that into the full
sequence for ``H / n`` heads, the HIP flash-attention kernels run on it unchanged (causal masking
stays exact because every head now sees the whole sequence), and a second all-to-all turns the
output back into sequence chunks.  Backward is the same two all-to-alls in reverse.

On MI355X the all-to-all is the right collective for this: each rank sends ``(n-1)/n`` of its
q/k/v/o slices once, directly over the point-to-point xGMI link to each peer (no ring hops), and
the per-rank activations of a long sequence fit the 288 GB HBM without recomputation.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _size(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def _seq_to_head(x, group):
    """[B, H, T/n, D] (sequence chunk, all heads) → [B, H/n, T, D] (full sequence, own heads)."""
    n = _size(group)
    if n == 1:
        return x
    B, H, Tl, D = x.shape
    if H % n:
        raise ValueError(f"{H} heads are not divisible by the sequence-parallel size {n}")
    inp = x.reshape(B, n, H // n, Tl, D).movedim(1, 0).contiguous()
    out = torch.empty_like(inp)
    dist.all_to_all_single(out, inp, group=group)
    return out.permute(1, 2, 0, 3, 4).reshape(B, H // n, n * Tl, D)


def _head_to_seq(x, group):
    """[B, H/n, T, D] → [B, H, T/n, D] (inverse of :func:`_seq_to_head`)."""
    n = _size(group)
    if n == 1:
        return x
    B, Hl, T, D = x.shape
    inp = x.reshape(B, Hl, n, T // n, D).permute(2, 0, 1, 3, 4).contiguous()
    out = torch.empty_like(inp)
    dist.all_to_all_single(out, inp, group=group)
    return out.movedim(0, 1).reshape(B, n * Hl, T // n, D)


class _SeqToHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _seq_to_head(x, group)

    @staticmethod
    def backward(ctx, g):
        return _head_to_seq(g, ctx.group), None


class _HeadToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _head_to_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return _seq_to_head(g, ctx.group), None


def seq_to_head(x, group=None):
    """Autograd-aware all-to-all: sequence-sharded [B, H, T/n, D] → head-sharded [B, H/n, T, D]."""
    return _SeqToHead.apply(x, group)


def head_to_seq(x, group=None):
    """Autograd-aware all-to-all: head-sharded [B, H/n, T, D] → sequence-sharded [B, H, T/n, D]."""
    return _HeadToSeq.apply(x, group)


def ulysses_attention(q, k, v, causal: bool = True, scale=None, group=None):
    """Attention over a sequence split across ``group``: q [B, H, T/n, D], k/v [B, Hkv, T/n, D]
    (rank r holds tokens ``[r·T/n, (r+1)·T/n)``) → this rank's [B, H, T/n, D] output chunk.
    The inner attention is ``ops.flash_attention`` (HIP kernels where supported, SDPA otherwise)."""
    from .. import ops

    qh, kh, vh = seq_to_head(q, group), seq_to_head(k, group), seq_to_head(v, group)
    return head_to_seq(ops.flash_attention(qh, kh, vh, causal=causal, scale=scale), group)


def shard_sequence(x, group=None, dim: int = 1):
    """This rank's contiguous chunk of ``x`` along ``dim`` (no autograd communication)."""
    n = _size(group)
    if x.shape[dim] % n:
        raise ValueError(f"length {x.shape[dim]} is not divisible by the sequence-parallel size {n}")
    return x.chunk(n, dim=dim)[_rank(group)]


def gather_sequence(x, group=None, dim: int = 1):
    """All-gather the sequence chunks of every rank along ``dim`` (forward only)."""
    n = _size(group)
    if n == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(n)]
    dist.all_gather(parts, x.contiguous(), group=group)
    return torch.cat(parts, dim=dim)


__all__ = ["seq_to_head", "head_to_seq", "ulysses_attention", "shard_sequence", "gather_sequence"]
