"""Context parallelism: ring attention over a CP group.

The reference has no long-context support (SP/CP "would be user code calling
``dist.all_to_all`` … inside cells").  ``parallel.sequence`` covers Ulysses (all-to-all, needs
``H % n == 0``); this module is the other standard scheme, for sequences whose activations do not
fit one GPU even after head sharding or whose head count is smaller than the group:

* every rank keeps its own query chunk(s); key/value chunks travel round the ring (one
  ``batch_isend_irecv`` per step, posted *before* the step's attention so the xGMI transfer of
  the next K/V block overlaps the HIP flash-attention kernels on the current one);
* each block is one call of the gfx950 flash kernels (``nbd::attn_fwd``), which return the
  block's log-sum-exp; blocks are merged exactly with the usual LSE rescaling (fp32 accumulator);
* backward replays the ring: ``nbd::attn_bwd`` is given the *merged* output and LSE, so each
  block's dQ/dK/dV is the exact slice of the full gradient; dQ accumulates locally and dK/dV
  accumulators travel with their K/V block (their transfer overlaps the next step's attention
  backward) and take one extra hop home at the end.

Causal load balance: with the contiguous layout rank r only needs kv chunks ≤ r (rank n-1 does n
blocks, rank 0 one).  ``layout="zigzag"`` splits the sequence into 2n chunks and gives rank r chunks
r and 2n-1-r, so every rank does the same number of (sub-)blocks at every step.

A ring (not one all-gather) is the right shape on MI355X: each step moves one K/V chunk over a
single point-to-point xGMI link, peak extra HBM is two K/V chunks instead of the whole sequence,
and the transfer hides behind attention compute once chunks are ≥ a few thousand tokens.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from .p2p import batch_isend_irecv
from .sequence import _rank, _size


def _global(group, r: int) -> int:
    return dist.get_global_rank(group, r) if group is not None else r


def _chunk_ids(r: int, n: int, layout: str) -> List[int]:
    if layout == "contiguous":
        return [r]
    if layout == "zigzag":
        return [r, 2 * n - 1 - r]
    raise ValueError(f"unknown context-parallel layout {layout!r} (contiguous | zigzag)")


def shard_context(x, group=None, dim: int = 2, layout: str = "contiguous"):
    """This rank's part of ``x`` along ``dim`` for ``layout`` (contiguous: chunk r of n; zigzag:
    chunks r and 2n-1-r of 2n, concatenated)."""
    n, r = _size(group), _rank(group)
    parts = 1 if layout == "contiguous" else 2
    if x.shape[dim] % (n * parts):
        raise ValueError(f"length {x.shape[dim]} is not divisible into {n * parts} context chunks")
    chunks = x.chunk(n * parts, dim=dim)
    return torch.cat([chunks[c] for c in _chunk_ids(r, n, layout)], dim=dim)


def gather_context(x, group=None, dim: int = 2, layout: str = "contiguous"):
    """Inverse of :func:`shard_context`: the full sequence on every rank (forward only)."""
    n = _size(group)
    if n == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(n)]
    dist.all_gather(parts, x.contiguous(), group=group)
    if layout == "contiguous":
        return torch.cat(parts, dim=dim)
    chunks = [None] * (2 * n)
    for r, p in enumerate(parts):
        a, b = p.chunk(2, dim=dim)
        chunks[r], chunks[2 * n - 1 - r] = a, b
    return torch.cat(chunks, dim=dim)


# ---------------------------------------------------------------------------------------------
# one attention block: HIP flash kernels where they apply, an fp32 reference otherwise
# ---------------------------------------------------------------------------------------------

def _hip_ok(q, k) -> bool:
    from ..ops.attention import flash_supported

    return (flash_supported(q) and k.shape[2] == q.shape[2] and k.dtype == q.dtype
            and q.shape[1] % k.shape[1] == 0)


def _fix(t):
    """``t`` itself when the HIP attention kernels can read it as a strided view, else a copy."""
    ok = t.stride(-1) == 1 and all(st % 8 == 0 for st in t.stride()[:-1]) and t.data_ptr() % 16 == 0
    return t if ok else t.contiguous()


def _rep(x, g: int):
    return x if g == 1 else x.repeat_interleave(g, dim=1)


def _blk_fwd(q, k, v, causal: bool, scale: float):
    """(o [B, H, Tq, D], lse [B, H, Tq] fp32) of softmax(q·kᵀ·scale)·v; o is bf16 from the HIP
    kernels, fp32 from the reference path."""
    if _hip_ok(q, k):
        from ..ops._lib import _require

        _require()
        return torch.ops.nbd.attn_fwd(_fix(q), _fix(k), _fix(v), causal, scale, None, None)
    g = q.shape[1] // k.shape[1]
    s = torch.matmul(q.float(), _rep(k, g).float().transpose(-1, -2)) * scale
    if causal:
        Tq, Tk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Tq, Tk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    return torch.matmul(torch.exp(s - lse.unsqueeze(-1)), _rep(v, g).float()), lse


def _blk_bwd(do, q, k, v, o, lse, causal: bool, scale: float):
    """This block's (dq, dk, dv) given the merged output ``o`` and merged ``lse`` of the rows."""
    if _hip_ok(q, k):
        B, H, T, D = q.shape
        Hkv = k.shape[1]
        dq = torch.empty(B, T, H, D, dtype=q.dtype, device=q.device).transpose(1, 2)
        dkv = torch.empty(B, T, 2, Hkv, D, dtype=q.dtype, device=q.device)
        dk, dv = dkv[:, :, 0].transpose(1, 2), dkv[:, :, 1].transpose(1, 2)
        torch.ops.nbd.attn_bwd(_fix(do), _fix(q), _fix(k), _fix(v), _fix(o), lse, causal, scale, dq, dk, dv,
                               None, None)
        return dq, dk, dv
    g = q.shape[1] // k.shape[1]
    qf, kf, vf, dof = q.float(), _rep(k, g).float(), _rep(v, g).float(), do.float()
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        Tq, Tk = s.shape[-2:]
        s = s.masked_fill(torch.ones(Tq, Tk, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    p = torch.exp(s - lse.unsqueeze(-1))
    dv = torch.matmul(p.transpose(-1, -2), dof)
    dp = torch.matmul(dof, vf.transpose(-1, -2))
    delta = (dof * o.float()).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = torch.matmul(ds, kf)
    dk = torch.matmul(ds.transpose(-1, -2), qf)
    if g > 1:
        B, H, Tk, D = dk.shape
        dk = dk.view(B, H // g, g, Tk, D).sum(2)
        dv = dv.view(B, H // g, g, Tk, D).sum(2)
    return dq, dk, dv


def _merge(o_acc, lse_acc, o_b, l_b, out=None):
    """Fold block (o_b, l_b) into the running (o_acc fp32, lse_acc) in place; with ``out`` (the
    rows' last block) the merged rows go to ``out`` instead of ``o_acc``.  One HIP pass
    (``nbd::attn_merge_``, csrc/kernels/ring.hip) for bf16 blocks, PyTorch otherwise."""
    if o_b.is_cuda and o_b.dtype == torch.bfloat16 and o_b.shape[-1] == 64:
        torch.ops.nbd.attn_merge_(o_acc, lse_acc, _fix(o_b), l_b, out)
        return
    l_new = torch.logaddexp(lse_acc, l_b)
    merged = (o_acc * torch.exp(lse_acc - l_new).unsqueeze(-1) + o_b.float() * torch.exp(l_b - l_new).unsqueeze(-1))
    lse_acc.copy_(l_new)
    (out if out is not None else o_acc).copy_(merged)


# ---------------------------------------------------------------------------------------------
# ring plumbing
# ---------------------------------------------------------------------------------------------

class _Ring:
    """Send to rank r+1 / receive from rank r-1 of ``group``, both posted in one batch.  Gloo has
    no device-memory point-to-point path, so CUDA tensors are staged through host memory there."""

    def __init__(self, group):
        self.group = group
        self.n, self.r = _size(group), _rank(group)
        self.nxt = _global(group, (self.r + 1) % self.n)
        self.prv = _global(group, (self.r - 1) % self.n)
        self.stage = dist.is_initialized() and dist.get_backend(group) == "gloo"

    def start(self, *send: torch.Tensor):
        """Post the exchange of every tensor in ``send``; returns a handle for :meth:`finish`."""
        dev = send[0].device
        if self.stage and dev.type != "cpu":
            send = tuple(t.cpu() for t in send)
        recv = tuple(torch.empty_like(t) for t in send)
        ops = []
        for a, b in zip(send, recv):
            ops += [dist.P2POp(dist.isend, a, self.nxt, self.group), dist.P2POp(dist.irecv, b, self.prv, self.group)]
        return batch_isend_irecv(ops), recv, dev, send

    @staticmethod
    def finish(handle):
        """The received tensors (a tuple, in the order sent), on the sender's device."""
        reqs, recv, dev, _send = handle
        for w in reqs:
            w.wait()
        return tuple(t.to(dev, non_blocking=True) if t.device != dev else t for t in recv)


def _blocks(r_q: int, r_kv: int, n: int, layout: str):
    """(q sub-chunk, kv sub-chunk, causal) triples rank ``r_q`` computes against rank ``r_kv``'s
    K/V for a causal mask (sub-chunks index into the rank's local concatenation)."""
    out = []
    for iq, cq in enumerate(_chunk_ids(r_q, n, layout)):
        for ik, ck in enumerate(_chunk_ids(r_kv, n, layout)):
            if ck < cq:
                out.append((iq, ik, False))
            elif ck == cq:
                out.append((iq, ik, True))
    return out


class _RingAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, group, layout):
        ring = _Ring(group)
        n, r = ring.n, ring.r
        parts = 1 if layout == "contiguous" else 2
        qs = q.chunk(parts, dim=2)
        sched = [(_blocks(r, (r - s) % n, n, layout) if causal
                  else [(iq, ik, False) for iq in range(parts) for ik in range(parts)]) for s in range(n)]
        left = [sum(b[0] == iq for step in sched for b in step) for iq in range(parts)]
        out = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        outs = out.chunk(parts, dim=2)
        o_acc, lse_acc = [None] * parts, [None] * parts
        kc, vc = (k.contiguous(), v.contiguous()) if n > 1 else (k, v)  # only sent tensors need packing
        for s in range(n):
            h = ring.start(kc, vc) if s < n - 1 else None
            ks, vs = kc.chunk(parts, dim=2), vc.chunk(parts, dim=2)
            for iq, ik, diag in sched[s]:
                o_b, l_b = _blk_fwd(qs[iq], ks[ik], vs[ik], diag, scale)
                left[iq] -= 1
                if lse_acc[iq] is None:
                    lse_acc[iq] = l_b.contiguous()
                    if left[iq] == 0:
                        outs[iq].copy_(o_b)
                    else:
                        o_acc[iq] = o_b.to(torch.float32, memory_format=torch.contiguous_format)
                else:
                    _merge(o_acc[iq], lse_acc[iq], o_b, l_b, outs[iq] if left[iq] == 0 else None)
            if h is not None:
                kc, vc = ring.finish(h)
        ctx.save_for_backward(q, k, v, out, *lse_acc)
        ctx.causal, ctx.scale, ctx.group, ctx.layout = causal, scale, group, layout
        return out

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, *ls = ctx.saved_tensors
        causal, scale, layout = ctx.causal, ctx.scale, ctx.layout
        ring = _Ring(ctx.group)
        n, r = ring.n, ring.r
        parts = 1 if layout == "contiguous" else 2
        do = do.contiguous()
        qs, os_, dos = (t.chunk(parts, dim=2) for t in (q, o, do))
        dq = [None] * parts
        kc, vc = (k.contiguous(), v.contiguous()) if n > 1 else (k, v)  # only sent tensors need packing
        dk = torch.zeros(k.shape, dtype=torch.float32, device=q.device)
        dv = torch.zeros(v.shape, dtype=torch.float32, device=q.device)
        pending = None  # the dK/dV accumulators in flight from the previous step
        for s in range(n):
            h = ring.start(kc, vc) if s < n - 1 else None
            src = (r - s) % n
            ks, vs = kc.chunk(parts, dim=2), vc.chunk(parts, dim=2)
            blocks = (_blocks(r, src, n, layout) if causal
                      else [(iq, ik, False) for iq in range(parts) for ik in range(parts)])
            contrib = []
            for iq, ik, diag in blocks:
                dq_b, dk_b, dv_b = _blk_bwd(dos[iq], qs[iq], ks[ik], vs[ik], os_[iq], ls[iq], diag, scale)
                if dq[iq] is None:
                    dq[iq] = dq_b.to(torch.float32, memory_format=torch.contiguous_format)
                else:
                    dq[iq].add_(dq_b)
                contrib.append((ik, dk_b, dv_b))
            # the accumulators of this step's K/V block arrive while its attention backward ran
            if pending is not None:
                dk, dv = ring.finish(pending)
            dks, dvs = dk.chunk(parts, dim=2), dv.chunk(parts, dim=2)
            for ik, dk_b, dv_b in contrib:
                dks[ik].add_(dk_b)
                dvs[ik].add_(dv_b)
            # ... and follow it to the next rank (after the last step: one extra hop home)
            if n > 1:
                pending = ring.start(dk, dv)
            if h is not None:
                kc, vc = ring.finish(h)
        if pending is not None:
            dk, dv = ring.finish(pending)
        dq = torch.cat(dq, dim=2).to(q.dtype)
        return dq, dk.to(k.dtype), dv.to(v.dtype), None, None, None, None


def ring_attention(q, k, v, causal: bool = True, scale: Optional[float] = None, group=None,
                   layout: str = "contiguous"):
    """Attention over a sequence split across ``group`` by :func:`shard_context`: q [B, H, Tl, D],
    k/v [B, Hkv, Tl, D] (``Hkv`` divides ``H``: grouped-query) → this rank's [B, H, Tl, D] output.
    Exact (same result as attention on the gathered sequence); HIP flash kernels per block for bf16,
    head dim 64 and chunks of a multiple of 128 tokens, an fp32 reference otherwise."""
    sc = float(scale) if scale is not None else q.shape[-1] ** -0.5
    if _size(group) == 1 and layout == "contiguous":
        from .. import ops

        return ops.flash_attention(q, k, v, causal=causal, scale=sc)
    return _RingAttention.apply(q, k, v, bool(causal), sc, group, layout)


def shift_labels(labels, ignore_index: int = -100):
    """Next-token targets aligned with the input positions (``out[:, t] = labels[:, t + 1]``, the
    last position ``ignore_index``).  A causal-LM loss under context parallelism must take its
    targets in this form, shifted on the *full* sequence before :func:`shard_context`: shifting
    inside a shard would pair the last token of a chunk with the first token of whatever chunk
    the layout puts next (zigzag: chunk 2n-1-r), and drop every chunk boundary's real target."""
    out = torch.full_like(labels, ignore_index)
    out[:, :-1] = labels[:, 1:]
    return out


def context_loss(loss_sum, n_valid, group=None):
    """This rank's share of the group-wide token mean: ``loss_sum · n / Σ_group n_valid``.

    ``loss_sum`` is the sum of this rank's per-token losses and ``n_valid`` its count of counted
    (non-``ignore_index``) targets.  Averaging the returned values — and their gradients, as DDP
    over a group containing the CP group does — over the group gives the mean over every counted
    token of the full sequences, however the ignored targets are spread over the shards (a plain
    average of per-shard means is biased as soon as the shards count different numbers of
    tokens).  The count is all-reduced without autograd; all ranks of ``group`` must call this."""
    n = _size(group)
    cnt = n_valid.detach().to(torch.float32).reshape(1).clone()
    if n > 1:
        dist.all_reduce(cnt, group=group)
    return loss_sum * (n / cnt[0])


def context_positions(t_local: int, group=None, layout: str = "contiguous", device=None):
    """Global token positions of this rank's ``t_local`` tokens under ``layout``."""
    n, r = _size(group), _rank(group)
    parts = 1 if layout == "contiguous" else 2
    tc = t_local // parts
    return torch.cat([torch.arange(c * tc, (c + 1) * tc, device=device) for c in _chunk_ids(r, n, layout)])


class CPCausalSelfAttention(torch.nn.Module):
    """GPT-2 attention over a context-parallel group: this rank's tokens' packed q|k|v projection,
    ring attention across the group, output projection — the wrapped module's own parameters."""

    def __init__(self, attn, group=None, layout: str = "contiguous"):
        super().__init__()
        self.c_attn, self.c_proj, self.n_head = attn.c_attn, attn.c_proj, attn.n_head
        self.hip_gemm = getattr(attn, "hip_gemm", False)
        self.group, self.layout = group, layout

    def forward(self, x, fast: bool = False):
        from .. import ops

        B, T, C = x.shape
        lin = ops.gemm_linear if (fast and self.hip_gemm) else ops.linear
        qkv = lin(x, self.c_attn.weight, self.c_attn.bias)
        H, D = self.n_head, C // self.n_head
        q, k, v = (t.view(B, T, H, D).transpose(1, 2) for t in qkv.split(C, dim=2))
        y = ring_attention(q, k, v, causal=True, group=self.group, layout=self.layout)
        return lin(y.transpose(1, 2).reshape(B, T, C), self.c_proj.weight, self.c_proj.bias)


def parallelize_gpt2_context(model, group=None, layout: str = "contiguous"):
    """Context parallelism for a (replicated) ``models.GPT2`` in place: every rank feeds its
    :func:`shard_context` part of each sequence (``idx``/``targets`` [B, T/n]; GPT-2's targets are
    already the next tokens, aligned with ``idx``); positions are the global ones, attention is
    :func:`ring_attention` over ``group``.  Each rank's loss is its :func:`context_loss` share, so
    averaging losses and gradients over ``group`` (e.g. DDP over a group that contains it) gives
    exactly the full-sequence loss and gradients, ignored targets included.  Attention dropout is
    not implemented in the ring blocks: a model with ``config.dropout > 0`` is refused rather than
    silently trained without it.  Returns the model."""
    p = float(getattr(getattr(model, "config", None), "dropout", 0.0) or 0.0)
    if p > 0.0:
        raise ValueError(f"parallelize_gpt2_context: dropout {p} is not supported by ring attention "
                         "(set config.dropout = 0.0)")
    for blk in model.h:
        blk.attn = CPCausalSelfAttention(blk.attn, group, layout)
    model.position_ids = lambda T, device: context_positions(T, group, layout, device)
    model.context_group = (group,)
    return model


class CPLlamaAttention(torch.nn.Module):
    """Llama attention over a context-parallel group: fused q|k|v projection, RoPE at this rank's
    global positions (``nbd::rope_`` in place on the projection — the fused-in-attention rotation
    assumes q and k share positions, which ring blocks do not), grouped-query ring attention,
    output projection; the wrapped module's own parameters."""

    def __init__(self, attn, group=None, layout: str = "contiguous"):
        super().__init__()
        self.qkv_proj, self.o_proj = attn.qkv_proj, attn.o_proj
        self.H, self.Hkv, self.D = attn.H, attn.Hkv, attn.D
        self.group, self.layout = group, layout

    def forward(self, x, cos, sin):
        from .. import ops

        B, T, _ = x.shape
        H, Hkv, D = self.H, self.Hkv, self.D
        qkv = ops.gemm_linear(x, self.qkv_proj.weight)
        if qkv._base is not None:  # the GEMM's output is a view of its autograd output: no in-place on it
            qkv = qkv.clone()
        qkv = ops.rope_(qkv, cos, sin, H + Hkv, D)
        q = qkv[:, :, : H * D].view(B, T, H, D).transpose(1, 2)
        k = qkv[:, :, H * D:(H + Hkv) * D].view(B, T, Hkv, D).transpose(1, 2)
        v = qkv[:, :, (H + Hkv) * D:].view(B, T, Hkv, D).transpose(1, 2)
        y = ring_attention(q, k, v, causal=True, group=self.group, layout=self.layout)
        return ops.gemm_linear(y.transpose(1, 2).reshape(B, T, H * D), self.o_proj.weight)


def parallelize_llama_context(model, group=None, layout: str = "contiguous"):
    """Context parallelism for a native ``models.llama`` ``LlamaModel`` or ``LlamaForCausalLM`` in
    place: every rank feeds its :func:`shard_context` part of each sequence; RoPE tables are taken
    at the rank's global positions and attention is :func:`ring_attention` over ``group``.

    ``LlamaForCausalLM`` then expects ``labels`` already shifted on the full sequence
    (:func:`shift_labels`, then :func:`shard_context`) and returns its :func:`context_loss` share.
    ``LlamaForSequenceClassification`` is refused: it pools the last non-pad token of the whole
    sequence, which lives on one rank only.  Returns the model."""
    from .. import ops
    from ..models.llama import LlamaForCausalLM, LlamaModel

    if isinstance(model, LlamaForCausalLM):
        base = model.model
        model.context_group = (group,)
    elif isinstance(model, LlamaModel):
        base = model
    else:
        raise TypeError(f"parallelize_llama_context: {type(model).__name__} is not supported (LlamaModel or "
                        "LlamaForCausalLM; a sequence-classification head pools one token of the whole sequence)")
    c = base.config
    cache = {}

    def rope(T, device):
        key = (str(device), T)
        if key not in cache:
            n = _size(group)
            cos, sin = ops.rope_tables(T * n, c.head_dim, c.rope_theta, device, scaling=c.rope_scaling)
            pos = context_positions(T, group, layout, device)
            cache[key] = (cos[pos].contiguous(), sin[pos].contiguous())
        return cache[key]

    base.rope = rope
    for layer in base.layers:
        layer.self_attn = CPLlamaAttention(layer.self_attn, group, layout)
    return model


__all__ = ["ring_attention", "shard_context", "gather_context", "context_positions", "shift_labels", "context_loss",
           "CPCausalSelfAttention",
           "parallelize_gpt2_context", "CPLlamaAttention", "parallelize_llama_context"]
