"""Tensor parallelism (Megatron-style column / row sharding) for cells.

The reference has no model parallelism at all (SURVEY.md §2.6 rows D4–D8: users would write the
collectives themselves in ``%%distributed`` cells).  This module gives those cells ready-made
building blocks whose compute runs on the HIP MFMA GEMM (``ops.gemm_linear`` / ``ops.mlp_gelu``)
and whose communication is one RCCL all-reduce per sharded block in each direction:

* :func:`copy_to_tp` / :func:`reduce_from_tp` / :func:`gather_from_tp` / :func:`scatter_to_tp` —
  the four autograd-aware conjugate collectives (identity ↔ all-reduce, all-gather ↔ split);
* :class:`ColumnParallelLinear` / :class:`RowParallelLinear` — ``nn.Linear`` with the output
  (column) or input (row) features split over the group; ``from_linear`` shards an existing
  full-size layer, so the ``%%rank[0]``-build + broadcast pattern (BASELINE config 3) feeds TP too;
* :func:`parallelize_gpt2` — GPT-2 blocks rewritten in place: attention heads and the MLP's hidden
  features split over the TP group, two all-reduces forward and two backward per block.

Why TP degree matters on MI355X: each all-reduce moves ``B·T·C`` activations over xGMI point-to-point
links (≈153 GB/s per link, 7 links per GPU), so TP pays off for wide layers on 2–4 GPUs that share
links directly; the 288 GB of HBM per GPU means plain DP fits models that would need TP elsewhere.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn


def _size(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


class _CopyToTP(torch.autograd.Function):
    """Identity forward; all-reduce of the gradient backward (input of a column-parallel layer)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if _size(ctx.group) > 1:
            g = g.contiguous()
            dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    """All-reduce forward (sum of the row-parallel partial products); identity backward."""

    @staticmethod
    def forward(ctx, x, group):
        y = x.contiguous()
        if y.data_ptr() == x.data_ptr():
            y = y.clone()
        if _size(group) > 1:
            dist.all_reduce(y, group=group)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None


def _all_gather_last(x, group):
    n = _size(group)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty((n * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=group)
    return out.view((n,) + tuple(x.shape)).movedim(0, -2).reshape(*x.shape[:-1], n * x.shape[-1])


class _GatherFromTP(torch.autograd.Function):
    """All-gather along the last dim forward; keep the own slice backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _all_gather_last(x, group)

    @staticmethod
    def backward(ctx, g):
        n = _size(ctx.group)
        if n == 1:
            return g, None
        return g.chunk(n, dim=-1)[_rank(ctx.group)].contiguous(), None


class _ScatterToTP(torch.autograd.Function):
    """Keep the own last-dim slice forward; all-gather of the gradient backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        n = _size(group)
        return x if n == 1 else x.chunk(n, dim=-1)[_rank(group)].contiguous()

    @staticmethod
    def backward(ctx, g):
        return _all_gather_last(g, ctx.group), None


def copy_to_tp(x, group=None):
    return _CopyToTP.apply(x, group)


def reduce_from_tp(x, group=None):
    return _ReduceFromTP.apply(x, group)


def gather_from_tp(x, group=None):
    return _GatherFromTP.apply(x, group)


def scatter_to_tp(x, group=None):
    return _ScatterToTP.apply(x, group)


def _linear(x, w, b=None):
    from .. import ops

    return ops.gemm_linear(x, w, b)


class ColumnParallelLinear(nn.Module):
    """``y = x·Wᵀ + b`` with W's output features split over the group: rank r holds rows
    ``[r·out/n, (r+1)·out/n)``.  The output stays sharded unless ``gather_output``."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, group=None,
                 gather_output: bool = False, device=None, dtype=None):
        super().__init__()
        n = _size(group)
        if out_features % n:
            raise ValueError(f"out_features={out_features} is not divisible by the TP size {n}")
        self.group, self.gather_output = group, gather_output
        self.in_features, self.out_features, self.local_out = in_features, out_features, out_features // n
        self.weight = nn.Parameter(torch.empty(self.local_out, in_features, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.zeros(self.local_out, device=device, dtype=dtype)) if bias else None
        nn.init.normal_(self.weight, std=0.02)

    @classmethod
    def from_linear(cls, lin: nn.Linear, group=None, gather_output: bool = False, rows=None):
        """Shard a full ``nn.Linear`` (identical on every rank).  ``rows`` overrides the row index
        list of this rank's shard (e.g. the q|k|v head rows of a packed attention projection)."""
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, group, gather_output,
                device="meta")
        if rows is None:
            n, r = _size(group), _rank(group)
            rows = torch.arange(r * m.local_out, (r + 1) * m.local_out)
        rows = torch.as_tensor(rows, device=lin.weight.device)
        m.weight = nn.Parameter(lin.weight.detach()[rows].clone())
        m.bias = nn.Parameter(lin.bias.detach()[rows].clone()) if lin.bias is not None else None
        return m

    def forward(self, x):
        y = _linear(copy_to_tp(x, self.group), self.weight, self.bias)
        return gather_from_tp(y, self.group) if self.gather_output else y


class RowParallelLinear(nn.Module):
    """``y = x·Wᵀ + b`` with W's input features split over the group: rank r holds columns
    ``[r·in/n, (r+1)·in/n)`` and multiplies its slice of ``x``; the partial products are summed by
    one all-reduce, then the (replicated) bias is added."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, group=None,
                 input_is_parallel: bool = True, device=None, dtype=None):
        super().__init__()
        n = _size(group)
        if in_features % n:
            raise ValueError(f"in_features={in_features} is not divisible by the TP size {n}")
        self.group, self.input_is_parallel = group, input_is_parallel
        self.in_features, self.out_features, self.local_in = in_features, out_features, in_features // n
        self.weight = nn.Parameter(torch.empty(out_features, self.local_in, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.zeros(out_features, device=device, dtype=dtype)) if bias else None
        nn.init.normal_(self.weight, std=0.02)

    @classmethod
    def from_linear(cls, lin: nn.Linear, group=None, input_is_parallel: bool = True):
        m = cls(lin.in_features, lin.out_features, lin.bias is not None, group, input_is_parallel,
                device="meta")
        r = _rank(group)
        m.weight = nn.Parameter(lin.weight.detach()[:, r * m.local_in:(r + 1) * m.local_in].clone())
        m.bias = nn.Parameter(lin.bias.detach().clone()) if lin.bias is not None else None
        return m

    def forward(self, x):
        if not self.input_is_parallel:
            x = scatter_to_tp(x, self.group)
        y = reduce_from_tp(_linear(x, self.weight), self.group)
        return y + self.bias if self.bias is not None else y


class TPCausalSelfAttention(nn.Module):
    """GPT-2 attention with this rank's heads: packed q|k|v rows of its heads (column-parallel),
    flash attention on ``n_head / n`` heads, row-parallel output projection."""

    def __init__(self, attn, group=None):
        super().__init__()
        n, r = _size(group), _rank(group)
        H = attn.n_head
        if H % n:
            raise ValueError(f"n_head={H} is not divisible by the TP size {n}")
        C = attn.c_attn.in_features
        D = C // H
        h0, h1 = r * (H // n) * D, (r + 1) * (H // n) * D
        rows = torch.cat([torch.arange(h0, h1) + i * C for i in range(3)])
        self.group, self.n_head = group, H // n
        self.c_attn = ColumnParallelLinear.from_linear(attn.c_attn, group, rows=rows)
        self.c_proj = RowParallelLinear.from_linear(attn.c_proj, group)

    def forward(self, x, fast: bool = False, kv=None):
        from .. import ops

        qkv = self.c_attn(x)
        if kv is not None:  # generation prefill: this rank's heads into its cache
            kv[0].store(kv[1], qkv)
        return self.c_proj(ops.attention_qkv(qkv, self.n_head, causal=True))

    def decode(self, x, ln, cache, layer: int, pos):
        """Generation step on this rank's heads: fused norm + q|k|v shard, decode attention on the
        local cache, the row-parallel projection's partial product (rank 0 adds bias and
        residual), one all-reduce."""
        from .. import ops

        first = _rank(self.group) == 0
        qkv = ops.linear_small(x, self.c_attn.weight, self.c_attn.bias, norm=("ln", ln.weight, ln.bias, ln.eps))
        a = cache.attend(layer, qkv, pos)
        y = ops.linear_small(a, self.c_proj.weight, self.c_proj.bias if first else None, residual=x if first else None)
        if _size(self.group) > 1:
            dist.all_reduce(y, group=self.group)
        return y


class TPMLP(nn.Module):
    """GPT-2 MLP with this rank's hidden features: ``c_fc`` column-parallel, GELU on the shard,
    ``c_proj`` row-parallel (GELU/GELU′ fused into the HIP GEMM epilogues on the GPU path)."""

    def __init__(self, mlp, group=None):
        super().__init__()
        self.group = group
        self.c_fc = ColumnParallelLinear.from_linear(mlp.c_fc, group)
        self.c_proj = RowParallelLinear.from_linear(mlp.c_proj, group)

    def forward(self, x, fast: bool = False):
        from .. import ops

        x = copy_to_tp(x, self.group)
        y = ops.mlp_gelu(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, None)
        y = reduce_from_tp(y, self.group)
        return y + self.c_proj.bias if self.c_proj.bias is not None else y

    def decode(self, x, ln):
        """Generation step on this rank's MLP features (one all-reduce; rank 0 adds bias + residual)."""
        from .. import ops

        first = _rank(self.group) == 0
        f = ops.linear_small(x, self.c_fc.weight, self.c_fc.bias, norm=("ln", ln.weight, ln.bias, ln.eps), act="gelu")
        y = ops.linear_small(f, self.c_proj.weight, self.c_proj.bias if first else None, residual=x if first else None)
        if _size(self.group) > 1:
            dist.all_reduce(y, group=self.group)
        return y


def parallelize_gpt2(model, group=None):
    """Shard every block of a (replicated, identically initialised) ``models.GPT2`` over ``group``
    in place: heads and MLP features split, embeddings / LayerNorms / LM head replicated.  Returns
    the model.  Combine with data parallelism over a different group for 2-D parallelism."""
    for blk in model.h:
        blk.attn = TPCausalSelfAttention(blk.attn, group)
        blk.mlp = TPMLP(blk.mlp, group)
    return model


class TPLlamaAttention(nn.Module):
    """Llama / Qwen2 / Mistral attention with this rank's query heads and the key/value heads they
    read (grouped-query attention splits by kv-head groups: ``Hkv`` must divide by the TP size);
    RoPE inside the HIP attention kernels as in the unsharded model; row-parallel ``o_proj``."""

    def __init__(self, attn, group=None):
        super().__init__()
        n, r = _size(group), _rank(group)
        H, Hkv, D = attn.H, attn.Hkv, attn.D
        if Hkv % n:
            raise ValueError(f"num_key_value_heads={Hkv} is not divisible by the TP size {n}")
        q0, q1 = r * (H // n) * D, (r + 1) * (H // n) * D
        k0, k1 = r * (Hkv // n) * D, (r + 1) * (Hkv // n) * D
        rows = torch.cat([torch.arange(q0, q1), H * D + torch.arange(k0, k1), (H + Hkv) * D + torch.arange(k0, k1)])
        self.group, self.H, self.Hkv, self.D, self.window = group, H // n, Hkv // n, D, attn.window
        self.qkv_proj = ColumnParallelLinear.from_linear(attn.qkv_proj, group, rows=rows)
        self.o_proj = RowParallelLinear.from_linear(attn.o_proj, group)

    def forward(self, x, cos, sin, kv=None):
        from .. import ops

        qkv = self.qkv_proj(x)
        if kv is not None:
            kv[0].store(kv[1], qkv, rope=(cos, sin))
        return self.o_proj(ops.attention_qkv(qkv, self.H, causal=True, n_kv_head=self.Hkv, rope=(cos, sin)))

    def decode(self, x, norm_w, eps, cache, layer: int, pos, rope):
        from .. import ops

        first = _rank(self.group) == 0
        qkv = ops.linear_small(x, self.qkv_proj.weight, self.qkv_proj.bias, norm=("rms", norm_w, eps))
        a = cache.attend(layer, qkv, pos, rope=rope)
        y = ops.linear_small(a, self.o_proj.weight, self.o_proj.bias if first else None, residual=x if first else None)
        if _size(self.group) > 1:
            dist.all_reduce(y, group=self.group)
        return y


class TPLlamaMLP(nn.Module):
    """SwiGLU MLP with this rank's intermediate features: its gate rows and the matching up rows
    (so SwiGLU stays in the GEMM epilogue on the shard), row-parallel ``down_proj``."""

    def __init__(self, mlp, group=None):
        super().__init__()
        n, r = _size(group), _rank(group)
        inter = mlp.down_proj.in_features
        if inter % n:
            raise ValueError(f"intermediate_size={inter} is not divisible by the TP size {n}")
        i0, i1 = r * inter // n, (r + 1) * inter // n
        rows = torch.cat([torch.arange(i0, i1), inter + torch.arange(i0, i1)])
        self.group = group
        self.gate_up_proj = ColumnParallelLinear.from_linear(mlp.gate_up_proj, group, rows=rows)
        self.down_proj = RowParallelLinear.from_linear(mlp.down_proj, group)

    def forward(self, x):
        from .. import ops

        x = copy_to_tp(x, self.group)
        return reduce_from_tp(ops.mlp_swiglu(x, self.gate_up_proj.weight, self.down_proj.weight), self.group)

    def decode(self, x, norm_w, eps):
        from .. import ops

        first = _rank(self.group) == 0
        f = ops.linear_small(x, self.gate_up_proj.weight, norm=("rms", norm_w, eps), act="swiglu")
        y = ops.linear_small(f, self.down_proj.weight, residual=x if first else None)
        if _size(self.group) > 1:
            dist.all_reduce(y, group=self.group)
        return y


def parallelize_llama(model, group=None):
    """Tensor parallelism for the native Llama family (``models.llama``: ``LlamaModel`` or a
    wrapper with ``.model``), in place on a replicated, identically initialised model: query /
    key-value heads and MLP features split over ``group``; embeddings, norms and heads
    replicated.  Training (autograd collectives) and generation (per-rank KV caches) both work."""
    inner = model.model if hasattr(model, "model") else model
    for layer in inner.layers:
        layer.self_attn = TPLlamaAttention(layer.self_attn, group)
        layer.mlp = TPLlamaMLP(layer.mlp, group)
    return model


__all__ = ["copy_to_tp", "reduce_from_tp", "gather_from_tp", "scatter_to_tp", "ColumnParallelLinear",
           "RowParallelLinear", "TPCausalSelfAttention", "TPMLP", "parallelize_gpt2", "TPLlamaAttention",
           "TPLlamaMLP", "parallelize_llama"]
