"""Expert parallelism: a top-k mixture-of-experts layer whose experts are split over an EP group.

Not in the reference (SURVEY.md §2.6 rows D4–D8: "EP … user code calling ``dist.all_to_all``
inside cells"); this is that code as a library layer.  Per forward:

1. the (replicated) router scores every local token, keeps the top-k experts and renormalises
   their gates;
2. the token copies are sorted by expert, the per-expert counts are exchanged with one small
   all-to-all, and the tokens themselves travel with one variable-split ``all_to_all_single`` to
   the ranks that own their experts (the only host sync: the split sizes);
3. each local expert runs its MLP on one contiguous slice (the HIP GEMM with GELU fused in the
   epilogues where the slice shape allows, ``F.linear`` otherwise);
4. the results return with the inverse all-to-all and are summed into their tokens, gate-weighted.

Backward is the same two all-to-alls with the split sizes swapped.  On MI355X every dispatch is a
single all-to-all over the direct xGMI links between every GPU pair — no ring hops — so EP degree
up to the full node (8) keeps each token one link away from its expert.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


def _size(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def _a2a(x, out_splits: List[int], in_splits: List[int], group):
    if _size(group) == 1:
        return x
    x = x.contiguous()
    out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
    dist.all_to_all_single(out, x, out_splits, in_splits, group=group)
    return out


class _AllToAll(torch.autograd.Function):
    """Variable-split all-to-all along dim 0; backward sends the gradients back the same way."""

    @staticmethod
    def forward(ctx, x, out_splits, in_splits, group):
        ctx.splits, ctx.group = (out_splits, in_splits), group
        return _a2a(x, out_splits, in_splits, group)

    @staticmethod
    def backward(ctx, g):
        out_splits, in_splits = ctx.splits
        return _a2a(g, in_splits, out_splits, ctx.group), None, None, None


def all_to_all(x, out_splits: List[int], in_splits: List[int], group=None):
    """Autograd-aware ``all_to_all_single`` of the rows of ``x``: ``in_splits[r]`` rows go to rank r,
    ``out_splits[r]`` rows arrive from rank r."""
    return _AllToAll.apply(x, list(out_splits), list(in_splits), group)


class MoE(nn.Module):
    """Top-k mixture of GELU-MLP experts, experts sharded over ``group`` (every rank must build it
    with the same seed so the router is replicated; rank r keeps experts
    ``[r·E/n, (r+1)·E/n)``).  ``forward(x)`` takes [..., C] tokens and returns the same shape; the
    Switch-style load-balancing loss of the last call is in ``self.aux_loss``."""

    def __init__(self, dim: int, hidden: int, n_experts: int, top_k: int = 2, group=None,
                 device=None, dtype=None):
        super().__init__()
        n = _size(group)
        if n_experts % n:
            raise ValueError(f"{n_experts} experts are not divisible by the expert-parallel size {n}")
        self.dim, self.hidden, self.n_experts, self.top_k, self.group = dim, hidden, n_experts, top_k, group
        self.n_local = n_experts // n
        self.first = _rank(group) * self.n_local
        kw = dict(device=device, dtype=dtype)
        self.router = nn.Linear(dim, n_experts, bias=False, **kw)
        w1 = torch.empty(n_experts, hidden, dim, **kw)
        w2 = torch.empty(n_experts, dim, hidden, **kw)
        nn.init.normal_(w1, std=1 / math.sqrt(dim))
        nn.init.normal_(w2, std=1 / math.sqrt(hidden))
        sl = slice(self.first, self.first + self.n_local)   # same draw on every rank, then keep the own experts
        self.w1 = nn.Parameter(w1[sl].clone())
        self.w2 = nn.Parameter(w2[sl].clone())
        self.aux_loss: Optional[torch.Tensor] = None

    def route(self, x2: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(expert ids [N, k], gates [N, k], router probabilities [N, E])."""
        probs = F.softmax(self.router(x2).float(), dim=-1)
        gates, idx = probs.topk(self.top_k, dim=-1)
        gates = gates / gates.sum(-1, keepdim=True)
        return idx, gates, probs

    def _expert(self, e: int, t: torch.Tensor) -> torch.Tensor:
        from .. import ops

        return ops.mlp_gelu(t, self.w1[e], None, self.w2[e], None)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        shape = x.shape
        x2 = x.reshape(-1, self.dim)
        N, k, E, n = x2.shape[0], self.top_k, self.n_experts, _size(self.group)
        idx, gates, probs = self.route(x2)
        # Switch-transformer balance loss: E · Σ_e (fraction of top-1 picks) · (mean probability)
        frac = torch.bincount(idx[:, 0], minlength=E).to(probs.dtype) / max(N, 1)
        self.aux_loss = E * (frac * probs.mean(0)).sum()

        flat_e = idx.reshape(-1)                                   # [N·k] expert of each token copy
        order = torch.argsort(flat_e, stable=True)
        tok = order // k                                           # source token of each sorted copy
        counts = torch.bincount(flat_e, minlength=E)               # per global expert
        recv_counts = counts.clone()
        if n > 1:                                                  # [n (src), E_local] after exchange
            recv_counts = torch.empty_like(counts)
            dist.all_to_all_single(recv_counts, counts, group=self.group)
        counts_h = counts.view(n, self.n_local).tolist()
        recv_h = recv_counts.view(n, self.n_local).tolist()
        send_splits = [sum(c) for c in counts_h]
        recv_splits = [sum(c) for c in recv_h]

        xs = all_to_all(x2[tok], recv_splits, send_splits, self.group)
        # received rows are grouped by source rank, then by local expert: regroup by expert
        le = torch.repeat_interleave(torch.arange(self.n_local, device=x.device).repeat(n),
                                     torch.tensor([c for row in recv_h for c in row], device=x.device))
        perm = torch.argsort(le, stable=True)
        xe = xs[perm]
        per_expert = [sum(recv_h[s][e] for s in range(n)) for e in range(self.n_local)]
        outs, o = [], 0
        for e, c in enumerate(per_expert):
            if c:
                outs.append(self._expert(e, xe[o:o + c]))
            o += c
        ye = torch.cat(outs) if outs else xe.new_zeros((0, self.dim))
        ys = torch.empty_like(ye).index_copy(0, perm, ye) if ye.shape[0] else ye
        y = all_to_all(ys, send_splits, recv_splits, self.group)   # back in this rank's sorted order
        w = gates.reshape(-1)[order].to(y.dtype).unsqueeze(1)
        out = torch.zeros_like(x2).index_add(0, tok, y * w)
        return out.reshape(shape)


__all__ = ["all_to_all", "MoE"]
