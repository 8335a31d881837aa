"""Pipeline parallelism: GPipe and 1F1B schedules over point-to-point send/recv.

Not in the reference (SURVEY.md §2.6 rows D4–D8: pipeline parallelism would be user code calling
``dist.send`` / ``dist.recv`` inside cells).  A stage is any ``nn.Module`` living on this rank;
:func:`pipeline_step` runs one optimizer step's worth of micro-batches through the stages of
``group`` (rank r of the group = stage r) and leaves the accumulated gradients in each stage's
parameters:

* ``schedule="gpipe"``: all forwards, then all backwards (activation memory ∝ micro-batches);
* ``schedule="1f1b"``: ``n_stages − r − 1`` warm-up forwards, then one-forward-one-backward, then the
  cool-down backwards — at most ``n_stages − r`` micro-batches of activations alive per stage.

Adjacent stages exchange activations forward and gradients backward; in the steady 1F1B phase the
send of one direction and the receive of the other are posted together (``batch_isend_irecv``) so
they overlap on the link.  On an MI355X node every stage pair is one direct xGMI link apart, so the
stage order can follow the model without regard to topology; with 288 GB per GPU, the 1F1B
memory bound matters mainly for very long sequences.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

from .p2p import batch_isend_irecv


def _size(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def _rank(group) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def _glob(group, r: int) -> int:
    return dist.get_global_rank(group, r) if group is not None else r


class _P2P:
    def __init__(self, group, shape, dtype, device):
        self.group, self.shape, self.dtype, self.device = group, tuple(shape), dtype, device
        self.stage, self.n = _rank(group), _size(group)
        self.prev = _glob(group, self.stage - 1) if self.stage > 0 else None
        self.next = _glob(group, self.stage + 1) if self.stage < self.n - 1 else None

    def _buf(self):
        return torch.empty(self.shape, dtype=self.dtype, device=self.device)

    def _run(self, ops):
        if ops:
            for w in batch_isend_irecv(ops):
                w.wait()

    def exchange(self, send_to=None, send=None, recv_from=None):
        ops, buf = [], None
        if send_to is not None:
            ops.append(dist.P2POp(dist.isend, send.contiguous(), send_to, self.group))
        if recv_from is not None:
            buf = self._buf()
            ops.append(dist.P2POp(dist.irecv, buf, recv_from, self.group))
        self._run(ops)
        return buf


def pipeline_step(stage: torch.nn.Module, micro_batches: Optional[Sequence[torch.Tensor]],
                  targets: Optional[Sequence[torch.Tensor]], loss_fn: Optional[Callable], n_micro: int,
                  act_shape, act_dtype=torch.float32, schedule: str = "1f1b", group=None):
    """Run ``n_micro`` micro-batches forward and backward through the pipeline.

    ``micro_batches`` are needed on the first stage only, ``targets`` and ``loss_fn(out, target)``
    on the last only; ``act_shape`` / ``act_dtype`` describe every inter-stage activation (one
    micro-batch).  Each micro-batch's loss is divided by ``n_micro``, so the gradients equal those of
    the mean loss over the whole batch.  Returns the summed (mean) loss on the last stage, None on
    the others."""
    if schedule not in ("1f1b", "gpipe"):
        raise ValueError(f"unknown schedule {schedule!r}")
    dev = next(stage.parameters()).device
    p = _P2P(group, act_shape, act_dtype, dev)
    first, last = p.stage == 0, p.stage == p.n - 1
    inputs: List[Optional[torch.Tensor]] = []
    outputs: List[torch.Tensor] = []
    total = torch.zeros((), device=dev)
    fwd_i = [0]

    def forward(x):
        i = fwd_i[0]
        fwd_i[0] += 1
        if first:
            x = micro_batches[i]
        else:
            x.requires_grad_()
        out = stage(x)
        if last:
            out = loss_fn(out, targets[i]) / n_micro
            total.add_(out.detach())
        inputs.append(None if first else x)
        outputs.append(out)
        return out

    def backward(g):
        x, out = inputs.pop(0), outputs.pop(0)
        torch.autograd.backward(out, None if last else g)
        return None if first else x.grad

    def recv_fwd():
        return None if first else p.exchange(recv_from=p.prev)

    if schedule == "gpipe":
        for _ in range(n_micro):
            y = forward(recv_fwd())
            if not last:
                p.exchange(send_to=p.next, send=y)
        for _ in range(n_micro):
            g = None if last else p.exchange(recv_from=p.next)
            gx = backward(g)
            if not first:
                p.exchange(send_to=p.prev, send=gx)
        return total if last else None

    warm = min(p.n - p.stage - 1, n_micro)
    for _ in range(warm):
        y = forward(recv_fwd())
        if not last:
            p.exchange(send_to=p.next, send=y)
    steady = n_micro - warm
    x = recv_fwd() if steady > 0 else None
    for i in range(steady):
        y = forward(x)
        g = None if last else p.exchange(send_to=p.next, send=y, recv_from=p.next)
        gx = backward(g)
        if i == steady - 1:
            if not first:
                p.exchange(send_to=p.prev, send=gx)
        else:
            x = p.exchange(send_to=p.prev if not first else None, send=gx,
                           recv_from=p.prev if not first else None)
    for _ in range(warm):
        g = p.exchange(recv_from=p.next)
        gx = backward(g)
        if not first:
            p.exchange(send_to=p.prev, send=gx)
    return total if last else None


def split_sequential(model: torch.nn.Sequential, n_stages: int, stage: int) -> torch.nn.Sequential:
    """Stage ``stage`` of ``model`` cut into ``n_stages`` contiguous runs of layers (balanced by
    parameter count)."""
    layers = list(model)
    L = len(layers)
    if not 0 < n_stages <= L:
        raise ValueError(f"cannot cut {L} layers into {n_stages} stages")
    cum, acc = [], 0
    for m in layers:
        acc += sum(p.numel() for p in m.parameters()) or 1
        cum.append(acc)
    bounds = [0]
    for s in range(1, n_stages):
        b = next(i + 1 for i, c in enumerate(cum) if c >= acc * s / n_stages)
        bounds.append(min(max(b, bounds[-1] + 1), L - (n_stages - s)))
    bounds.append(L)
    return torch.nn.Sequential(*layers[bounds[stage]:bounds[stage + 1]])


__all__ = ["pipeline_step", "split_sequential"]
