"""Point-to-point exchange for cells: ``batch_isend_irecv`` that also accepts this rank as a peer.

Reference: the reference exposes ``dist`` to cells and leaves point-to-point to the user
(``worker.py:160-167``); SURVEY §2.6 D5/§5.7 require ``send``/``recv`` and ``batch_isend_irecv`` to
work from cells over RCCL.  torch.distributed refuses a send or receive whose peer is the calling
rank (``_check_not_self_rank``), which makes every ring / pipeline schedule special-case the
degenerate group — a ring of one (context parallelism at cp=1), a pipeline whose two neighbouring
stages share a rank, a 1-GPU rehearsal of an N-GPU notebook.

Here an op whose peer is this rank is matched, in posting order, with the opposite op of the same
group, shape and dtype and served by one device copy on the current stream (what RCCL's own
self-send would do, minus a kernel launch on the NCCL stream and a stream join); every other op
goes to ``dist.batch_isend_irecv`` as one RCCL group.  The returned handles have the
``wait()`` / ``is_completed()`` surface of ``dist.Work``."""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class _Completed:
    """The handle of an exchange that finished when it was posted (stream-ordered copy)."""

    def wait(self, timeout=None) -> bool:
        return True

    def is_completed(self) -> bool:
        return True

    def result(self):
        return []


def _group_rank(group) -> int:
    return dist.get_rank(group) if group is not None else dist.get_rank()


def _global_peer(op: "dist.P2POp") -> int:
    peer = getattr(op, "peer", None)
    if peer is None:  # torch >= 2.6 P2POp may carry a group-relative peer instead
        return dist.get_global_rank(op.group, op.group_peer)
    return peer


def batch_isend_irecv(ops: List["dist.P2POp"]) -> List[object]:
    """``dist.batch_isend_irecv`` with self-peers allowed (module docstring)."""
    me = dist.get_rank()
    self_sends, self_recvs, rest = [], [], []
    for op in ops:
        if _global_peer(op) == me:
            (self_sends if op.op in (dist.isend, dist.send) else self_recvs).append(op)
        else:
            rest.append(op)
    if len(self_sends) != len(self_recvs):
        raise ValueError(f"batch_isend_irecv: {len(self_sends)} send(s) to this rank but {len(self_recvs)} "
                         "receive(s) from it")
    for s, r in zip(self_sends, self_recvs):
        if s.tensor.shape != r.tensor.shape or s.tensor.dtype != r.tensor.dtype:
            raise ValueError("batch_isend_irecv: a send to this rank and its matching receive differ in "
                             f"shape/dtype ({tuple(s.tensor.shape)}/{s.tensor.dtype} vs "
                             f"{tuple(r.tensor.shape)}/{r.tensor.dtype})")
        with torch.no_grad():
            r.tensor.copy_(s.tensor, non_blocking=True)
    works: List[object] = list(dist.batch_isend_irecv(rest)) if rest else []
    if self_sends and not works:
        works.append(_Completed())
    return works


def sendrecv(send: torch.Tensor, recv: torch.Tensor, dst: int, src: int, group: Optional[object] = None) -> None:
    """Send ``send`` to global rank ``dst`` while receiving ``recv`` from ``src`` (either may be
    this rank), blocking the current stream until both are done."""
    ops = [dist.P2POp(dist.isend, send, dst, group), dist.P2POp(dist.irecv, recv, src, group)]
    for w in batch_isend_irecv(ops):
        w.wait()


__all__ = ["batch_isend_irecv", "sendrecv"]
