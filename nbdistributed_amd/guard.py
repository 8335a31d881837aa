"""Fail-fast guard for collectives issued from ``%%rank [subset]`` cells.

Reference behaviour: ``%%rank [0]`` + ``dist.all_reduce(x)`` blocks
rank 0 forever, because the other ranks are not executing the cell; nothing detects or aborts
it (with ``-t`` unset the notebook hangs for good).

While a subset cell runs, the worker wraps the public ``torch.distributed`` collectives: a call
whose group contains a rank that is not executing this cell raises ``SubsetCollectiveError``
immediately, naming the missing ranks.  Collectives on groups made only of executing ranks
(``dist.new_group([0, 1])`` inside ``%%rank [0,1]``) and point-to-point ops between executing
ranks are allowed.  Calls made inside libraries through ``torch.distributed.<fn>`` are covered;
C++-internal collectives (e.g. torch DDP's reducer) are not — for those the RCCL communicator
abort in the interrupt watchdog is the backstop.
"""
from __future__ import annotations

import functools
import threading
from typing import Iterable, List, Optional, Set

COLLECTIVES = ["all_reduce", "broadcast", "all_gather", "all_gather_into_tensor", "reduce_scatter",
               "reduce_scatter_tensor", "all_to_all", "all_to_all_single", "barrier", "reduce", "gather", "scatter",
               "broadcast_object_list", "all_gather_object", "gather_object", "scatter_object_list",
               "monitored_barrier", "all_reduce_coalesced", "all_gather_coalesced"]
# isend/irecv are not wrapped: dist.P2POp checks them by identity (batch_isend_irecv)
P2P = {"send": "dst", "recv": "src"}


class SubsetCollectiveError(RuntimeError):
    pass


class CollectiveGuard:
    def __init__(self):
        self.active: Optional[Set[int]] = None
        self._installed = False
        self._orig = {}
        self._lock = threading.Lock()

    def _group_ranks(self, dist, group) -> List[int]:
        if group is None or group is dist.group.WORLD:
            return list(range(dist.get_world_size()))
        try:
            return list(dist.get_process_group_ranks(group))
        except Exception:
            return list(range(dist.get_world_size()))

    def _wrap(self, dist, name, fn, peer_arg=None):
        guard = self

        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            active = guard.active
            if active is not None and dist.is_initialized():
                if peer_arg is not None:
                    peer = kwargs.get(peer_arg, args[1] if len(args) > 1 else None)
                    if peer is not None and peer not in active:
                        raise SubsetCollectiveError(
                            f"dist.{name}(..., {peer_arg}={peer}) inside %%rank [{_fmt(active)}]: rank {peer} "
                            f"is not executing this cell, so this call would block forever. Run it in a "
                            f"%%distributed cell, or include rank {peer} in the %%rank spec.")
                else:
                    group = kwargs.get("group")
                    if group is None:
                        group = _positional_group(name, args)
                    members = self._group_ranks(dist, group)
                    missing = sorted(set(members) - active)
                    if missing:
                        raise SubsetCollectiveError(
                            f"dist.{name} on a group with ranks {_fmt(members)} inside %%rank [{_fmt(active)}]: "
                            f"ranks {missing} are not executing this cell, so this collective would block forever. "
                            f"Run it in a %%distributed cell, or use dist.new_group({sorted(active)}).")
            return fn(*args, **kwargs)

        wrapper.__wrapped_by_nbd__ = True
        return wrapper

    def install(self) -> None:
        with self._lock:
            if self._installed:
                return
            import torch.distributed as dist

            for name in COLLECTIVES:
                fn = getattr(dist, name, None)
                if fn is not None and not getattr(fn, "__wrapped_by_nbd__", False):
                    self._orig[name] = fn
                    setattr(dist, name, self._wrap(dist, name, fn))
            for name, arg in P2P.items():
                fn = getattr(dist, name, None)
                if fn is not None and not getattr(fn, "__wrapped_by_nbd__", False):
                    self._orig[name] = fn
                    setattr(dist, name, self._wrap(dist, name, fn, peer_arg=arg))
            self._installed = True

    def uninstall(self) -> None:
        with self._lock:
            if not self._installed:
                return
            import torch.distributed as dist

            for name, fn in self._orig.items():
                setattr(dist, name, fn)
            self._orig.clear()
            self._installed = False

    def enter(self, ranks: Optional[Iterable[int]], world_size: int) -> None:
        rs = set(ranks) if ranks is not None else None
        self.active = rs if rs is not None and len(rs) < world_size else None

    def exit(self) -> None:
        self.active = None


# positional index of `group` for functions that take it positionally
_GROUP_POS = {"all_reduce": 2, "broadcast": 2, "all_gather": 2, "all_gather_into_tensor": 2, "reduce_scatter": 3,
              "reduce_scatter_tensor": 3, "barrier": 0, "reduce": 3, "gather": 3, "scatter": 3,
              "all_to_all": 2, "all_to_all_single": 4, "broadcast_object_list": 2, "all_gather_object": 2,
              "gather_object": 3, "scatter_object_list": 3, "monitored_barrier": 0}


def _positional_group(name: str, args) -> object:
    i = _GROUP_POS.get(name)
    if i is not None and len(args) > i:
        return args[i]
    return None


def _fmt(ranks) -> str:
    from .utils.ranks import format_ranks

    return format_ranks(list(ranks))
