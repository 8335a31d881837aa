"""N-D process-group mesh for combining data / pipeline / context / tensor parallelism.

``ParallelMesh(dp=2, cp=2, tp=2)`` lays the world out as a row-major grid over the named axes
(the LAST axis varies fastest, so ``tp`` groups are consecutive ranks) and creates one process
group per line of the grid on every axis.  Every rank calls ``dist.new_group`` for every group in
the same order (a torch.distributed requirement), then keeps the groups it belongs to.

On an MI355X node the eight GPUs are fully connected by xGMI (one hop between any pair), so axis
order does not change link distance inside a node; it matters across nodes: keep the
communication-heavy axes (tp, cp — per-layer collectives) last so their groups stay inside a node,
and dp / pp (one bucketed all-reduce per step, point-to-point activations) first.
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Optional

import torch.distributed as dist


class ParallelMesh:
    """Named-axis process groups.  ``ParallelMesh(dp=2, cp=2)`` on 4 ranks: dp groups
    {0, 2} and {1, 3}, cp groups {0, 1} and {2, 3}.  Axes of size 1 get a group of one rank."""

    def __init__(self, backend: Optional[str] = None, **axes: int):
        if not axes:
            raise ValueError("ParallelMesh needs at least one axis, e.g. ParallelMesh(dp=2, tp=4)")
        self.names: List[str] = list(axes)
        self.shape: List[int] = [int(axes[a]) for a in self.names]
        world = dist.get_world_size() if dist.is_initialized() else 1
        total = 1
        for s in self.shape:
            total *= s
        if total != world:
            raise ValueError(f"mesh {dict(axes)} has {total} ranks but the world has {world}")
        me = dist.get_rank() if dist.is_initialized() else 0
        self.rank = me
        self.coords: Dict[str, int] = {}
        rem = me
        for a, s in zip(reversed(self.names), reversed(self.shape)):
            self.coords[a] = rem % s
            rem //= s
        self._groups: Dict[str, object] = {}
        self._members: Dict[str, List[int]] = {}
        strides = [1] * len(self.shape)
        for i in range(len(self.shape) - 2, -1, -1):
            strides[i] = strides[i + 1] * self.shape[i + 1]
        for ax, name in enumerate(self.names):
            others = [range(s) for i, s in enumerate(self.shape) if i != ax]
            for fixed in itertools.product(*others):
                members = []
                for v in range(self.shape[ax]):
                    c = list(fixed)
                    c.insert(ax, v)
                    members.append(sum(ci * st for ci, st in zip(c, strides)))
                g = dist.new_group(members, backend=backend) if dist.is_initialized() else None
                if me in members:
                    self._groups[name], self._members[name] = g, members

    def group(self, axis: str):
        """The process group of this rank along ``axis``."""
        return self._groups[axis]

    def members(self, axis: str) -> List[int]:
        """Global ranks of this rank's group along ``axis`` (in axis order)."""
        return list(self._members[axis])

    def size(self, axis: str) -> int:
        return self.shape[self.names.index(axis)]

    def coord(self, axis: str) -> int:
        """This rank's index along ``axis`` (= its rank inside :meth:`group`)."""
        return self.coords[axis]

    def __repr__(self) -> str:
        axes = ", ".join(f"{a}={s}" for a, s in zip(self.names, self.shape))
        return f"ParallelMesh({axes}; rank {self.rank} at {self.coords})"


__all__ = ["ParallelMesh"]
