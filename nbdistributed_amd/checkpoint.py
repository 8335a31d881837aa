"""Checkpoint / resume of worker namespaces (``%dist_checkpoint``).

The reference has none: worker namespaces die with the processes and the timeline cannot replay
(SURVEY §5.4).  Here named objects of every rank's namespace are saved with
``torch.distributed.checkpoint`` (DCP): each rank writes its own shard of the state in parallel
(288 GB of HBM per MI355X makes per-rank state large — no gather to rank 0), and loading works
in place into existing objects, so a session can be rebuilt after ``%dist_init``:

    %dist_checkpoint save /ckpt/step100 model opt step
    ... kernel restart / %dist_reset / %dist_init ...
    (re-create model/opt in a cell)
    %dist_checkpoint load /ckpt/step100 model opt step

Objects with ``state_dict()``/``load_state_dict()`` (modules, optimizers, LR schedulers, DDP
wrappers) go through their state dicts; tensors are saved directly; other picklable values are
stored per rank.

By default every rank's state is stored under its own keys (``rank{r}/name``), which is correct
whatever the ranks hold (DCP's default planner de-duplicates plain tensors across ranks on the
assumption that they are replicated).  ``replicated=True`` (``--replicated``) uses shared keys for
state that is identical on every rank (e.g. a DDP model), so DCP writes it once.
"""
from __future__ import annotations

import json
import os
import pickle
from typing import Any, Dict, List


def _is_stateful(obj: Any) -> bool:
    return hasattr(obj, "state_dict") and hasattr(obj, "load_state_dict")


def _key(n: str, rank: int, replicated: bool) -> str:
    return n if replicated else f"rank{rank}/{n}"


def save(ns: Dict[str, Any], names: List[str], path: str, replicated: bool = False) -> Dict[str, Any]:
    import torch
    import torch.distributed as dist
    import torch.distributed.checkpoint as dcp

    missing = [n for n in names if n not in ns]
    if missing:
        raise NameError(f"not defined on this rank: {missing}")
    rank = dist.get_rank() if dist.is_initialized() else 0
    state: Dict[str, Any] = {}
    plain: Dict[str, Any] = {}
    kinds: Dict[str, str] = {}
    for n in names:
        obj = ns[n]
        if _is_stateful(obj):
            state[_key(n, rank, replicated)] = obj.state_dict()
            kinds[n] = "stateful"
        elif isinstance(obj, torch.Tensor):
            state[_key(n, rank, replicated)] = obj
            kinds[n] = "tensor"
        else:
            plain[n] = obj
            kinds[n] = "object"
    os.makedirs(path, exist_ok=True)
    if state:
        dcp.save(state, checkpoint_id=os.path.join(path, "dcp"))
    with open(os.path.join(path, f"objects_rank{rank}.pkl"), "wb") as f:
        pickle.dump(plain, f)
    if rank == 0:
        with open(os.path.join(path, "manifest.json"), "w") as f:
            json.dump({"names": names, "kinds": kinds, "replicated": replicated,
                       "world_size": dist.get_world_size() if dist.is_initialized() else 1}, f)
    return {"rank": rank, "saved": names}


def load(ns: Dict[str, Any], names: List[str], path: str) -> Dict[str, Any]:
    import torch
    import torch.distributed as dist
    import torch.distributed.checkpoint as dcp

    rank = dist.get_rank() if dist.is_initialized() else 0
    with open(os.path.join(path, "manifest.json")) as f:
        manifest = json.load(f)
    kinds = manifest["kinds"]
    names = names or manifest["names"]
    replicated = manifest.get("replicated", False)
    world = dist.get_world_size() if dist.is_initialized() else 1
    if not replicated and manifest.get("world_size", world) != world:
        raise RuntimeError(f"checkpoint has per-rank state for {manifest['world_size']} ranks; this session has {world}")
    state: Dict[str, Any] = {}
    for n in names:
        k = kinds.get(n)
        if k is None:
            raise KeyError(f"{n!r} is not in checkpoint {path}")
        if k == "stateful":
            if n not in ns or not _is_stateful(ns[n]):
                raise NameError(f"create {n!r} (same type/shape) before loading its state")
            state[_key(n, rank, replicated)] = ns[n].state_dict()
        elif k == "tensor":
            if n not in ns or not isinstance(ns[n], torch.Tensor):
                raise NameError(f"create tensor {n!r} (same shape/dtype/device) before loading")
            state[_key(n, rank, replicated)] = ns[n]
    if state:
        dcp.load(state, checkpoint_id=os.path.join(path, "dcp"))
        for n in names:
            if kinds.get(n) == "stateful":
                ns[n].load_state_dict(state[_key(n, rank, replicated)])
    obj_file = os.path.join(path, f"objects_rank{rank}.pkl")
    if os.path.exists(obj_file):
        with open(obj_file, "rb") as f:
            plain = pickle.load(f)  # written by this framework for this rank
        for n in names:
            if kinds.get(n) == "object" and n in plain:
                ns[n] = plain[n]
    return {"rank": rank, "loaded": names}
