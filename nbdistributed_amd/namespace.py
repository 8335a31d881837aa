"""Worker-namespace introspection for the coordinator's "IDE support".

Reference behaviour: after every ``%%distributed`` cell the coordinator asks rank 0 for a full
description of its namespace (``worker.py:426-485``, ``magic.py:1131-1156``) — one extra round
trip per cell, with ``repr`` of every object computed twice — and then overwrites the kernel's
``user_ns`` with placeholders, including full-size CPU ``torch.zeros`` for every tensor
(``magic.py:1188-1195``).

Here rank 0 keeps a fingerprint of its namespace and returns only the *delta* (changed and
removed names) piggy-backed on its execute response, so the sync costs no extra round trip and
O(changed names) work.  Descriptions are plain dicts (picklable without torch) and tensors are
described by shape/dtype/device only; the coordinator turns them into meta-device tensors or
light proxies (``proxies.py``).
"""
from __future__ import annotations

import inspect
import sys
import types
from typing import Any, Dict, List, Optional, Tuple

REPR_LIMIT = 200
_HIDDEN = {"In", "Out", "exit", "quit", "get_ipython"}


def _is_public(name: str) -> bool:
    return not name.startswith("_") and name not in _HIDDEN


def _safe_repr(obj: Any, limit: int = REPR_LIMIT) -> str:
    try:
        r = repr(obj)
    except Exception as e:  # a user object whose __repr__ raises
        r = f"<{type(obj).__name__} (repr failed: {type(e).__name__})>"
    return r if len(r) <= limit else r[: limit - 3] + "..."


def describe(name: str, obj: Any) -> Dict[str, Any]:
    """Picklable description of one namespace entry."""
    t = type(obj)
    info: Dict[str, Any] = {"name": name, "type": t.__name__, "module": getattr(t, "__module__", "")}
    torch = sys.modules.get("torch")
    if torch is not None and isinstance(obj, torch.Tensor):
        info.update(kind="tensor", shape=tuple(obj.shape), dtype=str(obj.dtype), device=str(obj.device),
                    requires_grad=bool(obj.requires_grad))
        return info
    if torch is not None and isinstance(obj, torch.device):
        info.update(kind="device", device_type=obj.type, index=obj.index)
        return info
    if isinstance(obj, types.ModuleType):
        info.update(kind="module", module_name=obj.__name__, file=getattr(obj, "__file__", None))
        return info
    if torch is not None and isinstance(obj, torch.nn.Module):
        try:
            n_params = sum(p.numel() for p in obj.parameters())
        except Exception:
            n_params = None
        info.update(kind="nn_module", class_name=t.__name__, n_params=n_params, repr=_safe_repr(obj, 400))
        return info
    if isinstance(obj, type):
        info.update(kind="class", class_name=obj.__name__, doc=(inspect.getdoc(obj) or "")[:500])
        return info
    if callable(obj):
        try:
            sig = str(inspect.signature(obj))
        except (TypeError, ValueError):
            sig = "(*args, **kwargs)"
        info.update(kind="callable", signature=sig, doc=(inspect.getdoc(obj) or "")[:500],
                    qualname=getattr(obj, "__qualname__", name))
        return info
    if isinstance(obj, (bool, int, float, complex, str, bytes)) or obj is None:
        info.update(kind="builtin", repr=_safe_repr(obj))
        if not isinstance(obj, (str, bytes)) or len(obj) <= 1024:
            info["value"] = obj  # small immutable values travel as-is: local reads are exact
        return info
    if isinstance(obj, (list, tuple, dict, set, frozenset)):
        info.update(kind="container", length=len(obj), repr=_safe_repr(obj))
        return info
    info.update(kind="object", class_name=t.__name__, repr=_safe_repr(obj))
    return info


def _fingerprint(obj: Any) -> Tuple:
    torch = sys.modules.get("torch")
    if torch is not None and isinstance(obj, torch.Tensor):
        return (id(obj), "T", tuple(obj.shape), obj.dtype, obj.device)
    if isinstance(obj, (bool, int, float, complex, str, bytes)) or obj is None:
        return (type(obj), obj if not isinstance(obj, (str, bytes)) or len(obj) < 256 else hash(obj))
    if isinstance(obj, (list, dict, set)):
        return (id(obj), type(obj), len(obj))
    return (id(obj), type(obj))


class NamespaceTracker:
    """Tracks a namespace and produces deltas of public names."""

    def __init__(self) -> None:
        self._prints: Dict[str, Tuple] = {}

    def full(self, ns: Dict[str, Any]) -> Dict[str, Any]:
        self._prints = {}
        return self.delta(ns, full=True)

    def delta(self, ns: Dict[str, Any], full: bool = False) -> Dict[str, Any]:
        changed: List[Dict[str, Any]] = []
        seen = set()
        for name, obj in list(ns.items()):
            if not _is_public(name):
                continue
            seen.add(name)
            try:
                fp = _fingerprint(obj)
            except Exception:
                fp = (id(obj),)
            if not full and self._prints.get(name) == fp:
                continue
            self._prints[name] = fp
            try:
                changed.append(describe(name, obj))
            except Exception as e:
                changed.append({"name": name, "type": type(obj).__name__, "kind": "object",
                                "repr": f"<describe failed: {e}>"})
        removed = [n for n in self._prints if n not in seen]
        for n in removed:
            del self._prints[n]
        return {"changed": changed, "removed": removed, "full": full}


def namespace_info(ns: Dict[str, Any]) -> Dict[str, Dict[str, Any]]:
    """Full description, keyed by name (reference-compatible ``get_namespace_info`` result)."""
    return {n: describe(n, o) for n, o in list(ns.items()) if _is_public(n)}
