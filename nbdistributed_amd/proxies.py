"""Local stand-ins for rank-0 objects, so the notebook's completer/inspector "see" worker state.

Reference (``magic.py:1158-1314``): overwrites ``user_ns`` unconditionally with placeholders —
full-size ``torch.zeros`` allocated on the kernel's CPU for every tensor, ``[]``/``0``/``""`` for
builtins (so ``t = [1, 2, 3]`` reads back as ``[]``), functions generated with ``exec``.

Here (D-14):
* tensors become ``device='meta'`` tensors when torch is already loaded in the kernel (right
  shape/dtype/methods for completion, zero bytes), else a light ``RemoteTensor`` record;
* small immutable builtins arrive with their real value;
* callables are stubs carrying the remote ``inspect.Signature`` (as ``__signature__``) and
  docstring, raising ``RemoteOnlyError`` when called locally;
* a name the user defined locally is never overwritten: only names that are absent or that
  hold a proxy we created are (re)written, and proxies of names deleted on rank 0 are removed.
"""
from __future__ import annotations

import inspect
import sys
import types
from typing import Any, Dict, Optional


class RemoteOnlyError(RuntimeError):
    pass


class _RemoteBase:
    _nbd_proxy = True

    def __init__(self, info: Dict[str, Any]):
        self._nbd_info = info

    def __repr__(self) -> str:
        i = self._nbd_info
        return f"<remote {i.get('type')} '{i.get('name')}' on rank 0: {i.get('repr', '')}>"


class RemoteTensor(_RemoteBase):
    def __init__(self, info):
        super().__init__(info)
        self.shape = tuple(info.get("shape", ()))
        self.dtype = info.get("dtype")
        self.device = info.get("device")
        self.requires_grad = info.get("requires_grad", False)

    def size(self, dim: Optional[int] = None):
        return self.shape if dim is None else self.shape[dim]

    def dim(self) -> int:
        return len(self.shape)

    def __repr__(self) -> str:
        return f"<remote tensor shape={list(self.shape)} dtype={self.dtype} device={self.device} (rank 0)>"


class RemoteObject(_RemoteBase):
    pass


class RemoteModule(_RemoteBase):
    def __repr__(self) -> str:
        i = self._nbd_info
        return f"<remote nn.Module {i.get('class_name')} ({i.get('n_params')} params) on rank 0>"


def _callable_stub(info: Dict[str, Any]):
    name = info.get("name", "remote_fn")

    def stub(*args, **kwargs):
        raise RemoteOnlyError(f"{name} is defined on the workers; run it in a %%distributed cell")

    stub.__name__ = name
    stub.__qualname__ = info.get("qualname", name)
    stub.__doc__ = info.get("doc") or f"Remote callable {name}{info.get('signature', '')} (defined on rank 0)."
    sig = _parse_signature(info.get("signature", "(*args, **kwargs)"))
    if sig is not None:
        stub.__signature__ = sig
    stub._nbd_proxy = True
    stub._nbd_info = info
    return stub


def _parse_signature(text: str) -> Optional[inspect.Signature]:
    """Rebuild a Signature from its text without evaluating defaults or annotations."""
    import ast

    try:
        fn = ast.parse(f"def _f{text}: pass").body[0]
    except SyntaxError:
        return None
    a = fn.args
    params = []
    P = inspect.Parameter
    pos = list(a.posonlyargs) + list(a.args)
    defaults = [None] * (len(pos) - len(a.defaults)) + list(a.defaults)
    for i, arg in enumerate(pos):
        kind = P.POSITIONAL_ONLY if i < len(a.posonlyargs) else P.POSITIONAL_OR_KEYWORD
        d = defaults[i]
        params.append(P(arg.arg, kind, default=P.empty if d is None else _Src(ast.unparse(d))))
    if a.vararg:
        params.append(P(a.vararg.arg, P.VAR_POSITIONAL))
    for arg, d in zip(a.kwonlyargs, a.kw_defaults):
        params.append(P(arg.arg, P.KEYWORD_ONLY, default=P.empty if d is None else _Src(ast.unparse(d))))
    if a.kwarg:
        params.append(P(a.kwarg.arg, P.VAR_KEYWORD))
    try:
        return inspect.Signature(params)
    except ValueError:
        return None


class _Src:
    """A default value shown by its source text."""

    def __init__(self, src: str):
        self.src = src

    def __repr__(self) -> str:
        return self.src


def make_proxy(info: Dict[str, Any]) -> Any:
    kind = info.get("kind")
    if kind == "tensor":
        torch = sys.modules.get("torch")
        if torch is not None:
            try:
                dtype = getattr(torch, str(info.get("dtype", "torch.float32")).replace("torch.", ""))
                t = torch.empty(info.get("shape", ()), dtype=dtype, device="meta")
                return t
            except Exception:
                pass
        return RemoteTensor(info)
    if kind == "device":
        torch = sys.modules.get("torch")
        if torch is not None:
            try:
                return torch.device(info["device_type"], info.get("index"))
            except Exception:
                pass
        return RemoteObject(info)
    if kind == "module":
        mod = sys.modules.get(info.get("module_name", ""))
        if mod is not None:
            return mod
        m = types.ModuleType(info.get("module_name", info.get("name", "remote")))
        m.__doc__ = f"Module imported on the workers ({info.get('file')}); not imported in the kernel."
        m._nbd_proxy = True
        return m
    if kind == "builtin" and "value" in info:
        return info["value"]
    if kind == "callable":
        return _callable_stub(info)
    if kind == "class":
        cls = type(info.get("class_name", "RemoteClass"), (_RemoteBase,), {"__doc__": info.get("doc") or ""})
        cls._nbd_proxy = True
        return cls
    if kind == "nn_module":
        return RemoteModule(info)
    return RemoteObject(info)


class ProxyTable:
    """Applies namespace deltas to a shell namespace without clobbering local definitions."""

    def __init__(self):
        self.owned: Dict[str, int] = {}  # name -> id(proxy) we wrote

    def _ours(self, ns: Dict[str, Any], name: str) -> bool:
        return name in self.owned and name in ns and id(ns[name]) == self.owned[name]

    def apply(self, ns: Dict[str, Any], delta: Dict[str, Any]) -> int:
        n = 0
        for info in delta.get("changed", []):
            name = info.get("name")
            if not name:
                continue
            if name in ns and not self._ours(ns, name):
                continue  # user-defined locally: never overwrite
            try:
                obj = make_proxy(info)
            except Exception:
                continue
            ns[name] = obj
            self.owned[name] = id(obj)
            n += 1
        for name in delta.get("removed", []):
            if self._ours(ns, name):
                del ns[name]
            self.owned.pop(name, None)
        return n

    def clear(self, ns: Dict[str, Any]) -> None:
        for name in list(self.owned):
            if self._ours(ns, name):
                del ns[name]
        self.owned.clear()
