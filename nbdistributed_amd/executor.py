"""The worker's REPL engine: run one notebook cell in a persistent namespace.

Reference: ``worker.py:248-387``.  Behavioural differences:

* D-22: the reference first tries ``ast.parse(mode='eval')`` inside a ``try`` and falls back on
  ``SyntaxError``, which chains a spurious SyntaxError into every traceback; tracebacks also
  carry the worker's own frames and no source lines (filename ``'<string>'``).  Here the cell is
  parsed once, split into body + trailing expression, compiled under a unique filename that is
  registered in ``linecache``, and tracebacks are trimmed to user frames — they read like
  IPython's.
* D-19: the namespace is a real module registered as ``sys.modules['__main__']`` so functions
  and classes defined in cells are picklable (the reference's bare dict gives them
  ``__name__ == 'builtins'``).
* Top-level ``await`` works (``PyCF_ALLOW_TOP_LEVEL_AWAIT``), as in IPython.
* The last expression is stored in ``_`` (plus ``__``/``___``) like the IPython REPL.
"""
from __future__ import annotations

import ast
import asyncio
import linecache
import sys
import time
import traceback
import types
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

_TOP_LEVEL_AWAIT = getattr(ast, "PyCF_ALLOW_TOP_LEVEL_AWAIT", 0)
_THIS_FILE = __file__
_COMPILED_CACHE = 256  # compiled cells kept for re-runs


@dataclass
class ExecResult:
    status: str  # "ok" | "error" | "interrupted"
    value: Any = None
    has_value: bool = False
    error: Optional[str] = None
    ename: Optional[str] = None
    traceback: Optional[str] = None
    exec_s: float = 0.0
    t_start: float = 0.0
    t_end: float = 0.0
    filename: str = ""
    extra: Dict[str, Any] = field(default_factory=dict)


def make_namespace_module(name: str = "__main__") -> types.ModuleType:
    mod = types.ModuleType(name)
    mod.__dict__["__builtins__"] = __builtins__
    return mod


class CellExecutor:
    def __init__(self, module: Optional[types.ModuleType] = None, tag: str = "cell",
                 install_as_main: bool = True):
        self.module = module or make_namespace_module()
        self.ns: Dict[str, Any] = self.module.__dict__
        self.tag = tag
        self.count = 0
        self._compiled: "OrderedDict[tuple, tuple]" = OrderedDict()  # (source, echo) -> (filename, body, expr)
        if install_as_main:
            sys.modules["__main__"] = self.module

    def _register_source(self, code: str) -> str:
        self.count += 1
        filename = f"<{self.tag}-{self.count}>"
        lines = code.splitlines(keepends=True)
        if lines and not lines[-1].endswith("\n"):
            lines[-1] += "\n"
        linecache.cache[filename] = (len(code), None, lines, filename)
        return filename

    def _format_exc(self, etype, evalue, tb) -> str:
        # Drop the leading frames that belong to this engine so the traceback starts in the cell.
        while tb is not None and tb.tb_frame.f_code.co_filename == _THIS_FILE:
            tb = tb.tb_next
        return "".join(traceback.format_exception(etype, evalue, tb, chain=True))

    def _run_code(self, code_obj) -> Any:
        if code_obj.co_flags & 0x80:  # CO_COROUTINE: cell used top-level await
            coro = eval(code_obj, self.ns)
            return _run_coroutine(coro)
        return eval(code_obj, self.ns)

    def run(self, code: str, echo: bool = True, pre=None) -> ExecResult:
        """Execute one cell.  ``pre`` (optional callable) runs first, inside the same error
        handling as the cell (used by fault injection: an injected hang is interruptible and an
        injected exception is reported like the cell's own)."""
        t0 = time.time()
        p0 = time.perf_counter()
        # a re-run cell (same source, same echo mode) reuses its compiled code and its filename
        # (whose source is still registered): no parse / compile on the round trip
        hit = self._compiled.get((code, echo))
        if hit is not None:
            self._compiled.move_to_end((code, echo))
            filename = hit[0]
        else:
            filename = self._register_source(code)
        res = ExecResult(status="ok", t_start=t0, filename=filename)
        try:
            if pre is not None:
                pre()
            if hit is not None:
                _, body, expr = hit
            else:
                try:
                    tree = ast.parse(code, filename=filename, mode="exec")
                except SyntaxError as e:
                    res.status = "error"
                    res.ename = type(e).__name__
                    res.error = str(e)
                    res.traceback = "".join(traceback.format_exception_only(type(e), e))
                    return res
                last = body = expr = None
                if echo and tree.body and isinstance(tree.body[-1], ast.Expr):
                    last = tree.body.pop()
                if tree.body:
                    body = compile(tree, filename, "exec", flags=_TOP_LEVEL_AWAIT, dont_inherit=True)
                if last is not None:
                    expr = compile(ast.Expression(last.value), filename, "eval", flags=_TOP_LEVEL_AWAIT,
                                   dont_inherit=True)
                self._compiled[(code, echo)] = (filename, body, expr)
                if len(self._compiled) > _COMPILED_CACHE:
                    self._compiled.popitem(last=False)
            if body is not None:
                self._run_code(body)
            if expr is not None:
                value = self._run_code(expr)
                if value is not None:
                    res.value = value
                    res.has_value = True
                    self.ns["___"] = self.ns.get("__")
                    self.ns["__"] = self.ns.get("_")
                    self.ns["_"] = value
        except KeyboardInterrupt:
            res.status = "interrupted"
            res.ename = "KeyboardInterrupt"
            res.error = "interrupted"
            res.traceback = self._format_exc(*sys.exc_info())
        except SystemExit as e:
            # A cell calling sys.exit()/exit() must not kill the worker; report it like an error.
            res.status = "error"
            res.ename = "SystemExit"
            res.error = f"SystemExit({e.code!r}) raised in cell (worker kept alive)"
            res.traceback = self._format_exc(*sys.exc_info())
        except BaseException as e:  # noqa: BLE001 - everything from user code is reported
            res.status = "error"
            res.ename = type(e).__name__
            res.error = str(e)
            res.traceback = self._format_exc(*sys.exc_info())
        finally:
            res.exec_s = time.perf_counter() - p0
            res.t_end = time.time()
        return res


def _run_coroutine(coro):
    try:
        loop = asyncio.get_event_loop()
    except RuntimeError:
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
    if loop.is_closed():
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
    return loop.run_until_complete(coro)
