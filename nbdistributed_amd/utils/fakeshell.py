"""A minimal IPython-shaped shell for headless use (tests, benchmarks, scripts).

The PyTorch interpreter in this image has no IPython, but the magics should be exercised
exactly as a notebook would: input transformers (``input_transformers_cleanup``), cell-magic
dispatch on the first line (``%%name args``), line magics, and plain Python executed in the
kernel's own namespace.  ``HeadlessShell`` implements that subset of IPython's behaviour, so
``bench.py`` can time real ``%%distributed`` cells end to end and the tests can drive every
magic.  With a real IPython available, ``nbdistributed_amd`` registers against the real shell
instead (``magic.register``).
"""
from __future__ import annotations

import traceback
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional


class UsageError(Exception):
    pass


@dataclass
class ExecutionResult:
    error_in_exec: Optional[BaseException] = None
    result: Any = None

    @property
    def success(self) -> bool:
        return self.error_in_exec is None


class HeadlessShell:
    def __init__(self):
        self.user_ns: Dict[str, Any] = {}
        self.input_transformers_cleanup: List[Callable[[List[str]], List[str]]] = []
        self.line_magics: Dict[str, Callable] = {}
        self.cell_magics: Dict[str, Callable] = {}
        self.magics_obj = None

    def register_magic_function(self, fn, magic_kind="line", magic_name=None):
        name = magic_name or fn.__name__
        (self.line_magics if magic_kind == "line" else self.cell_magics)[name] = fn

    def load_extension(self, session: Any = None, writer: Any = None) -> Any:
        """``session``: drive an existing Session (bench.py's attached coordinator)."""
        from ..magic import MagicCore, _safe, CELL_MAGICS, LINE_MAGICS, rank_nospace_transform

        core = MagicCore(self, writer=writer, session=session)
        for n in LINE_MAGICS:
            self.register_magic_function(_safe(core, getattr(core, n)), "line", n)
        for n in CELL_MAGICS:
            self.register_magic_function(_safe(core, getattr(core, n)), "cell", n)
        self.input_transformers_cleanup.insert(0, rank_nospace_transform)
        self.core = core
        return core

    def transform(self, raw: str) -> str:
        lines = raw.splitlines(keepends=True)
        for t in list(self.input_transformers_cleanup):
            lines = t(lines)
        return "".join(lines)

    def run_cell(self, raw: str, raise_errors: bool = False) -> ExecutionResult:
        text = self.transform(raw)
        res = ExecutionResult()
        try:
            if text.startswith("%%"):
                first, _, body = text.partition("\n")
                name, _, args = first[2:].partition(" ")
                fn = self.cell_magics.get(name)
                if fn is None:
                    raise UsageError(f"Cell magic `%%{name}` not found.")
                res.result = fn(args, body)
            else:
                stripped = text.strip()
                if stripped.startswith("%") and "\n" not in stripped:
                    name, _, args = stripped[1:].partition(" ")
                    fn = self.line_magics.get(name)
                    if fn is None:
                        raise UsageError(f"Line magic function `%{name}` not found.")
                    res.result = fn(args)
                elif stripped:
                    exec(compile(text, "<headless-cell>", "exec"), self.user_ns)
        except BaseException as e:  # noqa: BLE001 - mirror IPython: the cell fails, the shell lives
            res.error_in_exec = e
            if raise_errors:
                raise
            render = getattr(e, "_render_traceback_", None)
            if render is not None:
                print("\n".join(render()))
            else:
                traceback.print_exc()
        return res

    def magic(self, line: str) -> Any:
        return self.run_cell("%" + line.lstrip("%")).result
