"""Fault injection for the failure-handling paths (SURVEY.md §5.3 "Fault injection: an env/magic
hook (crash / hang / stderr-flood at rank r) used by tests").

The reference has no fault injection and none of the recovery machinery it would exercise
(`process_manager.py:136-150` checks for dead workers once, after a 2 s sleep; a rank dying
mid-cell makes `communication.py:255-262` wait for the full timeout).  Here every failure path —
fail-fast on rank death, interrupt of a hung cell, stderr back-pressure, the subset-collective
guard — can be triggered deterministically, from the environment of the workers
(``NBD_FAULTS``) or at run time from the notebook (``%dist_fault``).

Spec grammar (several specs separated by ``;``)::

    kind[:arg][@ranks][#cell]

* ``kind``   — ``crash`` (``os._exit(arg or 77)``: no cleanup, like a segfault), ``abort``
  (SIGABRT), ``hang`` (block for ``arg`` seconds, forever if absent; interruptible with
  ``%dist_interrupt``), ``delay`` (sleep ``arg`` seconds, then run the cell), ``raise`` (the cell
  fails with :class:`InjectedFault`), ``flood`` (write ``arg`` KiB, default 256, to stderr
  before the cell runs).
* ``ranks``  — ``1``, ``0,2`` or ``0-3`` (default: every rank).
* ``cell``   — fire before the N-th cell executed after arming (1-based, default 1).

Each fault fires once.  Example: ``NBD_FAULTS="crash:7@1#3"`` kills rank 1 with exit code 7
as its third cell starts.
"""
from __future__ import annotations

import os
import signal
import sys
import time
from dataclasses import dataclass
from typing import List, Optional, Set

KINDS = ("crash", "abort", "hang", "delay", "raise", "flood")


class InjectedFault(RuntimeError):
    """Raised in a cell by a ``raise`` fault."""


@dataclass
class Fault:
    kind: str
    arg: Optional[float] = None
    ranks: Optional[Set[int]] = None  # None = every rank
    cell: int = 1

    def spec(self) -> str:
        s = self.kind
        if self.arg is not None:
            s += f":{self.arg:g}"
        if self.ranks is not None:
            s += "@" + ",".join(str(r) for r in sorted(self.ranks))
        if self.cell != 1:
            s += f"#{self.cell}"
        return s


def _parse_ranks(text: str) -> Set[int]:
    out: Set[int] = set()
    for part in text.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return out


def parse(spec: Optional[str]) -> List[Fault]:
    """Parse ``kind[:arg][@ranks][#cell]`` specs joined by ``;`` (see the module docstring)."""
    faults: List[Fault] = []
    for item in (spec or "").split(";"):
        item = item.strip()
        if not item:
            continue
        cell = 1
        if "#" in item:
            item, c = item.rsplit("#", 1)
            cell = int(c)
            if cell < 1:
                raise ValueError(f"fault cell index must be >= 1: {c!r}")
        ranks = None
        if "@" in item:
            item, r = item.split("@", 1)
            ranks = _parse_ranks(r)
        arg = None
        if ":" in item:
            item, a = item.split(":", 1)
            arg = float(a)
        kind = item.strip().lower()
        if kind not in KINDS:
            raise ValueError(f"unknown fault kind {kind!r} (one of {', '.join(KINDS)})")
        faults.append(Fault(kind, arg, ranks, cell))
    return faults


class FaultPlan:
    """The faults armed on one worker; :meth:`before_cell` runs at the start of every cell."""

    def __init__(self, rank: int, faults: Optional[List[Fault]] = None):
        self.rank = rank
        self.pending: List[List] = []  # [fault, cells still to go]
        self.fired: List[str] = []
        for f in faults or []:
            self.arm(f)

    def arm(self, f: Fault) -> bool:
        if f.ranks is not None and self.rank not in f.ranks:
            return False
        self.pending.append([f, f.cell])
        return True

    def clear(self) -> int:
        n = len(self.pending)
        self.pending.clear()
        return n

    def armed(self) -> List[str]:
        return [f"{f.spec()} (in {left} cell{'s' if left != 1 else ''})" for f, left in self.pending]

    def before_cell(self) -> None:
        due = []
        for entry in self.pending:
            entry[1] -= 1
            if entry[1] <= 0:
                due.append(entry)
        for entry in due:
            self.pending.remove(entry)
        for f, _ in due:
            self.fired.append(f.spec())
            _fire(f)


def _fire(f: Fault) -> None:
    if f.kind == "crash":
        try:
            sys.stdout.flush()
            sys.stderr.flush()
        except Exception:
            pass
        os._exit(int(f.arg) if f.arg is not None else 77)
    if f.kind == "abort":
        os.kill(os.getpid(), signal.SIGABRT)
        time.sleep(5)  # the signal is delivered asynchronously
        os._exit(134)
    if f.kind in ("hang", "delay"):
        end = None if f.arg is None else time.monotonic() + f.arg
        if f.kind == "delay" and end is None:
            end = time.monotonic() + 1.0
        while end is None or time.monotonic() < end:
            time.sleep(0.02)  # short sleeps: SIGINT (interrupt) lands promptly
        return
    if f.kind == "raise":
        raise InjectedFault(f"injected fault ({f.spec()})")
    if f.kind == "flood":
        kib = int(f.arg) if f.arg is not None else 256
        line = memoryview(("x" * 1023 + "\n").encode())
        for _ in range(kib):
            done = 0
            while done < len(line):
                done += os.write(2, line[done:])
        return
