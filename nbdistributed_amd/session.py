"""Shell-agnostic coordinator: the object that owns one distributed notebook session.

The reference spreads this state over ``DistributedMagic`` class *and* instance attributes
(``magic.py:95-121``, ``:493-505``), which is why ``%dist_shutdown`` and extension unload never
stop the workers (D-1).  Here a single ``Session`` owns the launcher, the control plane, the
timeline and the rendering of per-rank output; the IPython magics (``magic.py``) are a thin
adapter over it, and everything is usable (and tested) without IPython.

Cell execution path (reference: ``magic.py:1042-1129`` — thread + 100 ms main-thread polling;
``:1476-1565`` for ``%%rank``):

    Session.execute(code, ranks)
      -> CommunicationManager.submit()        one native send per rank (no polling anywhere)
      -> consume request events in the calling thread, as they arrive:
           stream chunk  -> per-(rank, stream) line buffer -> "🔹 Rank r:" block rendering
           response      -> flush that rank's partial lines, print its echo
           rank death    -> reported immediately, cell fails fast with the others' results
      -> timeline record, namespace delta for IDE proxies, DistributedExecutionError if any rank
         failed (so notebooks see a failed cell: reference D-9).
"""
from __future__ import annotations

import os
import queue
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from . import protocol as P
from .communication import CommunicationManager, PendingRequest, RankDied, RequestTimeout
from .config import get_config
from .process_manager import ProcessManager, find_free_port
from .timeline import Timeline

Writer = Callable[[str], None]

# Library chatter printed outside any cell (worker bring-up) that carries no information for the
# notebook user.  Everything else from a worker is shown.
_NOISE = ("[Gloo] Rank ", "amdgpu.ids: No such file or directory")


def _is_noise(line: str) -> bool:
    return any(n in line for n in _NOISE)


def _default_writer(text: str) -> None:
    out = sys.stdout  # resolved per call: IPython swaps sys.stdout per cell
    out.write(text)
    try:
        out.flush()
    except Exception:
        pass


class DistributedExecutionError(RuntimeError):
    """Raised after a cell failed on at least one rank.  IPython renders it through
    ``_render_traceback_`` as per-rank error blocks instead of a coordinator traceback."""

    def __init__(self, result: "CellResult"):
        self.result = result
        bad = sorted(set(result.errors) | set(result.dead))
        super().__init__(f"cell failed on rank(s) {bad}")

    def _render_traceback_(self) -> List[str]:
        lines: List[str] = []
        for r in sorted(self.result.errors):
            e = self.result.errors[r]
            lines.append(f"❌ Rank {r}: {e.get('ename') or 'Error'}: {e.get('error')}")
            tb = e.get("traceback") or ""
            lines.extend("   " + l for l in tb.rstrip().splitlines())
        for r in sorted(self.result.dead):
            lines.append(f"💀 Rank {r}: {self.result.dead[r]}")
        return lines

    def __str__(self) -> str:
        return "\n".join([super().__str__()] + self._render_traceback_())


@dataclass
class CellResult:
    seq: int
    ranks: List[int]
    results: Dict[int, Any]
    errors: Dict[int, Dict[str, Any]] = field(default_factory=dict)
    dead: Dict[int, str] = field(default_factory=dict)
    duration_s: float = 0.0
    ns_delta: Optional[Dict[str, Any]] = None
    interrupted: bool = False

    @property
    def ok(self) -> bool:
        return not self.errors and not self.dead

    def output(self, rank: int) -> str:
        d = self.results.get(rank)
        return d.get("output", "") if isinstance(d, dict) else ""


class _Renderer:
    """Per-rank block rendering of live output (fixes reference D-8: lines attributed to the
    wrong rank after the first poll, one line per write() chunk)."""

    def __init__(self, write: Writer, show_header: bool = True):
        self.write = write
        self.show_header = show_header
        self.last_rank: Optional[int] = None
        self.partial: Dict[tuple, str] = {}
        self.bytes = 0

    def _emit(self, rank: int, lines: List[str]) -> None:
        if not lines:
            return
        chunks = []
        if self.show_header and rank != self.last_rank:
            chunks.append(f"🔹 Rank {rank}:\n")
        self.last_rank = rank
        chunks.extend(f"  {l}\n" for l in lines)
        text = "".join(chunks)
        self.bytes += len(text)
        self.write(text)

    def stream(self, rank: int, stream: str, text: str) -> None:
        key = (rank, stream)
        buf = self.partial.get(key, "") + text
        if "\n" not in buf:
            self.partial[key] = buf
            return
        head, _, tail = buf.rpartition("\n")
        self.partial[key] = tail
        self._emit(rank, head.split("\n"))

    def flush_rank(self, rank: int) -> None:
        for key in [k for k in self.partial if k[0] == rank]:
            t = self.partial.pop(key)
            if t:
                self._emit(rank, [t])

    def result(self, rank: int, text: str) -> None:
        self.flush_rank(rank)
        if text:
            self._emit(rank, text.split("\n"))

    def note(self, rank: int, text: str) -> None:
        self.flush_rank(rank)
        self._emit(rank, [text])


class Session:
    """One distributed session: N workers, their control plane and their timeline."""

    def __init__(self, writer: Optional[Writer] = None):
        self.cfg = get_config()
        self.write: Writer = writer or _default_writer
        self.pm: Optional[ProcessManager] = None
        self.comm: Optional[CommunicationManager] = None
        self.num_processes = 0
        self.world_size = 0
        self.ready: Dict[int, Dict[str, Any]] = {}
        self.timeline = Timeline(self.cfg.timeline_capacity)
        self.gpu_ids: Optional[List[Optional[int]]] = None
        self.default_timeout: Optional[float] = None
        # optional absolute deadline (time.monotonic()): no request waits past it (benchmarks
        # that must hand in their result before an outer time limit)
        self.deadline: Optional[float] = None
        self.attached = False
        self.started_at: Optional[float] = None
        self.init_s: Optional[float] = None
        self._native_lock = threading.Lock()
        self.last_cell: Optional[CellResult] = None
        # why the last start()/attach() failed: ranks connected to the control plane / READY
        self.start_failure: Optional[Dict[str, Any]] = None

    # ------------------------------------------------------------------ lifecycle
    @property
    def active(self) -> bool:
        return self.comm is not None

    def _native_output(self, rank: int, text: str, stream: str) -> None:
        """Worker output that bypassed the transport (before capture started, or crash reports
        written to the original stderr)."""
        with self._native_lock:
            lines = [l for l in text.rstrip("\n").split("\n") if not _is_noise(l)]
            if lines:
                self.write("".join(f"[rank {rank} {stream}] {l}\n" for l in lines))

    def _background_output(self, rank: int, text: str, stream: str) -> None:
        """Output from a worker that belongs to no request in flight (background threads)."""
        with self._native_lock:
            lines = [l for l in text.rstrip("\n").split("\n") if l and not _is_noise(l)]
            if lines:
                self.write("".join(f"[rank {rank}] {l}\n" for l in lines))

    def start(self, num_processes: int = 2, master_addr: str = "localhost", gpu_ids: Optional[List[int]] = None,
              timeout: Optional[float] = None, backend: str = "auto", python: Optional[str] = None,
              extra_env: Optional[Dict[str, str]] = None, startup_timeout: Optional[float] = None) -> Dict[int, Dict]:
        if self.active:
            raise RuntimeError("session already running; shut it down first")
        t0 = time.perf_counter()
        self.default_timeout = timeout
        comm = CommunicationManager(num_processes, output_callback=self._background_output, default_timeout=timeout)
        pm = ProcessManager(output_callback=self._native_output,
                            exit_callback=lambda r, c: comm.mark_dead(r, f"process exited (exit code {c})"))
        self.comm, self.pm = comm, pm
        self.num_processes = self.world_size = num_processes
        try:
            pm.start_workers(num_processes, master_addr, gpu_ids, comm_endpoint=comm.endpoint, token=comm.token,
                             backend=backend, python=python, extra_env=extra_env)
            self.gpu_ids = [w.gpu_id for w in pm.workers]
            self.ready = comm.wait_ready(list(range(num_processes)),
                                         startup_timeout if startup_timeout is not None else self.cfg.startup_timeout_s,
                                         alive=pm.dead_ranks)
        except BaseException as e:
            self._record_start_failure(comm, e)
            self.shutdown(graceful=False)
            raise
        self.started_at = time.time()
        self.init_s = time.perf_counter() - t0
        return self.ready

    def attach(self, world_size: int, bind: Optional[str] = None, token: Optional[str] = None,
               timeout: Optional[float] = None, startup_timeout: Optional[float] = None,
               on_endpoint: Optional[Callable[[str, Optional[str]], None]] = None) -> Dict[int, Dict]:
        """Coordinate workers launched elsewhere (torchrun / srun / other hosts): bind, publish
        the endpoint (``on_endpoint``), wait for ``world_size`` READY messages."""
        if self.active:
            raise RuntimeError("session already running; shut it down first")
        comm = CommunicationManager(world_size, output_callback=self._background_output, default_timeout=timeout,
                                    endpoint=bind or f"tcp://{self.cfg.bind_host}:0", token=token,
                                    use_token=token is not None)
        self.comm = comm
        self.num_processes = self.world_size = world_size
        self.attached = True
        self.default_timeout = timeout
        if on_endpoint is not None:
            on_endpoint(comm.endpoint, comm.token)
        try:
            self.ready = comm.wait_ready(list(range(world_size)), startup_timeout or self.cfg.startup_timeout_s)
        except BaseException as e:
            self._record_start_failure(comm, e)
            self.shutdown(graceful=False)
            raise
        self.gpu_ids = [self.ready[r].get("gpu_id") for r in range(world_size)]
        self.started_at = time.time()
        return self.ready

    def _record_start_failure(self, comm: CommunicationManager, e: BaseException) -> None:
        ready = [r for r, d in comm.ready.items() if isinstance(d, dict) and "error" not in d]
        self.start_failure = {"connected": len(set(comm.connected) | set(ready)), "ready": len(ready),
                              "world": self.world_size, "error": f"{type(e).__name__}: {e}"}

    def shutdown(self, graceful: bool = True, timeout: float = 5.0) -> None:
        comm, pm = self.comm, self.pm
        self.comm = None
        self.pm = None
        if comm is not None:
            comm.stopping = True
        if comm is not None and graceful:
            alive = [r for r in range(self.num_processes) if r not in comm.dead]
            if alive:
                try:
                    req = comm.submit(alive, "shutdown", None, live=False)
                    req.done.wait(timeout)
                    comm._forget(req)
                except Exception:
                    pass
        if pm is not None:
            if graceful:
                pm.wait_exit(timeout)
            pm.shutdown(grace=1.0 if graceful else 0.2)
        if comm is not None:
            comm.shutdown()
        self.num_processes = 0
        self.ready = {}

    def _require(self) -> CommunicationManager:
        if self.comm is None:
            raise RuntimeError("No distributed workers running. Use %dist_init first.")
        return self.comm

    def _effective_timeout(self, timeout: Optional[float]) -> Optional[float]:
        t = timeout if timeout is not None else self.default_timeout
        if self.deadline is not None:
            left = max(0.0, self.deadline - time.monotonic())
            t = left if t is None else min(t, left)
        return t

    def all_ranks(self) -> List[int]:
        return list(range(self.num_processes))

    # ------------------------------------------------------------------ execution
    def execute(self, code: str, ranks: Optional[List[int]] = None, *, render: bool = True, echo: bool = True,
                ns_delta: bool = False, timeout: Optional[float] = None, kind: str = "distributed",
                raise_on_error: bool = True, show_header: bool = True) -> CellResult:
        comm = self._require()
        timeout = self._effective_timeout(timeout)
        ranks = self.all_ranks() if ranks is None else list(ranks)
        flags = (P.F_NS_DELTA if ns_delta and 0 in ranks else 0) | (0 if echo else P.F_NO_ECHO)
        t0 = time.perf_counter()
        payload: Any = code if len(ranks) == self.num_processes else {"code": code, "ranks": list(ranks)}
        req = comm.submit(ranks, "execute", payload, flags=flags, live=render)
        rec = self.timeline.start(req.seq, kind, ranks, code)
        renderer = _Renderer(self.write, show_header=show_header) if render else None
        interrupted = False
        try:
            if renderer is not None:
                self._consume(req, renderer, timeout)
            else:
                comm.wait(req, timeout if timeout is not None else self.default_timeout)
        except KeyboardInterrupt:
            # forward the interrupt to the workers and collect what they say
            interrupted = True
            comm.interrupt(ranks)
            try:
                if renderer is not None:
                    self._consume(req, renderer, timeout=self.cfg.interrupt_abort_s + 15.0)
                else:
                    comm.wait(req, self.cfg.interrupt_abort_s + 15.0)
            except (RequestTimeout, KeyboardInterrupt):
                pass
        except RequestTimeout:
            comm._forget(req)
            dur = time.perf_counter() - t0
            self.timeline.end(rec, req.results(), dur, "timeout")
            raise
        finally:
            comm._forget(req)
        dur = time.perf_counter() - t0
        results = req.results()
        errors = {r: d for r, d in results.items()
                  if isinstance(d, dict) and not d.get("dead") and (req.errors.get(r) or d.get("status") in ("error", "interrupted") or "error" in d)}
        delta = None
        if 0 in results and isinstance(results[0], dict):
            delta = results[0].get("ns_delta")
        res = CellResult(seq=req.seq, ranks=ranks, results=results, errors=errors, dead=dict(req.dead),
                         duration_s=dur, ns_delta=delta, interrupted=interrupted)
        status = "ok" if res.ok else ("interrupted" if interrupted else ("dead" if res.dead else "error"))
        self.timeline.end(rec, results, dur, status, renderer.bytes if renderer else 0)
        self.last_cell = res
        if raise_on_error and not res.ok:
            raise DistributedExecutionError(res)
        return res

    def _consume(self, req: PendingRequest, renderer: _Renderer, timeout: Optional[float]) -> None:
        deadline = None if timeout is None and self.default_timeout is None else \
            time.monotonic() + (timeout if timeout is not None else self.default_timeout)
        events = req.events
        while True:
            wait = 0.5 if deadline is None else max(0.0, min(0.5, deadline - time.monotonic()))
            try:
                # drain the socket from this thread until an event is queued (no hand-off from the
                # receive thread); another thread leading already -> block on the queue as before
                if self.comm.pump(lambda: not events.empty(), wait) is None:
                    ev = events.get(timeout=wait)
                else:
                    ev = events.get_nowait()
            except queue.Empty:
                if deadline is not None and time.monotonic() >= deadline:
                    missing = [r for r in req.ranks if r not in req.responses and r not in req.dead]
                    raise RequestTimeout(f"no reply from ranks {missing}", req.results())
                continue
            kind = ev[0]
            if kind == "stream":
                _, rank, stream, text = ev
                renderer.stream(rank, stream, text)
            elif kind == "response":
                rank = ev[1]
                d = req.responses.get(rank)
                echo = d.get("output", "") if isinstance(d, dict) else ""
                renderer.result(rank, echo)
            elif kind == "dead":
                renderer.note(ev[1], f"💀 rank {ev[1]} died: {ev[2]}")
            elif kind == "done":
                for r in req.ranks:
                    renderer.flush_rank(r)
                return

    # ------------------------------------------------------------------ other requests
    def sync(self, timeout: Optional[float] = None) -> Dict[int, Any]:
        comm = self._require()
        return comm.send_to_ranks(self.alive_ranks(), "sync", {}, timeout=self._effective_timeout(timeout))

    def alive_ranks(self) -> List[int]:
        comm = self._require()
        return [r for r in self.all_ranks() if r not in comm.dead]

    def status(self, timeout: float = 5.0) -> Dict[int, Dict[str, Any]]:
        comm = self._require()
        if self.pm is not None:
            st = self.pm.get_detailed_status(comm, timeout=timeout)
        else:  # attach mode: no local processes
            st = {r: {"pid": self.ready.get(r, {}).get("pid"), "running": r not in comm.dead, "returncode": None,
                      "gpu_id": self.ready.get(r, {}).get("gpu_id")} for r in self.all_ranks()}
            alive = [r for r in self.all_ranks() if r not in comm.dead]
            res = comm.send_to_ranks(alive, "get_status", {}, timeout=timeout)
            for r, d in res.items():
                if isinstance(d, dict) and "error" not in d:
                    st[r].update(d)
        for r, d in st.items():
            if r in comm.dead:
                d["dead_reason"] = comm.dead[r]
            if isinstance(d.get("gpu_ms"), dict):
                self.timeline.attach_gpu(r, d["gpu_ms"])
        return st

    def get_var(self, name: str, rank: int = 0, summary: bool = False, timeout: Optional[float] = None) -> Any:
        comm = self._require()
        res = comm.send_to_ranks([rank], "get_var", {"name": name, "summary": summary}, timeout=timeout)[rank]
        if isinstance(res, dict) and res.get("dead"):
            raise RankDied(rank, res["error"])
        return res

    def set_var(self, name: str, value: Any, ranks: Optional[List[int]] = None, to_device: bool = True,
                timeout: Optional[float] = None) -> Dict[int, Any]:
        comm = self._require()
        ranks = self.all_ranks() if ranks is None else ranks
        return comm.send_to_ranks(ranks, "set_var", {"name": name, "value": value, "to_device": to_device}, timeout=timeout)

    def namespace_info(self, rank: int = 0, timeout: Optional[float] = 30.0) -> Dict[str, Any]:
        comm = self._require()
        return comm.send_to_ranks([rank], "get_namespace_info", "", timeout=timeout)[rank]

    def interrupt(self, ranks: Optional[List[int]] = None, hard: bool = False, kill: bool = False) -> None:
        """Interrupt running cells.  Default: out-of-band message (SIGINT raised natively in the
        worker).  ``hard``: SIGINT straight to the processes.  ``kill``: SIGKILL the ranks (last
        resort for a rank blocked inside a non-abortable collective); the session becomes
        degraded and ``%dist_init`` replaces it."""
        comm = self._require()
        if kill and self.pm is not None:
            import signal as _signal

            for w in self.pm.workers:
                if (ranks is None or w.rank in ranks) and w.running:
                    try:
                        os.killpg(w.pid, _signal.SIGKILL)
                    except ProcessLookupError:
                        pass
        elif hard and self.pm is not None:
            self.pm.interrupt(ranks)
        else:
            comm.interrupt(ranks)

    def recover(self, timeout: float = 120.0) -> Dict[int, Any]:
        """Rebuild the process group on all ranks (after a communicator abort)."""
        comm = self._require()
        addr = self.pm.master_addr if self.pm is not None else "127.0.0.1"
        port = find_free_port(addr)
        return comm.send_to_ranks(self.alive_ranks(), "recover", {"master_port": port, "master_addr": addr},
                                  timeout=timeout)

    def profile(self, action: str, path_template: Optional[str] = None, timeout: float = 120.0, **kw) -> Dict[int, Any]:
        comm = self._require()
        data: Dict[str, Any] = {"action": action}
        if path_template:
            data["path_template"] = path_template
        data.update(kw)
        return comm.send_to_ranks(self.alive_ranks(), "profile", data, timeout=timeout)

    def call(self, name: str, args: Optional[Dict[str, Any]] = None, ranks: Optional[List[int]] = None,
             timeout: float = 30.0) -> Dict[int, Any]:
        """Invoke the worker-side call handler ``name`` (``DistributedWorker.calls``) on ``ranks``
        (default: every live rank)."""
        comm = self._require()
        return comm.send_to_ranks(ranks or self.alive_ranks(), "call", {"name": name, "args": args or {}},
                                  timeout=timeout)

    def fault(self, action: str = "arm", spec: str = "", timeout: float = 30.0) -> Dict[int, Any]:
        """Arm (``spec`` in the faults.py grammar), clear or list injected faults on every live rank."""
        from . import faults

        if action == "arm":
            faults.parse(spec)  # validate here: a bad spec fails in the notebook, not on the ranks
        return self.call("fault", {"action": action, "spec": spec}, timeout=timeout)

    def ping(self, timeout: float = 5.0) -> Dict[int, float]:
        """Control-plane round trip per rank (seconds)."""
        comm = self._require()
        t0 = time.perf_counter()
        req = comm.submit(self.alive_ranks(), "ping", None, live=False)
        comm.wait(req, timeout)
        return {r: t - t0 for r, t in ((r, req.t_first_reply.get(r, t0)) for r in req.ranks)}
