"""Coordinator side of the control plane.

Reference: ``src/nbdistributed/communication.py`` — a pyzmq ROUTER bound on ``tcp://*``
(:121-125), a background thread that polls every 100 ms (:168-202), an ``Event`` that only ever
fires for ``send_to_all`` (:193-197), a 10 ms sleep-poll for subset requests (:348-370),
timeouts that leak table entries and drop partial results (:262, :359).

Re-design:

* native ROUTER (``transport``), bound to a private Unix socket (or loopback/explicit TCP for
  attach mode) with a per-session token (D-17);
* one receive thread blocked in native ``recv`` (no polling); every request — all ranks or a
  subset — completes through the same lock-protected table of ``PendingRequest`` objects whose
  completion and live events (stream chunks, responses, deaths) are pushed the instant they
  arrive (D-4);
* leader/follower receive: a thread that waits for a request (``wait`` / ``pump``) parks the
  receive thread and drains the socket itself, so a reply costs no thread hand-off (receive
  thread -> Event -> waiter: ≈15-30 us per cell, ``benchmarks/transport_pingpong.py``); the
  receive thread takes over again as soon as nobody waits.  Both ends poll for up to
  ``Config.spin_us`` before sleeping (native ``NBD_OPT_RECV_SPIN_US`` / ``NBD_OPT_IO_SPIN_US``);
* fail-fast: a rank that dies (process exit reported by the launcher, socket EOF, or heartbeat
  timeout) resolves every request waiting on it with a ``dead`` entry, keeping the other ranks'
  results (D-18); a send to a disconnected rank fails immediately (ROUTER_MANDATORY);
* streamed output is decoded incrementally per (rank, stream) and routed by request id; output
  that arrives outside a request (background threads) goes to ``output_callback``.

The reference's programmatic API is kept: ``send_to_all``, ``send_to_rank``, ``send_to_ranks``,
``set_output_callback``, ``shutdown``, ``Message``.
"""
from __future__ import annotations

import codecs
import itertools
import logging
import os
import queue
import secrets
import shutil
import signal
import _signal  # the C module: no enum round trip per call (pump swaps the SIGINT handler per wait)
import tempfile
import threading
import time
from typing import Any, Callable, Dict, Iterable, List, Optional

from . import protocol as P
from .protocol import Message  # noqa: F401  (re-exported: reference API)
from .transport import (EV_AUTH_FAILED, EV_CONNECTED, EV_DISCONNECTED, EV_HANDSHAKE_FAILED, EV_HEARTBEAT_TIMEOUT,
                        OPT_IO_SPIN_US, OPT_RECV_SPIN_US, ROUTER, HostUnreachable, Socket, TransportError)

OutputCallback = Callable[[int, str, str], None]

MAX_CAPTURED_OUTPUT = 1 << 20  # per rank per request, kept for programmatic callers

log = logging.getLogger("nbdistributed_amd.comm")

LEAD_GRACE_S = 0.02  # the receive thread stays parked this long after a waiter stops draining
_SIGINT = int(signal.SIGINT)
_MAIN = threading.main_thread()

# Reference-order bring-up (``ProcessManager().start_workers(n, addr, gpu_ids)`` -> port, then
# ``CommunicationManager(n, port, ...)``, reference magic.py:493-504): the launcher picks the port
# and the session token and records them here; the CommunicationManager that later binds that port
# picks up the token.  Workers' DEALERs retry their connect until the ROUTER is bound, and requests
# wait for the READY handshake, so the first message after init cannot be lost (reference D-2).
_SPAWNED: Dict[int, Dict[str, Any]] = {}
_SPAWNED_LOCK = threading.Lock()


def register_spawned(port: int, token: Optional[str], num_processes: int) -> None:
    with _SPAWNED_LOCK:
        _SPAWNED[port] = {"token": token, "n": num_processes}


def _claim_spawned(port: Optional[int]) -> Optional[Dict[str, Any]]:
    if port is None:
        return None
    with _SPAWNED_LOCK:
        return _SPAWNED.pop(port, None)


class RankDied(RuntimeError):
    def __init__(self, rank: int, reason: str):
        super().__init__(f"rank {rank} died: {reason}")
        self.rank = rank
        self.reason = reason


class RequestTimeout(TimeoutError):
    def __init__(self, msg: str, partial: Dict[int, Any]):
        super().__init__(msg)
        self.partial = partial


class PendingRequest:
    """One request in flight to a set of ranks."""

    def __init__(self, seq: int, msg_type: str, ranks: List[int], live: bool):
        self.seq = seq
        self.msg_type = msg_type
        self.ranks = list(ranks)
        self.responses: Dict[int, Any] = {}
        self.errors: Dict[int, bool] = {}
        self.dead: Dict[int, str] = {}
        self.outputs: Dict[int, List[str]] = {r: [] for r in ranks}
        self._out_bytes: Dict[int, int] = {r: 0 for r in ranks}
        self.events: Optional[queue.SimpleQueue] = queue.SimpleQueue() if live else None
        self.done = threading.Event()
        self.t_sent = time.perf_counter()
        self.t_done: Optional[float] = None
        self.t_first_reply: Dict[int, float] = {}
        self._lock = threading.Lock()

    def _maybe_done(self) -> None:
        if len(self.responses) + len(self.dead) >= len(self.ranks) and not self.done.is_set():
            self.t_done = time.perf_counter()
            self.done.set()
            if self.events is not None:
                self.events.put(("done",))

    def on_response(self, rank: int, data: Any, error: bool) -> None:
        with self._lock:
            if rank not in self.outputs or rank in self.responses or rank in self.dead:
                return
            self.responses[rank] = data
            self.errors[rank] = error
            self.t_first_reply[rank] = time.perf_counter()
            if self.events is not None:
                self.events.put(("response", rank))
            self._maybe_done()

    def on_stream(self, rank: int, stream: str, text: str) -> None:
        with self._lock:
            if rank in self.outputs and self._out_bytes[rank] < MAX_CAPTURED_OUTPUT:
                self.outputs[rank].append(text)
                self._out_bytes[rank] += len(text)
            if self.events is not None:
                self.events.put(("stream", rank, stream, text))

    def on_dead(self, rank: int, reason: str) -> None:
        with self._lock:
            if rank not in self.outputs or rank in self.responses or rank in self.dead:
                return
            self.dead[rank] = reason
            if self.events is not None:
                self.events.put(("dead", rank, reason))
            self._maybe_done()

    def results(self) -> Dict[int, Any]:
        """Per-rank results; dead ranks get an error dict, execute results carry the streamed
        output merged into ``output`` (reference semantics)."""
        out: Dict[int, Any] = {}
        for r in self.ranks:
            if r in self.responses:
                d = self.responses[r]
                if self.msg_type == "execute" and isinstance(d, dict):
                    d = dict(d)
                    streamed = "".join(self.outputs.get(r, []))
                    echo = d.get("output") or ""
                    d["output"] = streamed + echo
                    d["echo"] = echo
                out[r] = d
            elif r in self.dead:
                out[r] = {"error": f"rank {r} died: {self.dead[r]}", "dead": True, "rank": r}
        return out


class CommunicationManager:
    """Coordinator endpoint: ROUTER socket + receive thread + request table."""

    def __init__(self, num_processes: int, base_port: Optional[int] = None, output_callback: Optional[OutputCallback] = None,
                 default_timeout: Optional[float] = None, endpoint: Optional[str] = None, token: Optional[str] = None,
                 heartbeat_ivl_ms: Optional[int] = None, heartbeat_timeout_ms: Optional[int] = None,
                 use_token: Optional[bool] = None):
        from .config import get_config

        cfg = get_config()
        self.num_processes = num_processes
        self.output_callback = output_callback
        self.default_timeout = default_timeout
        spawned = _claim_spawned(base_port) if endpoint is None and token is None else None
        # workers spawned before this bind: requests wait for their READY (reference order)
        self._await_ready: Optional[float] = cfg.startup_timeout_s if spawned is not None else None
        if spawned is not None:
            token, use_token = spawned["token"], spawned["token"] is not None
        if use_token is None:
            use_token = cfg.use_token
        self.token = token if token is not None else (secrets.token_hex(16) if use_token else None)
        self._tmpdir: Optional[str] = None
        if endpoint is None:
            if base_port is not None:
                endpoint = f"tcp://{cfg.bind_host}:{base_port}"
            elif cfg.transport == "tcp":
                endpoint = f"tcp://{cfg.bind_host}:0"
            else:
                base = tempfile.gettempdir()
                if len(base) > 60:
                    base = "/tmp"
                self._tmpdir = tempfile.mkdtemp(prefix="nbd-", dir=base)
                os.chmod(self._tmpdir, 0o700)
                endpoint = f"ipc://{self._tmpdir}/coord.sock"
        self.sock = Socket(ROUTER, token=self.token.encode() if self.token else None,
                           heartbeat_ivl_ms=cfg.heartbeat_ivl_ms if heartbeat_ivl_ms is None else heartbeat_ivl_ms,
                           heartbeat_timeout_ms=cfg.heartbeat_timeout_ms if heartbeat_timeout_ms is None else heartbeat_timeout_ms,
                           mandatory=True)
        if cfg.spin_us > 0:
            self.sock.set_int(OPT_RECV_SPIN_US, cfg.spin_us)
            self.sock.set_int(OPT_IO_SPIN_US, cfg.spin_us)
        self.endpoint = self.sock.bind(endpoint)
        self._seq = itertools.count(1)
        # who drains the socket: the receive thread, or one waiting thread (the "leader")
        self._pcv = threading.Condition()
        self._bg_pumping = False   # the receive thread is inside recv_batch / handling a batch
        self._leader: Optional[threading.Thread] = None  # the waiting thread draining the socket
        self._lead_end = 0.0
        self._lock = threading.Lock()
        self.pending: Dict[int, PendingRequest] = {}
        self.ready: Dict[int, Dict[str, Any]] = {}
        self.connected: Dict[int, float] = {}
        self.dead: Dict[int, str] = {}
        self.ready_cv = threading.Condition(self._lock)
        self._decoders: Dict[tuple, Any] = {}
        self.background: "queue.SimpleQueue" = queue.SimpleQueue()
        self.event_log: List[tuple] = []
        self.running = True
        self._closing = False
        self.stopping = False  # set by Session.shutdown: worker exits are expected from here on
        self.thread = threading.Thread(target=self._message_handler, name="nbd-comm", daemon=True)
        self.thread.start()

    # ------------------------------------------------------------------ reference API
    def set_output_callback(self, callback: Optional[OutputCallback]) -> None:
        self.output_callback = callback

    def send_to_all(self, msg_type: str, data: Any = None, timeout: Optional[float] = None,
                    raise_on_error: bool = False) -> Dict[int, Any]:
        return self.send_to_ranks(list(range(self.num_processes)), msg_type, data, timeout, raise_on_error)

    def send_to_rank(self, rank: int, msg_type: str, data: Any = None, timeout: Optional[float] = None) -> Any:
        return self.send_to_ranks([rank], msg_type, data, timeout).get(rank)

    def send_to_ranks(self, ranks: Iterable[int], msg_type: str, data: Any = None, timeout: Optional[float] = None,
                      raise_on_error: bool = False) -> Dict[int, Any]:
        req = self.submit(list(ranks), msg_type, data, live=False)
        self.wait(req, timeout)
        res = req.results()
        if req.outputs and self.output_callback is not None and msg_type == "execute":
            for r in req.ranks:
                txt = "".join(req.outputs.get(r, []))
                if txt:
                    self.output_callback(r, txt, "stdout")
        if raise_on_error:
            for r, v in res.items():
                if isinstance(v, dict) and v.get("dead"):
                    raise RankDied(r, req.dead[r])
        return res

    # ------------------------------------------------------------------ async API
    def submit(self, ranks: List[int], msg_type: str, data: Any = None, flags: int = 0, live: bool = True) -> PendingRequest:
        if self._await_ready is not None:
            # first request after a reference-order bring-up: the workers were spawned before this
            # socket was bound; wait for their READY instead of routing into the void
            self.wait_ready(list(range(self.num_processes)), self._await_ready)
            self._await_ready = None
        mtype = P.TYPE_CODES[msg_type]
        seq = next(self._seq)
        req = PendingRequest(seq, msg_type, ranks, live)
        e, body = P.encode_body(data)
        header = P.pack_header(mtype, P.COORDINATOR_RANK, seq, P.S_NONE, e, flags)
        with self._lock:
            self.pending[seq] = req
            dead_now = {r: self.dead[r] for r in ranks if r in self.dead}
        for r, why in dead_now.items():
            req.on_dead(r, why)
        live = [r for r in ranks if r not in dead_now]
        try:  # one native call fans the request out (the body is encoded once)
            status = self.sock.send_multi([P.worker_identity(r) for r in live], [header, body])
        except TransportError as ex:
            status = [2] * len(live)
            for r in live:
                req.on_dead(r, f"send failed: {ex}")
            return req
        for r, st in zip(live, status):
            if st == 1:
                req.on_dead(r, "not connected")
            elif st:
                req.on_dead(r, "send failed")
        return req

    def wait(self, req: PendingRequest, timeout: Optional[float] = None) -> PendingRequest:
        t = self.default_timeout if timeout is None else timeout
        ok = self.pump(req.done.is_set, t)
        if ok is None:  # another thread is draining the socket: it completes our request too
            ok = req.done.wait(t) if t is not None else _wait_forever(req.done)
        self._forget(req)
        if not ok:
            missing = [r for r in req.ranks if r not in req.responses and r not in req.dead]
            log.warning("%s seq %d timed out after %ss; no reply from %s", req.msg_type, req.seq, t, missing)
            raise RequestTimeout(f"{req.msg_type}: no reply from ranks {missing} within {t}s", req.results())
        return req

    def pump(self, ready: Callable[[], bool], timeout: Optional[float]) -> Optional[bool]:
        """Drain the socket from the calling thread until ``ready()`` (True) or ``timeout``
        seconds pass (False; None = no limit).  Returns None without waiting if another thread
        already leads — the caller then waits on its request's Event, which the leader sets.

        The receive thread is parked (woken out of its native wait) for the duration, so replies
        are decoded by the waiter itself.  In the main thread SIGINT is deferred to batch
        boundaries: a KeyboardInterrupt raised between the native dequeue and the handling of a
        batch would lose replies, so the handler only records it and wakes the native wait, and
        the interrupt is raised here once the batch is handled."""
        if ready():
            return True
        me = threading.current_thread()
        prev = hit = None
        try:  # (leadership is released in `finally` whatever interrupts this)
            with self._pcv:
                if self._leader is not None or not self.running:
                    return None
                self._leader = me  # the receive thread parks while a leader is set
                while self._bg_pumping:
                    self.sock.wake_recv()
                    self._pcv.wait(0.05)
            if me is _MAIN:
                cur = _signal.getsignal(_SIGINT)
                if callable(cur):  # (SIG_IGN / SIG_DFL / a C-level handler: left alone)
                    hit = []

                    def _deferred(signum, frame):
                        hit.append(signum)
                        self.sock.wake_recv()

                    try:
                        _signal.signal(_SIGINT, _deferred)
                        prev = cur
                    except (ValueError, TypeError):  # not the main interpreter
                        hit = None
            deadline = None if timeout is None else time.monotonic() + timeout
            while True:
                if ready():
                    return True
                if hit:  # a deferred Ctrl-C: the previous handler, now that no reply can be lost
                    hit.clear()
                    prev(_SIGINT, None)  # (default: raises KeyboardInterrupt)
                remaining = None if deadline is None else deadline - time.monotonic()
                if remaining is not None and remaining <= 0:
                    return False
                try:
                    batch = self.sock.recv_batch(timeout=0.5 if remaining is None else min(0.5, remaining))
                except TransportError:
                    return ready()
                for m in batch:
                    self._handle_message(m)
        finally:
            if prev is not None:
                _signal.signal(_SIGINT, prev)
            if self._leader is me:
                # no notify: the receive thread resumes on its own after LEAD_GRACE_S, so
                # back-to-back cells never wake it (and never have to park it again)
                self._lead_end = time.monotonic()
                self._leader = None

    def _forget(self, req: PendingRequest) -> None:
        with self._lock:
            self.pending.pop(req.seq, None)

    def interrupt(self, ranks: Optional[List[int]] = None) -> None:
        """Out-of-band interrupt: the workers' native I/O thread raises SIGINT on arrival."""
        ranks = list(range(self.num_processes)) if ranks is None else ranks
        header = P.pack_header(P.T_INTERRUPT, P.COORDINATOR_RANK, 0, P.S_NONE, P.E_NONE, 0)
        for r in ranks:
            try:
                self.sock.send([P.worker_identity(r), header, b""])
            except TransportError:
                pass

    # ------------------------------------------------------------------ liveness
    def mark_dead(self, rank: int, reason: str) -> None:
        with self._lock:
            if self._closing:
                return
            prev = self.dead.get(rank)
            if prev is not None and "exit code" in prev:
                return
            self.dead[rank] = reason
            reqs = list(self.pending.values())
            self.ready_cv.notify_all()
        for req in reqs:
            req.on_dead(rank, reason)
        self.event_log.append((time.time(), "dead", rank, reason))
        (log.debug if self.stopping else log.warning)("rank %d marked dead: %s (%d request(s) resolved)", rank, reason, len(reqs))

    def wait_ready(self, ranks: List[int], timeout: Optional[float], alive: Optional[Callable[[], Dict[int, int]]] = None) -> Dict[int, Dict[str, Any]]:
        """Block until every rank has sent READY.  Raises RuntimeError with the worker's own
        error if a bootstrap fails, or if a process exits first."""
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._lock:
            while True:
                errs = {r: self.ready[r] for r in ranks if r in self.ready and "error" in self.ready[r]}
                if errs:
                    r, e = next(iter(errs.items()))
                    raise RuntimeError(f"rank {r} failed to start: {e['error']}\n{e.get('traceback', '')}")
                dead = {r: self.dead[r] for r in ranks if r in self.dead}
                if dead:
                    raise RuntimeError(f"workers exited during startup: {dead}")
                if all(r in self.ready for r in ranks):
                    return {r: self.ready[r] for r in ranks}
                if alive is not None:
                    exited = {r: c for r, c in alive().items() if r in ranks}
                    if exited:
                        raise RuntimeError(f"workers exited during startup (rank: exit code): {exited}")
                remaining = None if deadline is None else deadline - time.monotonic()
                if remaining is not None and remaining <= 0:
                    missing = [r for r in ranks if r not in self.ready]
                    raise TimeoutError(f"ranks {missing} not ready after {timeout}s")
                self.ready_cv.wait(0.2 if remaining is None else min(0.2, remaining))

    # ------------------------------------------------------------------ receive thread
    def _decode_stream(self, rank: int, stream: int, body: bytes) -> str:
        key = (rank, stream)
        dec = self._decoders.get(key)
        if dec is None:
            dec = self._decoders[key] = codecs.getincrementaldecoder("utf-8")(errors="replace")
        return dec.decode(body)

    def _message_handler(self) -> None:
        while self.running:
            with self._pcv:
                # a waiting thread drains the socket meanwhile; after it stops, wait LEAD_GRACE_S
                # more in case the next cell follows at once (output that arrives while nobody
                # waits is delivered at most that late)
                while self.running and (self._leader is not None or
                                        time.monotonic() - self._lead_end < LEAD_GRACE_S):
                    self._pcv.wait(LEAD_GRACE_S)
                if not self.running:
                    break
                self._bg_pumping = True
            try:
                try:
                    batch = self.sock.recv_batch(timeout=None)  # every queued reply in one native call
                except TransportError:
                    break
                for m in batch:
                    self._handle_message(m)
            finally:
                with self._pcv:
                    self._bg_pumping = False
                    self._pcv.notify_all()

    def _handle_message(self, m) -> None:
        if True:
            if m.is_event:
                self._on_event(m.event, P.rank_of_identity(m.identity))
                return
            if len(m.frames) < 2:
                return
            rank = P.rank_of_identity(m.frames[0])
            try:
                h = P.unpack_header(m.frames[1])
            except ValueError:
                return
            body = m.frames[2] if len(m.frames) > 2 else b""
            if rank is None:
                rank = h.rank
            if h.mtype == P.T_STREAM:
                text = self._decode_stream(rank, h.stream, body)
                if not text:
                    return
                stream = P.STREAM_NAMES.get(h.stream, "stdout")
                with self._lock:
                    req = self.pending.get(h.seq)
                if req is not None and rank in req.outputs:
                    req.on_stream(rank, stream, text)
                else:
                    cb = self.output_callback
                    if cb is not None:
                        try:
                            cb(rank, text, stream)
                        except Exception:
                            pass
                    else:
                        self.background.put((rank, stream, text))
                return
            try:
                data = P.decode_body(h.enc, body)
            except Exception as e:
                data = {"error": f"undecodable reply: {e}", "rank": rank}
            if h.mtype == P.T_RESPONSE:
                with self._lock:
                    req = self.pending.get(h.seq)
                if req is not None:
                    req.on_response(rank, data, bool(h.flags & P.F_ERROR))
            elif h.mtype == P.T_READY:
                with self._lock:
                    self.ready[rank] = data if isinstance(data, dict) else {"status": data}
                    self.ready_cv.notify_all()

    def _on_event(self, event: int, rank: Optional[int]) -> None:
        if rank is None:
            return
        self.event_log.append((time.time(), event, rank))
        if event == EV_CONNECTED:
            with self._lock:
                self.connected[rank] = time.time()
                if rank in self.dead and "exit code" not in self.dead[rank]:
                    self.dead.pop(rank)  # reconnected (attach mode)
        elif event in (EV_DISCONNECTED, EV_HEARTBEAT_TIMEOUT):
            with self._lock:
                self.connected.pop(rank, None)
                closing = self._closing
            if not closing:
                why = "heartbeat timeout (no traffic from the worker)" if event == EV_HEARTBEAT_TIMEOUT else "connection lost"
                self.mark_dead(rank, why)
        elif event in (EV_HANDSHAKE_FAILED, EV_AUTH_FAILED):
            pass

    # ------------------------------------------------------------------ teardown
    def shutdown(self) -> None:
        with self._lock:
            self._closing = True
            self.running = False
            reqs = list(self.pending.values())
        for req in reqs:
            for r in req.ranks:
                req.on_dead(r, "coordinator shut down")
        with self._pcv:
            self._pcv.notify_all()
        self.sock.close()
        self.thread.join(timeout=2.0)
        if self._tmpdir:
            shutil.rmtree(self._tmpdir, ignore_errors=True)


def _wait_forever(ev: threading.Event) -> bool:
    # Event.wait() without timeout is not interruptible on some Pythons; loop in slices so a
    # KeyboardInterrupt in the kernel's main thread is delivered promptly.
    while not ev.wait(0.5):
        pass
    return True
