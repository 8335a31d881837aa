"""ctypes binding for the native ZMTP/3.1 DEALER/ROUTER transport (``libnbd_transport.so``).

The reference talks ZeroMQ through pyzmq (``src/nbdistributed/communication.py:121-125``,
``worker.py:154-157``).  pyzmq is not importable by the PyTorch-ROCm interpreter, so the
framework carries its own wire-compatible implementation (``csrc/transport``) behind a C ABI.
ctypes releases the GIL for every foreign call, so a thread blocked in :meth:`Socket.recv`
never stalls the interpreter.

Only standard library imports here: the coordinator may run on an interpreter without torch.
"""
from __future__ import annotations

import ctypes
import struct
import os
import threading
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Union

ROUTER = 1
DEALER = 2

KIND_MSG = 0
KIND_EVENT = 1

EV_CONNECTED = 1
EV_DISCONNECTED = 2
EV_HANDSHAKE_FAILED = 3
EV_HEARTBEAT_TIMEOUT = 4
EV_AUTH_FAILED = 5

EVENT_NAMES = {
    EV_CONNECTED: "connected",
    EV_DISCONNECTED: "disconnected",
    EV_HANDSHAKE_FAILED: "handshake_failed",
    EV_HEARTBEAT_TIMEOUT: "heartbeat_timeout",
    EV_AUTH_FAILED: "auth_failed",
}

OPT_IDENTITY = 1
OPT_TOKEN = 2
OPT_HEARTBEAT_IVL_MS = 3
OPT_HEARTBEAT_TIMEOUT_MS = 4
OPT_ROUTER_MANDATORY = 5
OPT_STREAM_FLUSH_US = 6
OPT_STREAM_MAX_BYTES = 7
OPT_SIGNAL_PREFIX = 8
OPT_RECONNECT_IVL_MS = 9
OPT_SNDHWM_BYTES = 10
OPT_RECV_SPIN_US = 11
OPT_IO_SPIN_US = 12

_lib = None
_lib_lock = threading.Lock()


class TransportError(RuntimeError):
    pass


class HostUnreachable(TransportError):
    """ROUTER send to an identity that is not connected (ROUTER_MANDATORY)."""


def _load():
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        path = os.environ.get("NBD_TRANSPORT_LIB")
        if not path:
            from .._native import build_transport

            path = str(build_transport())
        lib = ctypes.CDLL(path)
        vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        lib.nbd_version.restype = i
        lib.nbd_last_error.restype = ctypes.c_char_p
        lib.nbd_socket_new.argtypes = [i]
        lib.nbd_socket_new.restype = vp
        lib.nbd_setopt_int.argtypes = [vp, i, ctypes.c_int64]
        lib.nbd_setopt_bytes.argtypes = [vp, i, ctypes.c_char_p, sz]
        lib.nbd_bind.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, sz]
        lib.nbd_connect.argtypes = [vp, ctypes.c_char_p]
        lib.nbd_send.argtypes = [vp, i, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz)]
        lib.nbd_send_multi.argtypes = [vp, i, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), i,
                                       ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(sz), ctypes.POINTER(i)]
        lib.nbd_recv.argtypes = [vp, i, ctypes.POINTER(vp)]
        lib.nbd_recv_batch.argtypes = [vp, i, vp, sz, ctypes.POINTER(sz), i]
        lib.nbd_wake_recv.argtypes = [vp]
        lib.nbd_msg_kind.argtypes = [vp]
        lib.nbd_msg_event.argtypes = [vp]
        lib.nbd_msg_nframes.argtypes = [vp]
        lib.nbd_msg_frames.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(sz), i]
        lib.nbd_msg_free.argtypes = [vp]
        lib.nbd_peer_count.argtypes = [vp]
        lib.nbd_capture_fds.argtypes = [vp, i, ctypes.POINTER(i), ctypes.POINTER(i)]
        lib.nbd_capture_stop.argtypes = [vp]
        lib.nbd_stream_header.argtypes = [vp, i, ctypes.c_char_p, sz]
        lib.nbd_stream_flush.argtypes = [vp]
        lib.nbd_close.argtypes = [vp]
        lib.nbd_close.restype = None
        _lib = lib
        return lib


def library_path() -> str:
    lib = _load()
    return lib._name


def _err(lib) -> str:
    e = lib.nbd_last_error()
    return e.decode(errors="replace") if e else "unknown error"


_HDR3 = struct.Struct("=III")
_LEN = struct.Struct("=Q")


@dataclass
class Received:
    """One item from :meth:`Socket.recv`: a multipart message or a peer event."""

    kind: int
    frames: List[bytes] = field(default_factory=list)
    event: int = 0

    @property
    def is_event(self) -> bool:
        return self.kind == KIND_EVENT

    @property
    def event_name(self) -> str:
        return EVENT_NAMES.get(self.event, str(self.event))

    @property
    def identity(self) -> bytes:
        return self.frames[0] if self.frames else b""


class Socket:
    """A DEALER or ROUTER socket backed by the native I/O thread."""

    def __init__(self, kind: int, identity: Optional[bytes] = None, token: Optional[bytes] = None,
                 heartbeat_ivl_ms: int = 0, heartbeat_timeout_ms: int = 0, mandatory: bool = False):
        self._lib = _load()
        h = self._lib.nbd_socket_new(kind)
        if not h:
            raise TransportError(_err(self._lib))
        self._h = ctypes.c_void_p(h)
        self.kind = kind
        self._closed = False
        self._close_lock = threading.Lock()
        self._idcache: dict = {}
        if identity is not None:
            self.set_bytes(OPT_IDENTITY, identity)
        if token:
            self.set_bytes(OPT_TOKEN, token)
        if heartbeat_ivl_ms:
            self.set_int(OPT_HEARTBEAT_IVL_MS, heartbeat_ivl_ms)
        if heartbeat_timeout_ms:
            self.set_int(OPT_HEARTBEAT_TIMEOUT_MS, heartbeat_timeout_ms)
        if mandatory:
            self.set_int(OPT_ROUTER_MANDATORY, 1)

    # -- options -------------------------------------------------------------
    def set_int(self, opt: int, value: int) -> None:
        if self._lib.nbd_setopt_int(self._h, opt, int(value)) != 0:
            raise TransportError(_err(self._lib))

    def set_bytes(self, opt: int, value: bytes) -> None:
        if self._lib.nbd_setopt_bytes(self._h, opt, value, len(value)) != 0:
            raise TransportError(_err(self._lib))

    # -- connection ------------------------------------------------------------
    def bind(self, endpoint: str) -> str:
        buf = ctypes.create_string_buffer(512)
        if self._lib.nbd_bind(self._h, endpoint.encode(), buf, 512) != 0:
            raise TransportError(_err(self._lib))
        return buf.value.decode()

    def connect(self, endpoint: str) -> None:
        if self._lib.nbd_connect(self._h, endpoint.encode()) != 0:
            raise TransportError(_err(self._lib))

    @property
    def peer_count(self) -> int:
        return self._lib.nbd_peer_count(self._h)

    # -- data ------------------------------------------------------------------
    def send(self, frames: Sequence[Union[bytes, bytearray, memoryview]]) -> None:
        n = len(frames)
        fr = [f if isinstance(f, bytes) else bytes(f) for f in frames]
        ptrs = (ctypes.c_char_p * n)(*fr)
        lens = (ctypes.c_size_t * n)(*[len(f) for f in fr])
        if self._lib.nbd_send(self._h, n, ptrs, lens) != 0:
            msg = _err(self._lib)
            if msg.startswith("EHOSTUNREACH"):
                raise HostUnreachable(msg)
            raise TransportError(msg)

    def send_multi(self, identities: Sequence[bytes], frames: Sequence[Union[bytes, bytearray, memoryview]]) -> List[int]:
        """ROUTER: the same message to every identity in one native call (the body is encoded
        once).  Returns a status per identity: 0 sent, 1 no such peer, 2 other error."""
        k = len(identities)
        if k == 0:
            return []
        n = len(frames)
        fr = [f if isinstance(f, bytes) else bytes(f) for f in frames]
        ptrs = (ctypes.c_char_p * n)(*fr)
        lens = (ctypes.c_size_t * n)(*[len(f) for f in fr])
        # the identity arrays of a rank set are built once (every cell goes to the same ranks)
        key = tuple(identities)
        cached = self._idcache.get(key)
        if cached is None:
            if len(self._idcache) > 64:
                self._idcache.clear()
            cached = self._idcache[key] = ((ctypes.c_char_p * k)(*key), (ctypes.c_size_t * k)(*[len(x) for x in key]))
        status = (ctypes.c_int * k)()
        if self._lib.nbd_send_multi(self._h, k, cached[0], cached[1], n, ptrs, lens, status) < 0:
            raise TransportError(_err(self._lib))
        return list(status)

    def recv_batch(self, timeout: Optional[float] = None, max_msgs: int = 256) -> List[Received]:
        """Every queued message (up to ``max_msgs``) in one native call, waiting up to ``timeout``
        seconds (None = forever) for the first; [] on timeout; raises TransportError once the
        socket is closed."""
        ms = -1 if timeout is None else max(0, int(timeout * 1000))
        buf = getattr(self, "_rbuf", None)
        if buf is None:
            buf = self._rbuf = ctypes.create_string_buffer(1 << 16)
        used = ctypes.c_size_t()
        while True:
            n = self._lib.nbd_recv_batch(self._h, ms, buf, len(buf), ctypes.byref(used), max_msgs)
            if n == -2:  # a message larger than the buffer: grow and retry
                buf = self._rbuf = ctypes.create_string_buffer(max(used.value, 2 * len(buf)))
                continue
            break
        if n == 0:
            return []
        if n < 0:
            raise TransportError("socket closed")
        raw = ctypes.string_at(buf, used.value)
        out: List[Received] = []
        pos = 0
        unpack3, unpack1 = _HDR3.unpack_from, _LEN.unpack_from
        for _ in range(n):
            kind, event, nf = unpack3(raw, pos)
            pos += 12
            frames = []
            for _ in range(nf):
                (ln,) = unpack1(raw, pos)
                pos += 8
                frames.append(raw[pos:pos + ln])
                pos += ln
            out.append(Received(kind, frames, event))
        return out

    def wake_recv(self) -> None:
        """Make the recv / recv_batch call blocked right now (or the next one that would block)
        return as on a timeout."""
        self._lib.nbd_wake_recv(self._h)

    def recv(self, timeout: Optional[float] = None) -> Optional[Received]:
        """Block up to ``timeout`` seconds (None = forever).  Returns None on timeout; raises
        TransportError once the socket is closed."""
        ms = -1 if timeout is None else max(0, int(timeout * 1000))
        out = ctypes.c_void_p()
        rc = self._lib.nbd_recv(self._h, ms, ctypes.byref(out))
        if rc == 1:
            return None
        if rc != 0:
            raise TransportError("socket closed")
        m = out.value
        try:
            kind = self._lib.nbd_msg_kind(m)
            n = self._lib.nbd_msg_nframes(m)
            ptrs = (ctypes.c_void_p * n)()
            lens = (ctypes.c_size_t * n)()
            self._lib.nbd_msg_frames(m, ptrs, lens, n)
            frames = [ctypes.string_at(ptrs[i], lens[i]) if lens[i] else b"" for i in range(n)]
            ev = self._lib.nbd_msg_event(m) if kind == KIND_EVENT else 0
        finally:
            self._lib.nbd_msg_free(m)
        return Received(kind=kind, frames=frames, event=ev)

    # -- worker-side output capture -------------------------------------------
    def capture_fds(self, stdout: bool = True, stderr: bool = True):
        """Redirect this process's fd 1/2 into natively drained pipes.  Returns the dup'ed
        original descriptors (stdout_fd, stderr_fd), -1 where not captured."""
        a, b = ctypes.c_int(-1), ctypes.c_int(-1)
        mask = (1 if stdout else 0) | (2 if stderr else 0)
        if self._lib.nbd_capture_fds(self._h, mask, ctypes.byref(a), ctypes.byref(b)) != 0:
            raise TransportError(_err(self._lib))
        return a.value, b.value

    def capture_stop(self) -> None:
        self._lib.nbd_capture_stop(self._h)

    def stream_header(self, stream: int, header: bytes) -> None:
        if self._lib.nbd_stream_header(self._h, stream, header, len(header)) != 0:
            raise TransportError(_err(self._lib))

    def stream_flush(self) -> None:
        self._lib.nbd_stream_flush(self._h)

    # -- lifecycle ---------------------------------------------------------------
    def close(self) -> None:
        with self._close_lock:
            if self._closed:
                return
            self._closed = True
        self._lib.nbd_close(self._h)

    @property
    def closed(self) -> bool:
        return self._closed

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
