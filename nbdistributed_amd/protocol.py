"""Wire protocol between the coordinator and the workers.

The reference pickles a whole ``Message`` dataclass into one ZMQ frame
(``src/nbdistributed/communication.py:30-62``; ``worker.py:58, 233``).  Here a message is two
ZMTP frames:

* frame 0 — a fixed 28-byte typed header (magic, version, type, stream, body encoding, flags,
  rank, sequence id, timestamp).  Routing, correlation and stream demultiplexing only ever
  read this header; the coordinator never unpickles output chunks.
* frame 1 — the body, encoded per the header: raw UTF-8 (code, stdout/stderr text), raw
  bytes, or pickle (protocol 5) for structured payloads.

``Message`` keeps the reference's field names (msg_id, msg_type, rank, data, timestamp) so
programmatic users of the reference API keep working.
"""
from __future__ import annotations

import pickle
import struct
import time
from dataclasses import dataclass, field
from typing import Any, List, Optional

MAGIC = b"NB"
VERSION = 1
HEADER = struct.Struct("<2sBBBBHiQd")  # magic, ver, type, stream, enc, flags, rank, seq, ts
HEADER_SIZE = HEADER.size

COORDINATOR_RANK = -1

# message types -----------------------------------------------------------------------------
T_EXECUTE = 1
T_GET_VAR = 2
T_SET_VAR = 3
T_SYNC = 4
T_GET_STATUS = 5
T_GET_NAMESPACE_INFO = 6
T_SHUTDOWN = 7
T_RESPONSE = 8
T_STREAM = 9
T_READY = 10
T_INTERRUPT = 11
T_PING = 12
T_RECOVER = 13
T_PROFILE = 14
T_CALL = 15  # invoke a registered worker-side handler by name (extensibility hook)

TYPE_NAMES = {
    T_EXECUTE: "execute",
    T_GET_VAR: "get_var",
    T_SET_VAR: "set_var",
    T_SYNC: "sync",
    T_GET_STATUS: "get_status",
    T_GET_NAMESPACE_INFO: "get_namespace_info",
    T_SHUTDOWN: "shutdown",
    T_RESPONSE: "response",
    T_STREAM: "stream_output",
    T_READY: "ready",
    T_INTERRUPT: "interrupt",
    T_PING: "ping",
    T_RECOVER: "recover",
    T_PROFILE: "profile",
    T_CALL: "call",
}
TYPE_CODES = {v: k for k, v in TYPE_NAMES.items()}

# stream ids (T_STREAM) ---------------------------------------------------------------------
S_NONE = 0
S_STDOUT = 1
S_STDERR = 2
S_RESULT = 3
STREAM_NAMES = {S_NONE: "", S_STDOUT: "stdout", S_STDERR: "stderr", S_RESULT: "result"}
STREAM_CODES = {v: k for k, v in STREAM_NAMES.items()}

# body encodings ------------------------------------------------------------------------------
E_PICKLE = 0
E_UTF8 = 1
E_BYTES = 2
E_NONE = 3

# header flags ----------------------------------------------------------------------------------
F_NS_DELTA = 1 << 0  # execute: attach a namespace delta to the response (IDE sync)
F_NO_ECHO = 1 << 1  # execute: do not echo the last expression
F_ERROR = 1 << 2  # response: the handler failed

# Prefix of an interrupt message's header frame.  The native transport raises SIGINT in the
# worker the moment such a frame arrives (NBD_OPT_SIGNAL_PREFIX), even while the interpreter is
# busy running a cell.
INTERRUPT_PREFIX = MAGIC + bytes([VERSION, T_INTERRUPT])


def worker_identity(rank: int) -> bytes:
    """Routing identity of rank ``rank`` (same naming as the reference, worker.py:155-156)."""
    return f"worker_{rank}".encode()


def rank_of_identity(ident: bytes) -> Optional[int]:
    if ident.startswith(b"worker_"):
        try:
            return int(ident[7:])
        except ValueError:
            return None
    return None


def pack_header(mtype: int, rank: int, seq: int, stream: int = S_NONE, enc: int = E_PICKLE,
                flags: int = 0, ts: Optional[float] = None) -> bytes:
    return HEADER.pack(MAGIC, VERSION, mtype, stream, enc, flags, rank, seq, time.time() if ts is None else ts)


@dataclass
class Header:
    mtype: int
    stream: int
    enc: int
    flags: int
    rank: int
    seq: int
    ts: float

    @property
    def type_name(self) -> str:
        return TYPE_NAMES.get(self.mtype, str(self.mtype))


def unpack_header(buf: bytes) -> Header:
    if len(buf) < HEADER_SIZE:
        raise ValueError("short header")
    magic, ver, mtype, stream, enc, flags, rank, seq, ts = HEADER.unpack_from(buf)
    if magic != MAGIC or ver != VERSION:
        raise ValueError(f"bad header magic/version {magic!r}/{ver}")
    return Header(mtype, stream, enc, flags, rank, seq, ts)


def encode_body(data: Any, enc: Optional[int] = None):
    """Pick the cheapest encoding for ``data``; returns (enc, bytes)."""
    if enc is None:
        if data is None:
            return E_NONE, b""
        if isinstance(data, str):
            return E_UTF8, data.encode("utf-8", errors="surrogateescape")
        if isinstance(data, (bytes, bytearray)):
            return E_BYTES, bytes(data)
        return E_PICKLE, pickle.dumps(data, protocol=5)
    if enc == E_UTF8:
        return enc, data.encode("utf-8", errors="surrogateescape")
    if enc == E_BYTES:
        return enc, bytes(data)
    if enc == E_NONE:
        return enc, b""
    return E_PICKLE, pickle.dumps(data, protocol=5)


def decode_body(enc: int, body: bytes) -> Any:
    if enc == E_UTF8:
        return body.decode("utf-8", errors="replace")
    if enc == E_BYTES:
        return body
    if enc == E_NONE:
        return None
    return pickle.loads(body)


def encode(mtype: int, rank: int, seq: int, data: Any = None, stream: int = S_NONE, flags: int = 0,
           enc: Optional[int] = None) -> List[bytes]:
    e, body = encode_body(data, enc)
    return [pack_header(mtype, rank, seq, stream, e, flags), body]


@dataclass
class Message:
    """Reference-compatible message object (``communication.py:30-62``).

    ``msg_id`` is the decimal sequence id of the request it belongs to; ``rank`` is -1 for the
    coordinator."""

    msg_id: str
    msg_type: str
    rank: int
    data: Any
    timestamp: float = field(default_factory=time.time)
    stream: str = ""
    flags: int = 0

    def to_frames(self) -> List[bytes]:
        mtype = TYPE_CODES.get(self.msg_type)
        if mtype is None:
            raise ValueError(f"unknown message type {self.msg_type!r}")
        return encode(mtype, self.rank, int(self.msg_id), self.data, STREAM_CODES.get(self.stream, 0), self.flags)

    @classmethod
    def from_frames(cls, frames: List[bytes]) -> "Message":
        h = unpack_header(frames[0])
        data = decode_body(h.enc, frames[1] if len(frames) > 1 else b"")
        return cls(str(h.seq), h.type_name, h.rank, data, h.ts, STREAM_NAMES.get(h.stream, ""), h.flags)
