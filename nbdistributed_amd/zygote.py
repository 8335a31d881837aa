"""Zygote: a pre-warmed fork server for worker processes (fast ``%dist_init``).

A worker's bring-up is dominated by ``import torch`` (1.2–1.8 s warm, measured:
``benchmarks/init_time.py``); the reference pays a fixed 2 s sleep on top
(``process_manager.py:137``).  The zygote is started in the background when the extension loads:
it imports torch, torch.distributed and the worker runtime — but never touches HIP (no
``torch.cuda`` call, no HIP library loaded), so forking it is safe — and then serves spawn
requests on a private Unix socket.

Protocol (one connection per worker): the coordinator sends a JSON request (argv, env, cwd) with
the write ends of the worker's stdout/stderr pipes attached as SCM_RIGHTS; the zygote forks, the
child calls ``setsid()``, installs the fds and env, and runs ``worker.main(argv)``; the zygote
replies ``{"pid": ...}`` and later ``{"exit": code}`` when it reaps the child.  ``ZygoteProc``
gives the launcher a ``subprocess.Popen``-like handle (pid, poll, wait, returncode, stdout,
stderr), so the rest of the launcher is unchanged.  The zygote exits when its parent (the
notebook kernel) goes away, killing its children's process groups.
"""
from __future__ import annotations

import array
import io
import json
import os
import select
import signal
import socket
import struct
import subprocess
import sys
import tempfile
import threading
import time
import traceback
from typing import Dict, List, Optional

MAX_MSG = 1 << 20


# ----------------------------------------------------------------------------- server side
def _recv_request(conn: socket.socket):
    fds = array.array("i")
    msg, anc, _flags, _addr = conn.recvmsg(MAX_MSG, socket.CMSG_SPACE(2 * fds.itemsize))
    for level, typ, data in anc:
        if level == socket.SOL_SOCKET and typ == socket.SCM_RIGHTS:
            fds.frombytes(data[: len(data) - (len(data) % fds.itemsize)])
    return json.loads(msg.decode()), list(fds)


def _send(conn: socket.socket, obj) -> None:
    try:
        conn.sendall(json.dumps(obj).encode() + b"\n")
    except OSError:
        pass


def serve(path: str) -> int:
    os.environ.setdefault("TORCH_CPP_LOG_LEVEL", "ERROR")
    ppid = os.getppid()
    import torch  # noqa: F401  (the point of the zygote)
    import torch.distributed  # noqa: F401

    from . import worker as W  # noqa: F401
    from .parallel import backend  # noqa: F401

    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass
    srv.bind(path)
    os.chmod(path, 0o600)
    srv.listen(64)
    sys.stdout.write("ZYGOTE READY\n")
    sys.stdout.flush()
    children: Dict[int, socket.socket] = {}
    conns: List[socket.socket] = []
    while True:
        if os.getppid() != ppid:  # the kernel died: take our children with us
            for pid in children:
                try:
                    os.killpg(pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
            return 0
        r, _, _ = select.select([srv] + conns, [], [], 0.1)
        for s in r:
            if s is srv:
                c, _ = srv.accept()
                conns.append(c)
                continue
            try:
                req, fds = _recv_request(s)
            except (OSError, ValueError):
                conns.remove(s)
                s.close()
                continue
            if not req:
                conns.remove(s)
                s.close()
                continue
            if req.get("op") == "ping":
                _send(s, {"pong": os.getpid()})
                continue
            sys.stdout.flush()
            sys.stderr.flush()
            pid = os.fork()
            if pid == 0:  # ---------------- child: becomes the worker
                code = 1
                try:
                    srv.close()
                    for c in conns:
                        c.close()
                    os.setsid()
                    devnull = os.open(os.devnull, os.O_RDONLY)
                    os.dup2(devnull, 0)
                    if len(fds) >= 2:
                        os.dup2(fds[0], 1)
                        os.dup2(fds[1], 2)
                    for fd in fds + [devnull]:
                        if fd > 2:
                            os.close(fd)
                    os.environ.clear()
                    os.environ.update(req.get("env", {}))
                    os.chdir(req.get("cwd") or "/")
                    sys.stdout = io.TextIOWrapper(os.fdopen(1, "wb", buffering=0), write_through=True)
                    sys.stderr = io.TextIOWrapper(os.fdopen(2, "wb", buffering=0), write_through=True)
                    sys.__stdout__, sys.__stderr__ = sys.stdout, sys.stderr
                    W._PROCESS_T0 = time.time()
                    code = W.main(req["argv"]) or 0
                except SystemExit as e:
                    code = e.code if isinstance(e.code, int) else 1
                except BaseException:
                    traceback.print_exc()
                    code = 1
                finally:
                    try:
                        sys.stdout.flush()
                        sys.stderr.flush()
                    except Exception:
                        pass
                    os._exit(code)
            for fd in fds:
                os.close(fd)
            children[pid] = s
            conns.remove(s)  # this connection now only carries the exit notification
            _send(s, {"pid": pid})
        # reap
        while children:
            try:
                pid, status = os.waitpid(-1, os.WNOHANG)
            except ChildProcessError:
                break
            if pid == 0:
                break
            code = os.waitstatus_to_exitcode(status) if hasattr(os, "waitstatus_to_exitcode") else status >> 8
            c = children.pop(pid, None)
            if c is not None:
                _send(c, {"exit": code})
                c.close()


# ----------------------------------------------------------------------------- client side
class ZygoteProc:
    """subprocess.Popen-like handle for a zygote-forked worker."""

    def __init__(self, conn: socket.socket, pid: int, stdout, stderr, pending: bytes = b""):
        self._conn = conn
        self.pid = pid
        self.stdout = stdout
        self.stderr = stderr
        self.returncode: Optional[int] = None
        self._done = threading.Event()
        self._buf = pending
        threading.Thread(target=self._watch, daemon=True, name=f"nbd-zygote-watch-{pid}").start()

    def _watch(self) -> None:
        try:
            while True:
                if b"\n" in self._buf:
                    chunk = b""
                else:
                    chunk = self._conn.recv(4096)
                    if not chunk:
                        break
                self._buf += chunk
                while b"\n" in self._buf:
                    line, self._buf = self._buf.split(b"\n", 1)
                    msg = json.loads(line.decode())
                    if "exit" in msg:
                        self.returncode = int(msg["exit"])
        except OSError:
            pass
        if self.returncode is None:  # zygote vanished: fall back to probing the pid
            while _alive(self.pid):
                time.sleep(0.1)
            self.returncode = -9
        self._done.set()
        try:
            self._conn.close()
        except OSError:
            pass

    def poll(self) -> Optional[int]:
        return self.returncode if self._done.is_set() else None

    def wait(self, timeout: Optional[float] = None) -> int:
        if not self._done.wait(timeout):
            raise subprocess.TimeoutExpired(f"worker pid {self.pid}", timeout)
        return self.returncode  # type: ignore[return-value]


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


class Zygote:
    """Client handle: starts the server process and spawns workers through it."""

    def __init__(self, python: str):
        self.python = python
        self.dir = tempfile.mkdtemp(prefix="nbd-zygote-", dir="/tmp")
        os.chmod(self.dir, 0o700)
        self.path = os.path.join(self.dir, "zygote.sock")
        env = dict(os.environ)
        repo_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = repo_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env.setdefault("TORCH_CPP_LOG_LEVEL", "ERROR")
        self.proc = subprocess.Popen([python, "-m", "nbdistributed_amd.zygote", self.path], env=env,
                                     stdin=subprocess.DEVNULL, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                     start_new_session=True)
        self.ready = threading.Event()
        self.error: Optional[str] = None
        threading.Thread(target=self._wait_ready, daemon=True, name="nbd-zygote-ready").start()

    def _wait_ready(self) -> None:
        line = self.proc.stdout.readline()
        if line.strip() == b"ZYGOTE READY":
            self.ready.set()
            # keep draining so the zygote never blocks on a full pipe
            threading.Thread(target=lambda: [None for _ in iter(self.proc.stdout.readline, b"")], daemon=True).start()
            threading.Thread(target=lambda: [None for _ in iter(self.proc.stderr.readline, b"")], daemon=True).start()
        else:
            err = self.proc.stderr.read().decode(errors="replace")
            self.error = f"zygote failed to start: {line!r} {err[-2000:]}"
            self.ready.set()

    @property
    def alive(self) -> bool:
        return self.proc.poll() is None and self.error is None

    def wait_ready(self, timeout: float) -> bool:
        return self.ready.wait(timeout) and self.error is None and self.proc.poll() is None

    def spawn(self, argv: List[str], env: Dict[str, str], cwd: str) -> ZygoteProc:
        out_r, out_w = os.pipe()
        err_r, err_w = os.pipe()
        conn = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            conn.connect(self.path)
            payload = json.dumps({"argv": argv, "env": env, "cwd": cwd}).encode()
            conn.sendmsg([payload], [(socket.SOL_SOCKET, socket.SCM_RIGHTS, array.array("i", [out_w, err_w]))])
            buf = b""
            while b"\n" not in buf:
                chunk = conn.recv(4096)
                if not chunk:
                    raise RuntimeError("zygote closed the connection")
                buf += chunk
        except BaseException:
            for fd in (out_r, err_r):
                os.close(fd)
            conn.close()
            raise
        finally:
            os.close(out_w)
            os.close(err_w)
        line, rest = buf.split(b"\n", 1)
        pid = int(json.loads(line.decode())["pid"])
        return ZygoteProc(conn, pid, os.fdopen(out_r, "rb"), os.fdopen(err_r, "rb"), pending=rest)

    def close(self) -> None:
        try:
            os.killpg(self.proc.pid, signal.SIGTERM)
        except (ProcessLookupError, PermissionError):
            pass
        try:
            self.proc.wait(2)
        except subprocess.TimeoutExpired:
            try:
                os.killpg(self.proc.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
        try:
            os.unlink(self.path)
            os.rmdir(self.dir)
        except OSError:
            pass


_shared: Optional[Zygote] = None
_shared_lock = threading.Lock()


def get_zygote(python: str, start: bool = True) -> Optional[Zygote]:
    """Process-wide zygote for ``python`` (started on first call)."""
    global _shared
    with _shared_lock:
        if _shared is not None and (_shared.python != python or not _shared.alive):
            _shared.close()
            _shared = None
        if _shared is None and start:
            _shared = Zygote(python)
            import atexit

            atexit.register(_shared.close)
        return _shared


if __name__ == "__main__":
    sys.exit(serve(sys.argv[1]))
