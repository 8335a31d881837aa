"""Native ZMTP/3.1 transport: loopback, fan-in/out, large frames, events, auth, heartbeats,
reconnect, out-of-band interrupt, fd capture, and wire interop with real libzmq."""
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import textwrap
import threading
import time

import pytest

from nbdistributed_amd import transport as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _drain_event(sock, kind=T.EV_CONNECTED, timeout=5.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        m = sock.recv(0.5)
        if m is not None and m.is_event and m.event == kind:
            return m
    raise AssertionError(f"event {kind} not seen")


@pytest.fixture(params=["tcp", "ipc"])
def endpoint(request, tmp_path):
    if request.param == "tcp":
        return "tcp://127.0.0.1:0"
    return f"ipc://{tmp_path}/t.sock"


def test_router_dealer_roundtrip(endpoint):
    r = T.Socket(T.ROUTER, mandatory=True)
    ep = r.bind(endpoint)
    d = T.Socket(T.DEALER, identity=b"worker_0")
    d.connect(ep)
    ev = _drain_event(r)
    assert ev.identity == b"worker_0"
    d.send([b"a", b"", b"c" * 1000])
    m = r.recv(5)
    assert m.frames == [b"worker_0", b"a", b"", b"c" * 1000]
    r.send([b"worker_0", b"reply"])
    got = None
    for _ in range(5):
        got = d.recv(5)
        if not got.is_event:
            break
    assert got.frames == [b"reply"]
    d.close()
    r.close()


def test_fan_out_fan_in_8_peers():
    r = T.Socket(T.ROUTER, mandatory=True)
    ep = r.bind("tcp://127.0.0.1:0")
    ds = []
    for i in range(8):
        d = T.Socket(T.DEALER, identity=f"worker_{i}".encode())
        d.connect(ep)
        ds.append(d)
    seen = set()
    while len(seen) < 8:
        seen.add(_drain_event(r).identity)
    for rnd in range(50):
        for i in range(8):
            r.send([f"worker_{i}".encode(), str(rnd).encode()])
        for i, d in enumerate(ds):
            m = d.recv(5)
            while m.is_event:
                m = d.recv(5)
            assert m.frames == [str(rnd).encode()]
            d.send([f"{i}:{rnd}".encode()])
        got = set()
        for _ in range(8):
            got.add(r.recv(5).frames[1])
        assert got == {f"{i}:{rnd}".encode() for i in range(8)}
    for d in ds:
        d.close()
    r.close()


def test_send_multi_fans_out_once_and_reports_missing_peers():
    r = T.Socket(T.ROUTER, mandatory=True)
    ep = r.bind("tcp://127.0.0.1:0")
    ds = [T.Socket(T.DEALER, identity=f"worker_{i}".encode()) for i in range(4)]
    for d in ds:
        d.connect(ep)
    seen = set()
    while len(seen) < 4:
        seen.add(_drain_event(r).identity)
    idents = [f"worker_{i}".encode() for i in range(4)] + [b"worker_9"]
    for rnd in range(20):
        status = r.send_multi(idents, [b"hdr", str(rnd).encode()])
        assert status == [0, 0, 0, 0, 1]  # worker_9 never connected: EHOSTUNREACH
        for d in ds:
            m = d.recv(5)
            while m.is_event:
                m = d.recv(5)
            assert m.frames == [b"hdr", str(rnd).encode()]
    assert r.send_multi([], [b"x"]) == []
    # batched receive: every queued reply in one call, in arrival order, frames intact
    for i, d in enumerate(ds):
        d.send([f"r{i}".encode(), b"", os.urandom(100_000) if i == 3 else b"small"])
    got = []
    deadline = time.time() + 10
    while len(got) < 4 and time.time() < deadline:
        got += [m for m in r.recv_batch(1) if not m.is_event]
    assert sorted(m.frames[1] for m in got) == [b"r0", b"r1", b"r2", b"r3"]
    assert all(m.frames[2] == b"" for m in got)
    assert {len(m.frames[3]) for m in got} == {5, 100_000}  # > the 64 KiB batch buffer: grown
    assert r.recv_batch(0.05) == []
    for d in ds:
        d.close()
    r.close()


def test_large_frame_64mib():
    r = T.Socket(T.ROUTER)
    ep = r.bind("ipc://" + tempfile.mkdtemp() + "/big.sock")
    d = T.Socket(T.DEALER, identity=b"w")
    d.connect(ep)
    _drain_event(r)
    big = os.urandom(1 << 20) * 64
    d.send([big])
    m = r.recv(30)
    assert len(m.frames[1]) == len(big) and m.frames[1] == big
    d.close()
    r.close()


def test_mandatory_routing_and_disconnect_event():
    r = T.Socket(T.ROUTER, mandatory=True)
    ep = r.bind("tcp://127.0.0.1:0")
    with pytest.raises(T.HostUnreachable):
        r.send([b"nobody", b"x"])
    d = T.Socket(T.DEALER, identity=b"w1")
    d.connect(ep)
    _drain_event(r)
    d.close()
    ev = _drain_event(r, T.EV_DISCONNECTED)
    assert ev.identity == b"w1"
    with pytest.raises(T.HostUnreachable):
        r.send([b"w1", b"x"])
    r.close()


def test_token_auth_rejects_wrong_token():
    r = T.Socket(T.ROUTER, token=b"secret")
    ep = r.bind("tcp://127.0.0.1:0")
    bad = T.Socket(T.DEALER, identity=b"bad", token=b"nope")
    bad.connect(ep)
    _drain_event(r, T.EV_AUTH_FAILED)
    good = T.Socket(T.DEALER, identity=b"good", token=b"secret")
    good.connect(ep)
    assert _drain_event(r).identity == b"good"
    assert r.peer_count == 1
    for s in (bad, good, r):
        s.close()


def test_dealer_connects_before_router_binds(tmp_path):
    ep = f"ipc://{tmp_path}/late.sock"
    d = T.Socket(T.DEALER, identity=b"early")
    d.connect(ep)
    d.send([b"queued before bind"])  # held until the handshake completes
    time.sleep(0.3)
    r = T.Socket(T.ROUTER)
    r.bind(ep)
    _drain_event(r)
    m = r.recv(5)
    assert m.frames == [b"early", b"queued before bind"]
    d.close()
    r.close()


def test_heartbeat_timeout_detects_silent_peer():
    r = T.Socket(T.ROUTER, heartbeat_ivl_ms=50, heartbeat_timeout_ms=400)
    ep = r.bind("tcp://127.0.0.1:0")
    port = int(ep.rsplit(":", 1)[1])
    # a raw peer that completes the ZMTP handshake and then goes silent (like a frozen process)
    s = socket.create_connection(("127.0.0.1", port))
    greet = bytearray(64)
    greet[0], greet[8], greet[9], greet[10], greet[11] = 0xFF, 1, 0x7F, 3, 1
    greet[12:16] = b"NULL"
    s.sendall(bytes(greet))
    props = b"\x0bSocket-Type" + (6).to_bytes(4, "big") + b"DEALER" + b"\x08Identity" + (6).to_bytes(4, "big") + b"frozen"
    body = b"\x05READY" + props
    s.sendall(bytes([4, len(body)]) + body)
    assert _drain_event(r).identity == b"frozen"
    t0 = time.time()
    ev = _drain_event(r, T.EV_HEARTBEAT_TIMEOUT, timeout=5)
    assert ev.identity == b"frozen" and time.time() - t0 < 3
    s.close()
    r.close()


def _run_child(code: str, timeout: float = 30) -> subprocess.CompletedProcess:
    env = dict(os.environ, PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_signal_prefix_raises_sigint_in_busy_process(tmp_path):
    ep = f"ipc://{tmp_path}/sig.sock"
    r = T.Socket(T.ROUTER)
    r.bind(ep)
    code = f"""
        import time
        from nbdistributed_amd import transport as T
        d = T.Socket(T.DEALER, identity=b"w")
        d.set_bytes(T.OPT_SIGNAL_PREFIX, b"INT!")
        d.connect({ep!r})
        d.send([b"ready"])
        try:
            while True:   # busy in pure Python: only a signal can stop this
                sum(range(1000))
        except KeyboardInterrupt:
            print("interrupted")
    """
    proc = subprocess.Popen([sys.executable, "-c", textwrap.dedent(code)], env=dict(os.environ, PYTHONPATH=ROOT),
                            stdout=subprocess.PIPE, text=True)
    _drain_event(r, timeout=20)
    m = r.recv(20)
    assert m.frames[1] == b"ready"
    r.send([b"w", b"INT!now"])
    out, _ = proc.communicate(timeout=20)
    assert "interrupted" in out
    r.close()


def test_fd_capture_streams_python_and_c_output(tmp_path):
    ep = f"ipc://{tmp_path}/cap.sock"
    r = T.Socket(T.ROUTER)
    r.bind(ep)
    code = f"""
        import os, sys
        from nbdistributed_amd import transport as T
        d = T.Socket(T.DEALER, identity=b"w")
        d.set_int(T.OPT_STREAM_FLUSH_US, 1000)
        d.connect({ep!r})
        # stream chunks are not queued before the connection is up (the worker streams only after
        # its READY handshake): wait for the coordinator's ack first
        d.send([b"HI"])
        while True:
            m = d.recv(30)
            if m is not None and not m.is_event:
                break
        d.stream_header(1, b"OUT")
        d.stream_header(2, b"ERR")
        d.capture_fds()
        sys.stdout.reconfigure(line_buffering=True)
        print("python line")
        os.system("echo shell line")
        print("to stderr", file=sys.stderr)
        sys.stdout.flush(); sys.stderr.flush()
        d.stream_flush()
        d.send([b"DONE"])
        d.close()
    """
    proc = subprocess.Popen([sys.executable, "-c", textwrap.dedent(code)], env=dict(os.environ, PYTHONPATH=ROOT))
    out, err = b"", b""
    deadline = time.time() + 60  # a loaded host (pytest -n) can take many seconds to start the child
    while time.time() < deadline:
        m = r.recv(1)
        if m is None or m.is_event:
            continue
        if m.frames[1] == b"HI":
            r.send([m.frames[0], b"ACK"])
            continue
        if m.frames[1] == b"DONE":
            break
        if m.frames[1] == b"OUT":
            out += m.frames[2]
        elif m.frames[1] == b"ERR":
            err += m.frames[2]
    proc.wait(10)
    assert b"python line\n" in out and b"shell line\n" in out
    assert b"to stderr\n" in err
    r.close()


def test_many_threads_sending_concurrently():
    r = T.Socket(T.ROUTER)
    ep = r.bind("tcp://127.0.0.1:0")
    d = T.Socket(T.DEALER, identity=b"w")
    d.connect(ep)
    _drain_event(r)
    N, K = 8, 500

    def sender(i):
        for k in range(K):
            d.send([f"{i}".encode(), k.to_bytes(4, "little")])

    th = [threading.Thread(target=sender, args=(i,)) for i in range(N)]
    for t in th:
        t.start()
    last = {}
    for _ in range(N * K):
        m = r.recv(10)
        i = m.frames[1]
        k = int.from_bytes(m.frames[2], "little")
        assert last.get(i, -1) == k - 1  # per-sender order preserved
        last[i] = k
    for t in th:
        t.join()
    d.close()
    r.close()


PY39 = "/opt/conda/bin/python3.9"


@pytest.mark.skipif(not os.path.exists(PY39), reason="no python3.9 + pyzmq oracle")
def test_wire_interop_with_libzmq(tmp_path):
    chk = subprocess.run([PY39, "-c", "import zmq"], capture_output=True)
    if chk.returncode != 0:
        pytest.skip("pyzmq not importable by the oracle interpreter")
    code = f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import zmq
        from nbdistributed_amd import transport as T
        ctx = zmq.Context()
        r = T.Socket(T.ROUTER, mandatory=True)
        ep = r.bind("tcp://127.0.0.1:0")
        d = ctx.socket(zmq.DEALER); d.setsockopt(zmq.IDENTITY, b"worker_7"); d.setsockopt(zmq.HEARTBEAT_IVL, 50)
        d.connect(ep)
        ev = r.recv(5); assert ev.is_event and ev.identity == b"worker_7", ev
        d.send_multipart([b"a", b"b" * 300])
        m = r.recv(5); assert m.frames == [b"worker_7", b"a", b"b" * 300], m
        time.sleep(0.3)
        r.send([b"worker_7", b"reply", b""])
        assert d.poll(3000); assert d.recv_multipart() == [b"reply", b""]
        zr = ctx.socket(zmq.ROUTER); zr.bind("ipc://{tmp_path}/z.sock")
        od = T.Socket(T.DEALER, identity=b"worker_3", heartbeat_ivl_ms=50)
        od.connect("ipc://{tmp_path}/z.sock")
        od.send([b"hello", b"x" * 70000])
        assert zr.poll(3000); fr = zr.recv_multipart(); assert fr[0] == b"worker_3" and len(fr[2]) == 70000
        zr.send_multipart([b"worker_3", b"back"])
        m = od.recv(5)
        while m.is_event: m = od.recv(5)
        assert m.frames == [b"back"]
        print("INTEROP OK")
        od.close(); r.close(); d.close(0); zr.close(0); ctx.term()
    """
    res = subprocess.run([PY39, "-c", textwrap.dedent(code)], capture_output=True, text=True, timeout=60)
    assert "INTEROP OK" in res.stdout, res.stdout + res.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("san", ["thread", "address"])
def test_transport_under_sanitizer(tmp_path, san):
    """Host-side sanitizers on the native transport (GPU sanitizers are not available)."""
    from nbdistributed_amd._native import build_transport

    lib = build_transport(sanitize=san, out=tmp_path / f"libnbd_{san}.so")
    rt = subprocess.run(["g++", f"-print-file-name=lib{'tsan' if san == 'thread' else 'asan'}.so"],
                        capture_output=True, text=True).stdout.strip()
    if not os.path.exists(rt):
        pytest.skip("sanitizer runtime not installed")
    code = """
        import threading, time
        from nbdistributed_amd import transport as T
        r = T.Socket(T.ROUTER, mandatory=True, heartbeat_ivl_ms=20, heartbeat_timeout_ms=2000)
        ep = r.bind("tcp://127.0.0.1:0")
        ds = []
        for i in range(4):
            d = T.Socket(T.DEALER, identity=f"w{i}".encode(), heartbeat_ivl_ms=20)
            d.connect(ep); ds.append(d)
        n = 0
        while n < 4:
            m = r.recv(5)
            if m.is_event: n += 1
        def pump(i):
            for k in range(300):
                ds[i].send([b"x" * (k % 700)])
        th = [threading.Thread(target=pump, args=(i,)) for i in range(4)]
        [t.start() for t in th]
        got = 0
        while got < 1200:
            m = r.recv(5)
            if not m.is_event:
                got += 1
                r.send([m.frames[0], b"ack"])
        [t.join() for t in th]
        for d in ds: d.close()
        r.close()
        print("SAN OK")
    """
    env = dict(os.environ, PYTHONPATH=ROOT, NBD_TRANSPORT_LIB=str(lib), LD_PRELOAD=rt,
               TSAN_OPTIONS="halt_on_error=1 report_signal_unsafe=0", ASAN_OPTIONS="detect_leaks=0:halt_on_error=1")
    res = subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=env, capture_output=True, text=True,
                         timeout=180)
    report = res.stderr
    assert "SAN OK" in res.stdout, report[-4000:]
    assert "WARNING: ThreadSanitizer" not in report and "ERROR: AddressSanitizer" not in report, report[-4000:]
