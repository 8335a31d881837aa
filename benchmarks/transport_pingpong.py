#!/usr/bin/env python3
"""Control-plane hop costs: ROUTER (this process) <-> DEALER echo process over the native
transport, without the framework's protocol or exec on top — what a ``%%distributed`` round
trip pays for wake-ups and thread hand-offs alone.

    python benchmarks/transport_pingpong.py [--n 3000] [--endpoint ipc|tcp]

Cases (each: p50 / p90 of n round trips of a 64-byte message):
  * ``direct``  — the coordinator's main thread receives the reply itself;
  * ``thread``  — a receive thread gets it and hands it over with a threading.Event;
  * ``threadspin`` — as ``thread``, the waiting thread polling the Event (GIL yielded) for up to
                  200 us before sleeping on it;
each with the receiver poll window (``NBD_OPT_RECV_SPIN_US``) and the I/O thread poll window
(``NBD_OPT_IO_SPIN_US``) off and on, on both ends.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nbdistributed_amd.transport import (DEALER, OPT_IO_SPIN_US, OPT_RECV_SPIN_US, ROUTER,  # noqa: E402
                                         Socket)

ECHO = r"""
import sys
sys.path.insert(0, sys.argv[1])
from nbdistributed_amd.transport import DEALER, OPT_IO_SPIN_US, OPT_RECV_SPIN_US, Socket
s = Socket(DEALER, identity=b"echo")
s.set_int(OPT_RECV_SPIN_US, int(sys.argv[3]))
s.set_int(OPT_IO_SPIN_US, int(sys.argv[4]))
s.connect(sys.argv[2])
s.send([b"hello"])
while True:
    for m in s.recv_batch(timeout=None):
        if m.frames[0] == b"bye":
            s.close()
            sys.exit(0)
        s.send(m.frames)
"""


def run_case(endpoint, n, recv_spin, io_spin, mode):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = Socket(ROUTER, mandatory=True)
    r.set_int(OPT_RECV_SPIN_US, recv_spin)
    r.set_int(OPT_IO_SPIN_US, io_spin)
    ep = r.bind(endpoint)
    child = subprocess.Popen([sys.executable, "-c", ECHO, root, ep, str(recv_spin), str(io_spin)])
    try:
        while True:  # the hello
            b = r.recv_batch(timeout=30)
            if any(not m.is_event for m in b):
                break
        payload = b"x" * 64
        ev = threading.Event()
        stop = [False]
        if mode in ("thread", "threadspin"):
            def pump():
                while not stop[0]:
                    for m in r.recv_batch(timeout=0.2):
                        if not m.is_event:
                            ev.set()
            th = threading.Thread(target=pump, daemon=True)
            th.start()
        ts = []
        for i in range(n + 200):
            t0 = time.perf_counter()
            r.send([b"echo", payload])
            if mode == "thread":
                ev.wait()
                ev.clear()
            elif mode == "threadspin":  # yield the GIL in a bounded poll before sleeping on the Event
                end = t0 + 200e-6
                while not ev.is_set() and time.perf_counter() < end:
                    time.sleep(0)
                ev.wait()
                ev.clear()
            else:
                got = False
                while not got:
                    got = any(not m.is_event for m in r.recv_batch(timeout=None))
            if i >= 200:
                ts.append(time.perf_counter() - t0)
        stop[0] = True
        r.send([b"echo", b"bye"])
        child.wait(10)
    finally:
        if child.poll() is None:
            child.kill()
        r.close()
    ts.sort()
    return {"mode": mode, "recv_spin_us": recv_spin, "io_spin_us": io_spin,
            "p50_us": round(ts[len(ts) // 2] * 1e6, 1), "p90_us": round(ts[int(len(ts) * 0.9)] * 1e6, 1),
            "min_us": round(ts[0] * 1e6, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=3000)
    ap.add_argument("--endpoint", default="ipc", choices=["ipc", "tcp"])
    ap.add_argument("--modes", default="thread,threadspin,direct")
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="nbdpp-", dir="/tmp")
    ep = f"ipc://{d}/pp.sock" if a.endpoint == "ipc" else "tcp://127.0.0.1:0"
    for mode in a.modes.split(","):
        for rs, io in ((0, 0), (200, 0), (0, 200), (200, 200)):
            print(json.dumps(run_case(ep, a.n, rs, io, mode)), flush=True)


if __name__ == "__main__":
    main()
