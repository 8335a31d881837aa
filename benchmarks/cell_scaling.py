#!/usr/bin/env python3
"""Trivial-cell round trip vs world size (1..8 ranks) — the control plane's fan-out/fan-in cost.

    HIP_VISIBLE_DEVICES= python benchmarks/cell_scaling.py [--steps 500] [--loop-send]

Workers use the gloo backend (no GPU), so this isolates the coordinator <-> worker path that
bench.py's headline `%%distributed` p50 measures at N GPUs.  ``--loop-send`` A/Bs the native
multicast (one `nbd_send_multi` call per cell) against one `nbd_send` per rank.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nbdistributed_amd.benchmarking import bench_cells  # noqa: E402
from nbdistributed_amd.session import Session  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--loop-send", action="store_true")
    a = ap.parse_args()
    out = {}
    for n in [int(x) for x in a.worlds.split(",")]:
        s = Session(writer=lambda t: None)
        s.start(n, backend="gloo")
        try:
            if a.loop_send:
                sock = s.comm.sock

                def loop(idents, frames, sock=sock):
                    st = []
                    for i in idents:
                        try:
                            sock.send([i] + list(frames))
                            st.append(0)
                        except Exception:
                            st.append(2)
                    return st

                sock.send_multi = loop
            bench_cells(s, 50, 10)
            r = bench_cells(s, a.steps, 0)
            out[n] = {k: round(v, 4) for k, v in r.items() if k.endswith("_ms")}
            print(n, out[n], flush=True)
        finally:
            s.shutdown()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
