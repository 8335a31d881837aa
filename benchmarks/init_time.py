#!/usr/bin/env python3
"""Time %dist_init (session start to every rank READY) and each worker's bring-up phases.

    python benchmarks/init_time.py [-n 1] [--repeat 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nbdistributed_amd.session import Session  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", type=int, default=1)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--backend", default="auto")
    a = ap.parse_args()
    out = []
    for i in range(a.repeat):
        s = Session(writer=lambda t: None)
        t = time.perf_counter()
        ready = s.start(a.n, backend=a.backend)
        total = time.perf_counter() - t
        t = time.perf_counter()
        s.execute("1", render=False)
        first = time.perf_counter() - t
        out.append({"dist_init_s": total, "first_cell_ms": first * 1e3,
                    "rank0": {k: ready[0].get(k) for k in ("init_s", "init_phases", "process_start_to_ready_s", "backend")}})
        s.shutdown()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
