#!/usr/bin/env python3
"""Where a trivial %%distributed cell's round trip goes: coordinator-side cProfile over N cells,
and the worker-reported execution time (exec_s) vs the end-to-end latency.

    HIP_VISIBLE_DEVICES= python benchmarks/prof_cell.py [--cells 3000] [--world 1]
"""
import argparse
import cProfile
import os
import pstats
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nbdistributed_amd.session import Session  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=3000)
    ap.add_argument("--world", type=int, default=1)
    a = ap.parse_args()
    s = Session(writer=lambda t: None)
    s.start(a.world, backend="gloo")
    try:
        for _ in range(300):
            s.execute("1 + 1", render=False)
        rtt, ex = [], []
        for _ in range(a.cells):
            t = time.perf_counter()
            r = s.execute("1 + 1", render=False)
            rtt.append((time.perf_counter() - t) * 1e6)
            ex.append(max(v.get("exec_s", 0.0) for v in r.results.values()) * 1e6)
        print(f"world {a.world}: round trip p50 {statistics.median(rtt):.1f} us, worker exec p50 "
              f"{statistics.median(ex):.1f} us, min rtt {min(rtt):.1f} us", flush=True)
        if os.environ.get("NBD_WORKER_TIMING") == "1":
            ph = {}
            for _ in range(500):
                r = s.execute("1 + 1", render=False)
                for k, v in r.results[0].get("timing_us", {}).items():
                    ph.setdefault(k, []).append(v)
            print("worker phases p50 (us):", {k: statistics.median(v) for k, v in ph.items()}, flush=True)
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(a.cells):
            s.execute("1 + 1", render=False)
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(20)
    finally:
        s.shutdown()


if __name__ == "__main__":
    main()
