#!/usr/bin/env python3
"""GPU busy vs idle time per training step from a rocprofv3 kernel trace: is an eager step
host-bound (the GPU waits for launches), and in which part of the step?

    python benchmarks/trace_gaps.py PROF_DIR [--marker adamw] [--steps 10]

Steps are delimited by the optimizer kernels (the last kernel whose name matches --marker before
a gap, i.e. the end of each step's update).  For the last --steps steps it prints wall time,
the union of kernel intervals (busy), idle time, and idle time split into thirds of the step
(forward-ish / early backward / late backward + update), plus the largest gaps with the kernels
around them.
"""
from __future__ import annotations

import argparse
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from trace_seq import load, short  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--marker", default="adamw")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    rows = load(a.prof_dir)
    pat = re.compile(a.marker, re.I)
    # step ends: the last marker kernel of each run of marker kernels
    ends = [i for i in range(len(rows) - 1) if pat.search(rows[i][2]) and not pat.search(rows[i + 1][2])]
    if pat.search(rows[-1][2]):
        ends.append(len(rows) - 1)
    assert len(ends) > a.steps, f"only {len(ends)} steps found"
    ends = ends[-(a.steps + 1):]
    tot_wall = tot_busy = 0.0
    thirds = [0.0, 0.0, 0.0]
    gaps = []
    for s in range(a.steps):
        lo, hi = ends[s] + 1, ends[s + 1]
        t0, t1 = rows[ends[s]][1], rows[hi][1]
        wall = t1 - t0
        busy = 0
        cur_s, cur_e = None, None
        prev_end = t0
        for i in range(lo, hi + 1):
            st, en, name = rows[i]
            if st > prev_end:
                g = st - prev_end
                frac = (prev_end - t0) / wall
                thirds[min(2, int(frac * 3))] += g
                gaps.append((g, rows[i - 1][2], name, frac))
            if cur_s is None or st > cur_e:
                if cur_s is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = st, en
            else:
                cur_e = max(cur_e, en)
            prev_end = max(prev_end, en)
        busy += cur_e - cur_s
        tot_wall += wall
        tot_busy += busy
    n = a.steps
    print(f"steps {n}: wall {tot_wall / n / 1e6:.3f} ms  busy {tot_busy / n / 1e6:.3f} ms  "
          f"idle {(tot_wall - tot_busy) / n / 1e6:.3f} ms  (idle by thirds of the step: "
          + " / ".join(f"{t / n / 1e6:.3f}" for t in thirds) + " ms)")
    gaps.sort(reverse=True)
    print(f"largest gaps (µs, position in step, kernel before -> after):")
    for g, before, after, frac in gaps[:a.top]:
        print(f"  {g / 1e3:8.1f}  {frac:4.2f}  {short(before)[:50]} -> {short(after)[:50]}")


if __name__ == "__main__":
    main()
