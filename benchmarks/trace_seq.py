#!/usr/bin/env python3
"""Kernel sequence of one step from a rocprofv3 kernel trace: where the small library kernels
(copies, fills, torch elementwise) sit between the framework's kernels.

    python benchmarks/trace_seq.py PROF_DIR [--marker adamw] [--pattern 'copyBuffer|fillBuffer|at::native']

Step = from the first kernel after the last-but-one optimizer run to the end of the last one.
Prints every kernel of that step (name shortened, duration, gap before it) and, for the kernels
matching --pattern, the kernel before and after them.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re


def short(name: str) -> str:
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"void ", "", name)
    return name[:90]


def load(prof_dir: str):
    files = glob.glob(os.path.join(prof_dir, "**", "*kernel_trace.csv"), recursive=True)
    assert files, f"no kernel_trace.csv under {prof_dir}"
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--marker", default="adamw")
    ap.add_argument("--pattern", default=r"copyBuffer|fillBuffer|at::native")
    ap.add_argument("--all", action="store_true", help="print every kernel of the step")
    a = ap.parse_args()
    rows = load(a.prof_dir)
    # optimizer runs: consecutive marker kernels
    runs, prev = [], False
    for i, (_, _, n) in enumerate(rows):
        m = a.marker in n
        if m and not prev:
            runs.append([i, i])
        if m:
            runs[-1][1] = i
        prev = m
    assert len(runs) >= 2, "need two optimizer runs"
    lo, hi = runs[-2][1] + 1, runs[-1][1] + 1
    step = rows[lo:hi]
    t0 = step[0][0]
    print(f"# step: {len(step)} kernels, {(step[-1][1] - t0) / 1e6:.3f} ms wall")
    pat = re.compile(a.pattern)
    counts = {}
    for i, (s, e, n) in enumerate(step):
        gap = (s - step[i - 1][1]) / 1e3 if i else 0.0
        if a.all:
            print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:7.1f} us  gap {gap:6.1f}  {short(n)}")
        if pat.search(n):
            k = short(n)
            counts[k] = counts.get(k, 0) + 1
            before = short(step[i - 1][2]) if i else "-"
            after = short(step[i + 1][2]) if i + 1 < len(step) else "-"
            print(f"[{i:4d}] {k}  ({(e - s) / 1e3:.1f} us)\n        after  {before}\n        before {after}")
    print("\n# matches per step")
    for k, v in sorted(counts.items(), key=lambda kv: -kv[1]):
        print(f"{v:4d}  {k}")


if __name__ == "__main__":
    main()
