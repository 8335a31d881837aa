#!/usr/bin/env python3
"""Print the kernel sequence of the last N dispatches of a rocprofv3 ``--kernel-trace`` CSV run
(one graph replay of a step): name, grid, duration and the idle gap before each kernel, plus a
count of the rocclr copy / fill kernels and the kernels next to them — where a step's
``__amd_rocclr_copyBuffer`` / ``fillBufferAligned`` come from.

    python benchmarks/trace_sequence.py gpurun_out/prof_dir [--last 700] [--marker adamw_flat]
"""
import argparse
import collections
import csv
import glob
import os
import re


def short(n: str, k: int = 70) -> str:
    n = re.sub(r"\(.*", "", n.replace("void ", ""))
    return n if len(n) <= k else n[: k - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--last", type=int, default=700)
    ap.add_argument("--full", action="store_true", help="print every kernel of the window")
    a = ap.parse_args()
    paths = glob.glob(os.path.join(a.prof_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for p in paths:
        for r in csv.DictReader(open(p)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r.get("Grid_Size_X") or 0)))
    rows.sort()
    win = rows[-a.last:]
    print(f"{len(rows)} dispatches; window = last {len(win)}, {(win[-1][1] - win[0][0]) / 1e3:.1f} us")
    busy = sum(e - s for s, e, _, _ in win)
    print(f"busy {busy / 1e3:.1f} us, idle {(win[-1][1] - win[0][0] - busy) / 1e3:.1f} us")
    cnt = collections.Counter()
    ctx = collections.Counter()
    prev_end = None
    for i, (s, e, n, g) in enumerate(win):
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = e
        if "rocclr" in n or a.full:
            before = short(win[i - 1][2], 50) if i else "-"
            after = short(win[i + 1][2], 50) if i + 1 < len(win) else "-"
            if "rocclr" in n:
                cnt[(short(n, 40), g)] += 1
                ctx[(short(n, 30), before, after)] += 1
            if a.full:
                print(f"{i:5d} {short(n):72s} grid {g:9d} {(e - s) / 1e3:8.2f} us  gap {gap:6.2f}")
    print("\nrocclr kernels (name, grid): count")
    for k, v in cnt.most_common():
        print(f"  {k}: {v}")
    print("\nrocclr kernels by neighbours (kernel, before, after): count")
    for k, v in ctx.most_common(30):
        print(f"  {v:4d}  {k}")


if __name__ == "__main__":
    main()
