#!/usr/bin/env python3
"""Timeline view of a rocprofv3 kernel trace: GPU busy vs idle (launch gaps) over the last N
steps, and device time by kernel family.

    python benchmarks/trace_gaps.py PROF_DIR [--marker SUBSTR] [--steps 5] [--out FILE.md]

A "step" boundary is each launch of the kernel whose name contains --marker (default: the AdamW
kernel, launched once per bucket: the first of each consecutive run counts).
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict

FAMILIES = [
    ("gemm (nbd)", r"nbd::gemm::gemm_kernel|nbd::gemm::g256|nbd::gemm::pair_kernel"),
    ("gemm (hipBLASLt)", r"^Cijk_|^Custom_Cijk"),
    ("gemm split-K reduce", r"nbd::gemm::reduce_kernel"),
    ("attention", r"nbd::attn::"),
    ("layer/rms norm", r"nbd::norm::"),
    ("cross-entropy", r"xent"),
    ("optimizer", r"adamw|nbd::optim"),
    ("embedding", r"nbd::embed::"),
    ("bucket / copy", r"nbd::multi_copy|bucket|copyBuffer|fillBuffer"),
    ("rccl", r"ncclDevKernel|rccl|nccl"),
    ("torch elementwise", r"at::native::"),
]


def family(name: str) -> str:
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--marker", default="adamw_flat_kernel")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.prof_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # step boundaries: first marker kernel of each run of marker kernels
    starts = []
    prev_marker = False
    for i, (s, e, n) in enumerate(rows):
        m = a.marker in n
        if m and not prev_marker:
            starts.append(i)
        prev_marker = m
    if len(starts) < a.steps + 1:
        raise SystemExit(f"only {len(starts)} step markers found")
    lo, hi = starts[-a.steps - 1], starts[-1]
    sel = rows[lo:hi]
    span = sel[-1][1] - sel[0][0]
    # busy = union of kernel intervals
    busy = 0
    cur_s, cur_e = sel[0][0], sel[0][1]
    gaps = []
    for s, e, n in sel[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    fam = defaultdict(float)
    for s, e, n in sel:
        fam[family(n)] += (e - s)
    steps = a.steps
    lines = [f"# GPU timeline over the last {steps} steps ({os.path.basename(a.prof_dir)})", "",
             f"* kernels per step: {len(sel) / steps:.0f}",
             f"* span per step: {span / steps / 1e6:.3f} ms; GPU busy (union of kernels) {busy / steps / 1e6:.3f} ms "
             f"({100 * busy / span:.1f} %); idle {(span - busy) / steps / 1e6:.3f} ms in {len(gaps) / steps:.0f} gaps",
             f"* gaps > 5 us per step: {sum(1 for g, _ in gaps if g > 5000) / steps:.1f} "
             f"({sum(g for g, _ in gaps if g > 5000) / steps / 1e3:.1f} us)", "",
             "| family | ms / step | % of kernel time |", "|---|---|---|"]
    tot = sum(fam.values())
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        lines.append(f"| {k} | {v / steps / 1e6:.3f} | {100 * v / tot:.1f} |")
    lines += ["", "Largest gaps (before kernel):", ""]
    for g, n in sorted(gaps, reverse=True)[:10]:
        lines.append(f"* {g / 1e3:.1f} us before `{n[:100]}`")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
