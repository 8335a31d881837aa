#!/usr/bin/env python3
"""Per-kernel timeline of graph-replayed decode steps from a rocprofv3 database (run_results.db):
one token's kernels with durations, and a per-family total.

    python benchmarks/decode_timeline.py gpurun_out/prof_gen/run_results.db [--skip 300] [--out FILE]
"""
from __future__ import annotations

import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="decode_kernel")
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--occurrence", type=int, default=1, help="which decode run (graph runs of B=1 come first)")
    ap.add_argument("--skip", type=int, default=20, help="decode steps skipped inside the run")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = list(cur.execute("select start, end, name, grid_x, workgroup_x from kernels order by start"))
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    # runs of decode kernels separated by > 1 ms (generate calls, capture warm-ups)
    runs, cur_run = [], [marks[0]]
    for i in marks[1:]:
        if rows[i][0] - rows[cur_run[-1]][1] > 1e6:
            runs.append(cur_run)
            cur_run = []
        cur_run.append(i)
    runs.append(cur_run)
    run = runs[min(a.occurrence, len(runs) - 1)]
    first = run[a.skip * a.layers]
    nxt = run[(a.skip + 1) * a.layers]
    seq = rows[first:nxt]
    span = seq[-1][1] - seq[0][0]
    fam = defaultdict(lambda: [0, 0.0])
    lines = [f"# one decode step ({len(seq)} kernels, {span / 1e3:.1f} us from first attention to the next)", "",
             "| t (us) | dur (us) | grid/wg | kernel |", "|---|---|---|---|"]
    t0 = seq[0][0]
    for s, e, n, g, w in seq:
        lines.append(f"| {(s - t0) / 1e3:.1f} | {(e - s) / 1e3:.2f} | {g}/{w} | `{n[:80]}` |")
        key = n.split("(")[0].split("<")[0][:60]
        fam[key][0] += 1
        fam[key][1] += (e - s) / 1e3
    lines += ["", "| kernel | count | total us |", "|---|---|---|"]
    for k, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| `{k}` | {c} | {t:.1f} |")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        open(a.out, "w").write(text)


if __name__ == "__main__":
    main()
