#!/usr/bin/env python3
"""Condense a rocprofv3 ``--kernel-trace --stats`` CSV directory into a committed markdown summary.

    python benchmarks/summarize_rocprof.py gpurun_out/prof_ops profiles/ops_rocprof.md [--title T]
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
import sqlite3


def short(name: str, n: int = 110) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name) if name.startswith("void ") or "(" in name else name
    return name if len(name) <= n else name[: n - 3] + "..."


def db_rows(path):
    """rocprofv3's SQLite output (ROCm 7 default): the same per-kernel statistics as the CSV
    ``kernel_stats`` file, and the first dispatch's resources per kernel."""
    c = sqlite3.connect(path)
    q = ("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
         "from kernels group by name")
    agg = list(c.execute(q))
    total = sum(r[2] for r in agg) or 1.0
    rows = [{"Name": n, "Calls": str(k), "TotalDurationNs": str(t), "AverageNs": str(av), "MinNs": str(mn),
             "MaxNs": str(mx), "Percentage": str(100.0 * t / total)} for n, k, t, av, mn, mx in agg]
    res = {}
    for n, v, a, sg, lds, wx, gx in c.execute(
            "select name, vgpr_count, accum_vgpr_count, sgpr_count, lds_size, workgroup_x, grid_x from kernels"):
        res.setdefault(n, (v, a, sg, lds, wx, gx))
    return rows, res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("out")
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    stats = glob.glob(os.path.join(a.prof_dir, "**", "*kernel_stats.csv"), recursive=True)
    trace = glob.glob(os.path.join(a.prof_dir, "**", "*kernel_trace.csv"), recursive=True)
    lines = [f"# {a.title}", "", f"Source: `rocprofv3 --kernel-trace --stats` ({os.path.basename(a.prof_dir)})", ""]
    res = {}
    if trace:
        for r in csv.DictReader(open(trace[0])):
            nm = r["Kernel_Name"]
            if nm not in res:
                res[nm] = (r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("SGPR_Count"), r.get("LDS_Block_Size"),
                           r.get("Workgroup_Size_X"), r.get("Grid_Size_X"))
    tables = [list(csv.DictReader(open(path))) for path in stats]
    if not stats:
        for path in glob.glob(os.path.join(a.prof_dir, "**", "*.db"), recursive=True):
            rows, r2 = db_rows(path)
            tables.append(rows)
            res.update(r2)
    for rows in tables:
        total = sum(float(r["TotalDurationNs"]) for r in rows)
        ours = [r for r in rows if "nbd::" in r["Name"]]
        if ours:
            lines += ["## nbdistributed_amd HIP kernels", "",
                      "| kernel | calls | avg µs | min µs | max µs | VGPR | AGPR | SGPR | LDS B | block | grid |",
                      "|---|---|---|---|---|---|---|---|---|---|---|"]
            for r in ours:
                v = res.get(r["Name"], ("",) * 6)
                lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                             f"{float(r['MinNs']) / 1e3:.1f} | {float(r['MaxNs']) / 1e3:.1f} | {v[0]} | {v[1]} | {v[2]} | "
                             f"{v[3]} | {v[4]} | {v[5]} |")
            lines.append("")
        lines += [f"## Top {a.top} kernels by total time (all {len(rows)} kernels, {total / 1e6:.2f} ms total)", "",
                  "| kernel | calls | total ms | avg µs | % |", "|---|---|---|---|---|"]
        for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: a.top]:
            lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                         f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
        lines.append("")
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()
