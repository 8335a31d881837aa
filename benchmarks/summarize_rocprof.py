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


def short(name: str, n: int = 110) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name) if name.startswith("void ") or "(" in name else name
    return name if len(name) <= n else name[: n - 3] + "..."


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
    for path in stats:
        rows = list(csv.DictReader(open(path)))
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
