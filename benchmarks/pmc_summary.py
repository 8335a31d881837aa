#!/usr/bin/env python3
"""Reduce rocprofv3 CSV output (counter_collection + kernel_trace) to a per-kernel table.

    python benchmarks/pmc_summary.py DIR [DIR ...] --out profiles/x.md [--filter nbd]

For every kernel name: dispatch count, mean duration (kernel_trace) and the mean of each counter
per dispatch (counter_collection; per-SE values are summed within a dispatch first).  Derived:
MfmaUtil (MFMA busy cycles / (GRBM_GUI_ACTIVE x 1024 SIMDs)), LDS bank-conflict cycles per LDS instruction, HBM bytes from
FETCH_SIZE/WRITE_SIZE (KiB units; FETCH under-counts wide streams on gfx950 — see
MI355X_MICROARCH.md §HBM) and the implied GB/s.
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)  # drop the parameter list
    return name[:90]


def load(dirs):
    counters = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    durs = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = (short(row["Kernel_Name"]), f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                    counters[k][row["Counter_Name"]] += float(row["Counter_Value"])
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    durs[short(row["Kernel_Name"])].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    per_kernel = defaultdict(lambda: defaultdict(list))
    for (kname, _f, _d), cs in counters.items():
        for c, v in cs.items():
            per_kernel[kname][c].append(v)
    return per_kernel, durs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", required=True)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    per_kernel, durs = load(a.dirs)
    names = sorted(set(per_kernel) | set(durs), key=lambda k: -sum(durs.get(k, [0])))
    cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_VALU_MFMA_BUSY_CYCLES",
            "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_BUSY_CYCLES", "FETCH_SIZE", "WRITE_SIZE", "GRBM_GUI_ACTIVE"]
    lines = ["| kernel | calls | mean µs | " + " | ".join(cols) + " | MfmaUtil % | LDS confl/inst | HBM GB/s (F+W) |",
             "|---" * (len(cols) + 6) + "|"]
    for k in names:
        if a.filter and not re.search(a.filter, k):
            continue
        d = durs.get(k, [])
        mean_us = sum(d) / len(d) if d else float("nan")
        c = {n: (sum(v) / len(v)) for n, v in per_kernel.get(k, {}).items()}
        gui = c.get("GRBM_GUI_ACTIVE")
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        # rocprof's MfmaUtil: MFMA busy cycles over (GPU-active cycles x SIMD count); 256 CUs x 4 SIMDs
        mfma_pct = f"{100 * mf / (gui * 1024):.2f}" if mf is not None and gui else ""
        lds = c.get("SQ_INSTS_LDS")
        confl = f"{c['SQ_LDS_BANK_CONFLICT'] / lds:.3f}" if lds and "SQ_LDS_BANK_CONFLICT" in c else ""
        hbm = ""
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c and d:
            hbm = f"{(c['FETCH_SIZE'] + c['WRITE_SIZE']) * 1024 / (mean_us * 1e3):.0f}"
        vals = [f"{c[n]:.4g}" if n in c else "" for n in cols]
        lines.append(f"| `{k}` | {len(d)} | {mean_us:.1f} | " + " | ".join(vals) + f" | {mfma_pct} | {confl} | {hbm} |")
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main()
