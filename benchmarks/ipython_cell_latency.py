#!/usr/bin/env python3
"""The trivial-cell round trip under a REAL IPython InteractiveShell.

bench.py's ``cell_magic_p50_ms`` drives the magics through ``utils.fakeshell.HeadlessShell``;
this measures the same cell through IPython's own ``run_cell`` — input transformers (auto mode
rewrites the cell to ``%%distributed``), cell-magic dispatch, the ``pre/post_run_cell`` events,
history, displayhook — with default settings (``ide_sync`` namespace delta, per-rank renderer).
The kernel side runs on /opt/conda/bin/python3.9 (IPython 7.29, no torch: the coordinator never
imports it); the workers run the PyTorch interpreter on CPU/gloo.  The reference's number for the
same cell is 111.6 ms (2 GPUs, ``00_accelerate.ipynb:1127``) and 112.7-113.6 ms measured on this
CPU box.

    python benchmarks/ipython_cell_latency.py [--ranks 1,2,4,8] [--steps 200]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nbdistributed_amd.benchmarking import IPYTHON_PY, bench_cells_ipython  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    if not os.path.exists(IPYTHON_PY):
        print("no IPython interpreter at", IPYTHON_PY, file=sys.stderr)
        return 2
    res = bench_cells_ipython([int(x) for x in a.ranks.split(",")], a.steps, a.warmup, timeout_s=1800)
    print(f"{'ranks':>5} {'auto p50':>10} {'auto p90':>10} {'%%distributed p50':>18} {'%%rank[0] p50':>14}  (ms, real IPython {sys.version.split()[0]} workers)")
    for n, d in res.items():
        print(f"{n:>5} {d['auto']['p50_ms']:10.3f} {d['auto']['p90_ms']:10.3f} {d['explicit']['p50_ms']:18.3f} "
              f"{d['rank0']['p50_ms']:14.3f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
