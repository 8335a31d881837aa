"""Host cost of one kernel launch on this stack (``torch.ops.nbd.launch_probe``, csrc/kernels/probe.hip).

    python benchmarks/launch_probe.py [--n 20000]

Modes: 0 hipLaunchKernelGGL (16-B args), 1 GEMM-sized args (256 B), 2 hipModuleLaunchKernel
(function resolved once, packed argument buffer), 3 = 0 + device guard + stream getter +
error check, 4 = 3 + an at::empty, 5 = 0 with an 8 x 256 grid.  Also times a torch op launch
(``torch.add`` into a preallocated output) from Python for scale.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nbdistributed_amd.ops import _lib  # noqa: E402

NAMES = {0: "ggl_small", 1: "ggl_big_args", 2: "module_launch", 3: "ggl+guard+stream+check", 4: "…+at::empty",
         5: "ggl_grid8x256"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    a = ap.parse_args()
    assert _lib.load_library(), _lib._load_error
    x = torch.zeros(1024, device="cuda")
    out = {}
    for rep in range(2):
        for mode, name in NAMES.items():
            us = torch.ops.nbd.launch_probe(x, a.n, mode)
            out[name] = round(us, 3)
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.n):
            torch.add(x, 1.0, out=y)
        out["torch.add(out=) from python"] = round((time.perf_counter() - t) / a.n * 1e6, 3)
        torch.cuda.synchronize()
        print(rep, out, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
