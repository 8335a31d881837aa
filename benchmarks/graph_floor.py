"""Per-kernel time floor on this stack: N back-to-back tiny kernels, eager (one stream) and replayed
from one HIP graph, timed with events — what each extra kernel in a small-model step costs even
when it does (almost) nothing.

    python benchmarks/graph_floor.py [--n 500]

Kernels: a 1-element in-place add (one workgroup), the same on 1 M elements (≈1000 workgroups),
and ``torch.ops.nbd.launch_probe``'s empty kernel is not used (it syncs).  Prints µs per kernel.
"""
from __future__ import annotations

import argparse
import json

import torch


def per_kernel_us(fn, n: int, graph: bool) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        run = g.replay
    else:
        run = fn
    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(5):
        a.record()
        run()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b))
    return best * 1e3 / n


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500)
    a = ap.parse_args()
    out = {}
    for name, numel in (("1 elem", 1), ("64 K elem", 1 << 16), ("1 M elem", 1 << 20)):
        x = torch.zeros(numel, device="cuda")

        def fn(x=x):
            for _ in range(a.n):
                x.add_(1.0)

        out[name] = {"eager_us": round(per_kernel_us(fn, a.n, False), 2),
                     "graph_us": round(per_kernel_us(fn, a.n, True), 2)}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
