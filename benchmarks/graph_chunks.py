#!/usr/bin/env python3
"""What a HIP graph launch costs the GPU: the same N tiny kernels replayed as ONE graph, as
N / k graphs of k kernels (launched back to back, like the per-block graphs of the eager Llama
step: ops.block_graphs, docs/FINDINGS.md §30), and issued eagerly — µs per kernel and the implied
extra GPU time per graph launch.  Kernels: in-place adds on 64 K elements (≈ the per-block
kernels' latency class).

    python benchmarks/graph_chunks.py [--n 420] [--k 7,14,35]
"""
from __future__ import annotations

import argparse

import torch


_BIG = None


def timed(run, reps: int = 7, ahead: bool = False) -> float:
    """Best GPU span of `run` in µs.  ahead: a ≈1 ms matmul is queued first and the span starts
    after it, so the host has issued everything before the GPU gets there (GPU cost alone)."""
    global _BIG
    if ahead and _BIG is None:
        _BIG = torch.randn(6144, 6144, device="cuda", dtype=torch.bfloat16)
    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(reps):
        if ahead:
            for _ in range(4):
                torch.mm(_BIG, _BIG)
        a.record()
        run()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b))
    return best * 1e3  # µs


def capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=420)
    ap.add_argument("--k", default="7,14,35")
    ap.add_argument("--numel", type=int, default=1 << 16)
    a = ap.parse_args()
    x = torch.zeros(a.numel, device="cuda")

    def kernels(m):
        def fn():
            for _ in range(m):
                x.add_(1.0)
        return fn

    for ahead in (False, True):
        tag = "GPU-only (host ahead)" if ahead else "as issued"
        eager = timed(kernels(a.n), ahead=ahead)
        one = capture(kernels(a.n))
        t_one = timed(one.replay, ahead=ahead)
        print(f"[{tag}] {a.n} kernels: eager {eager / a.n:.2f} us/kernel, one graph {t_one / a.n:.2f} us/kernel",
              flush=True)
        for k in [int(v) for v in a.k.split(",")]:
            gs = [capture(kernels(k)) for _ in range(a.n // k)]

            def run(gs=gs):
                for g in gs:
                    g.replay()

            t = timed(run, ahead=ahead)
            per_launch = (t - t_one) / len(gs)
            print(f"[{tag}] {len(gs)} graphs x {k} kernels: {t / a.n:.2f} us/kernel, +{per_launch:.2f} us per graph "
                  f"launch over one graph", flush=True)


if __name__ == "__main__":
    main()
