"""Ring attention (parallel.context) on one GPU: the zigzag layout at world size 1 runs the same
block decomposition, LSE merge and merged-LSE backward as a real ring (minus the transfers), so
its time over plain flash attention on the whole sequence is the ring's compute overhead.

    python benchmarks/ring_bench.py [--T 8192 16384 32768]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from nbdistributed_amd import ops
from nbdistributed_amd.parallel.context import ring_attention


def _time(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, nargs="+", default=[4096, 16384, 32768])
    ap.add_argument("--H", type=int, default=12)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for T in args.T:
        q, k, v, do = (torch.randn(1, args.H, T, 64, device=dev, dtype=torch.bfloat16) for _ in range(4))
        for t in (q, k, v):
            t.requires_grad_(True)

        def flash():
            ops.flash_attention(q, k, v, causal=True).backward(do)

        def ring():
            ring_attention(q, k, v, causal=True, layout="zigzag").backward(do)

        tf, tr = _time(flash), _time(ring)
        flops = 4 * args.H * T * T * 64 / 2 * 3.5  # causal fwd (2 GEMMs) + bwd (5 GEMMs)
        print(json.dumps({"T": T, "H": args.H, "flash_fwd_bwd_ms": round(tf, 3), "ring_zigzag_fwd_bwd_ms": round(tr, 3),
                          "ring_overhead": round(tr / tf, 3), "flash_tflops": round(flops / tf / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
