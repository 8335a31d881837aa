#!/usr/bin/env python3
"""A/B: the LM head's weight gradient (hipBLASLt, dlogitsᵀ·h, 50304 x 768 x 8192 bf16) written
into a fresh tensor vs straight into a slice of a larger bucket buffer (``out=``, what DDP's
gradient views do, ops/graddst.py), interleaved rounds in one process.

    python benchmarks/lmhead_out_ab.py [--rounds 4] [--iters 10]
"""
import argparse

import torch


def _t(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    N, V, C = 8192, 50304, 768
    g = torch.Generator(device="cuda").manual_seed(0)
    dl = (torch.randn(N, V, device="cuda", generator=g) * 1e-3).to(torch.bfloat16)
    h = torch.randn(N, C, device="cuda", generator=g).to(torch.bfloat16)
    bucket = torch.zeros(V * C + 4096 + 64, device="cuda", dtype=torch.bfloat16)
    arms = {}
    for off in (0, 64, 4096):  # element offsets of the slice in the bucket (64 = 128 B, the planner's alignment)
        view = bucket[off:off + V * C].view(V, C)
        arms[f"out=bucket[{off}:]"] = lambda v=view: torch.mm(dl.t(), h, out=v)
    arms["fresh"] = lambda: torch.mm(dl.t(), h)
    fresh_buf = torch.empty(V, C, device="cuda", dtype=torch.bfloat16)
    arms["out=fresh"] = lambda: torch.mm(dl.t(), h, out=fresh_buf)
    arms["fresh+copy"] = lambda: bucket[64:64 + V * C].view(V, C).copy_(torch.mm(dl.t(), h))
    res = {k: [] for k in arms}
    for _ in range(a.rounds):
        for k, fn in arms.items():
            res[k].append(_t(fn, a.iters))
    flops = 2.0 * N * V * C
    for k, ts in res.items():
        print(f"{k:22s} " + " ".join(f"{t:7.1f}" for t in ts) + f"  best {min(ts):.1f} us {flops / min(ts) / 1e6:.0f} TF/s")


if __name__ == "__main__":
    main()
