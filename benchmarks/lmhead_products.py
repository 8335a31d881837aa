#!/usr/bin/env python3
"""The GPT-2 small LM head's three products, each on the hand-written kernels and on hipBLASLt
(back-to-back launches between two events, median of rounds; random data): forward
logits = h·Wᵀ (8192 x 50688 x 768), input gradient dh = dlogits·W (split 8 ways along the
vocabulary), weight gradient dW = dlogitsᵀ·h (whole rounds + a split tail).  What
``ops.loss.HEAD_PRODUCTS`` ("auto") is chosen from.

    python benchmarks/lmhead_products.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nbdistributed_amd.ops import loss as L  # noqa: E402


def bench(fn, reps=10, rounds=5, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / reps * 1e3)
    return statistics.median(ts), min(ts)


def main():
    from nbdistributed_amd import ops

    ops._require()
    N, V, C = 8192, 50688, 768
    torch.manual_seed(0)
    h = (torch.randn(N, C, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(V, C, device="cuda") * 0.05).to(torch.bfloat16)
    dl = (torch.randn(N, V, device="cuda") * 1e-3).to(torch.bfloat16)
    out_w = torch.empty(V, C, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * N * V * C
    rows = [("fwd", lambda: L._hip_logits(h, w), lambda: torch.mm(h, w.t())),
            ("dgrad", lambda: L._hip_dgrad(dl, w), lambda: torch.mm(dl, w)),
            ("wgrad", lambda: L._hip_wgrad(dl, h, out=out_w), lambda: torch.mm(dl.t(), h, out=out_w))]
    for r in range(2):  # two interleaved rounds
        for name, hip, lib in rows:
            th, th_min = bench(hip)
            tl, tl_min = bench(lib)
            print(f"round {r} {name:6s} N={N} V={V} C={C}  hip {th:.1f} us (min {th_min:.1f}, {fl / th / 1e6:.0f} TF/s)"
                  f"  hipblaslt {tl:.1f} us (min {tl_min:.1f}, {fl / tl / 1e6:.0f} TF/s)  hip/lib {th / tl:.3f}",
                  flush=True)


if __name__ == "__main__":
    main()
