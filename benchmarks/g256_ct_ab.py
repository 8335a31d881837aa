#!/usr/bin/env python3
"""256x256 kernel (gemm256.hip) schedule variants on the three layouts, against the 128x128 8-wave kernel and hipBLASLt — same process, random operands,
interleaved rounds (cdna_hip_programming.md §5.4 rules 24/25).  Each HIP variant's result is
checked against an fp32 torch product of the same bf16 operands.

    python benchmarks/g256_ct_ab.py [--rounds 3] [--iters 10] [--shapes lm,sq,gpt2] [--variants 4,0]

Round 5 ran it with two temporary variants 6 / 7 (= 4 / 0 with each operand half a contiguous
128-row / 128-column block instead of bands of 64 rows / 32 columns, so a transposed image's DMA
reads whole 256-B runs per k-row): no gain on any layout, removed (docs/FINDINGS.md §33,
profiles/g256_contig_halves_ab_r5.txt); and with a temporary persistent variant 6 (one workgroup
per CU walking the tiles, C stored straight from the accumulators): slower on the LM-head forward,
removed (profiles/g256_persistent_ab_r5.txt).  Variant 6 now = 4 with non-temporal C stores.
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from nbdistributed_amd import ops  # noqa: E402
from nbdistributed_amd.ops import gemm as G  # noqa: E402


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default="lm,sq,gpt2")
    ap.add_argument("--variants", default="4,0")
    a = ap.parse_args()
    ops.load_library()
    V = 50432
    groups = set(a.shapes.split(","))
    shapes = []
    if "sq" in groups:
        shapes += [("sq4096 nt", 4096, 4096, 4096, False, False, (1,)),
                   ("sq4096 dgrad", 4096, 4096, 4096, False, True, (1,)),
                   ("sq4096 wgrad", 4096, 4096, 4096, True, True, (1,))]
    if "lm" in groups:
        shapes += [("lm fwd", 8192, V, 768, False, False, (1,)),
                   ("lm dgrad", 8192, 768, V, False, True, (2, 4, 8)),
                   ("lm wgrad", V, 768, 8192, True, True, (1, 2))]
    if "gpt2" in groups:
        shapes += [("c_fc dgrad", 8192, 768, 3072, False, True, (1, 2, 4)),
                   ("c_fc wgrad", 3072, 768, 8192, True, True, (1, 2, 4)),
                   ("c_attn fwd", 8192, 2304, 768, False, False, (1,))]
    variants = [int(v) for v in a.variants.split(",")]
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, N, K, a_km, b_kn, splits in shapes:
        A = (torch.rand(*((K, M) if a_km else (M, K)), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(*((K, N) if b_kn else (N, K)), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        At = A.t() if a_km else A
        Bt = B if b_kn else B.t()
        ref = At.float() @ Bt.float()
        scale = ref.abs().max().item()
        arms = {"hipblaslt": lambda: torch.mm(At, Bt)}
        for s in splits:
            if (K // s) % 64 == 0:
                arms[f"t128x128/s{s}"] = (lambda s=s: G.matmul(A, B, a_km=a_km, b_kn=b_kn, tile=82128128, splits=s))
                if M % 256 == 0 and N % 256 == 0:
                    for v in variants:
                        arms[f"g256v{v}/s{s}"] = (lambda s=s, v=v: G.matmul(A, B, a_km=a_km, b_kn=b_kn,
                                                                           tile=80256256 + (v + 2) * 1000000, splits=s))
        errs = {}
        for k, fn in arms.items():
            out = fn()
            torch.cuda.synchronize()
            errs[k] = ((out.float() - ref).abs().max().item()) / scale
        ts = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                fn()
                ts[k].append(timed(fn, a.iters))
        flop = 2.0 * M * N * K
        row = sorted(((statistics.median(v), k) for k, v in ts.items()))
        print(f"{name:14s} M={M} N={N} K={K}", flush=True)
        for t, k in row:
            print(f"    {k:16s} {t:9.1f} us {flop / t / 1e6:7.0f} TF/s  err {errs[k]:.1e}", flush=True)
        del A, B, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
