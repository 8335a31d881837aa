#!/usr/bin/env python3
"""256x256 phase-interleaved GEMM (gemm256.hip) vs the 128x128 family (gemm.hip) vs hipBLASLt on
large products: square 4096/8192 and the GPT-2 LM head (8192 tokens x padded vocab x 768) in its
three layouts.  Random bf16 operands (zero-filled ones read high: cdna_hip_programming.md §5.4
rule 25); interleaved rounds in one process (rule 24); median of the per-round medians.

    python benchmarks/gemm256_bench.py [--rounds 3] [--iters 20]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from nbdistributed_amd.ops import gemm as G  # noqa: E402


def bench(fn, iters):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


G256_VARIANTS = [int(v) for v in os.environ.get("NBD_G256_VARIANTS", "0").split(",")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="all")
    a = ap.parse_args()
    from nbdistributed_amd import ops

    ops.load_library()
    V = int(os.environ.get("NBD_VOCAB_PAD", "50432"))
    shapes = [
        ("sq4096 fwd", 4096, 4096, 4096, False, False),
        ("sq8192 fwd", 8192, 8192, 8192, False, False),
        ("lmhead fwd", 8192, V, 768, False, False),
        ("lmhead dgrad", 8192, 768, V, False, True),
        ("lmhead wgrad", V, 768, 8192, True, True),
        ("gpt2 c_fc fwd", 8192, 3072, 768, False, False),
        # Llama-3.2-1B-class Linear forwards at 8192 tokens (hidden 2048, q|k|v 3072, MLP 8192)
        ("llama1b qkv", 8192, 3072, 2048, False, False),
        ("llama1b o_proj", 8192, 2048, 2048, False, False),
        ("llama1b down", 8192, 2048, 8192, False, False),
    ]
    only = None if a.shapes == "all" else set(a.shapes.split(","))
    shapes = [sh for sh in shapes if only is None or sh[0].split()[0] in only]
    g = torch.Generator(device="cuda").manual_seed(0)
    res = {}
    for name, M, N, K, a_km, b_kn in shapes:
        A = (torch.rand(*((K, M) if a_km else (M, K)), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(*((K, N) if b_kn else (N, K)), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        At = A.t() if a_km else A
        Bt = B if b_kn else B.t()
        flop = 2.0 * M * N * K
        variants = {"hipblaslt": lambda: torch.mm(At, Bt)}
        for tile in (2128128, 82128128):
            if M % 128 == 0 and N % 128 == 0:
                for s in (1, 2, 4, 8):
                    if (K // s) % 64 == 0 and (s == 1 or K >= 4096):
                        variants[f"t{tile}/s{s}"] = (lambda t=tile, s=s: G.matmul(A, B, a_km=a_km, b_kn=b_kn, tile=t, splits=s))
        if M % 256 == 0 and N % 256 == 0:
            for v in G256_VARIANTS:
                for s in (1, 2, 4, 8):
                    if (K // s) % 64 == 0 and (s == 1 or K >= 4096):
                        variants[f"g256v{v}/s{s}"] = (lambda s=s, v=v: G.matmul(A, B, a_km=a_km, b_kn=b_kn,
                                                                               tile=80256256 + (v + 2) * 1000000, splits=s))
        ref = torch.mm(At.float(), Bt.float()) if M * N * K <= 8192 * 8192 * 768 else None
        for vn, fn in variants.items():
            if ref is not None and vn != "hipblaslt":
                err = float((fn().float() - ref).abs().max() / ref.abs().max())
                if err > 1e-2:
                    print(f"{name} {vn}: WRONG err {err:.3e}", flush=True)
        times = {vn: [] for vn in variants}
        for _ in range(a.rounds):
            for vn, fn in variants.items():
                times[vn].append(bench(fn, a.iters))
        row = {vn: statistics.median(ts) for vn, ts in times.items()}
        res[name] = row
        best = min(row, key=row.get)
        line = "  ".join(f"{vn} {t:7.1f}us {flop / t / 1e6:6.0f}TF" for vn, t in sorted(row.items(), key=lambda kv: kv[1]))
        print(f"{name:14s} M={M} N={N} K={K}  best {best}\n    {line}", flush=True)
        del A, B, At, Bt, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
