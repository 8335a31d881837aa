#!/usr/bin/env python3
"""Forced-kernel A/B for the forward Linear products: every listed tile hint against the tuned
choice (ops/gemm.py ``config``) and torch/hipBLASLt, back-to-back launches timed with HIP events
(gemm_bench.timeit_pipelined), with a numerics check of each hint against torch.

    python benchmarks/gemm_tile_ab.py [--hints 82128192,83128192] [--gelu] [--shape M,N,K]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from benchmarks.gemm_bench import timeit_pipelined  # noqa: E402
from nbdistributed_amd.ops import gemm as G  # noqa: E402

SHAPES = (("gpt2.c_attn", 8192, 2304, 768), ("gpt2.attn.c_proj", 8192, 768, 768), ("gpt2.c_fc", 8192, 3072, 768),
          ("gpt2.mlp.c_proj", 8192, 768, 3072))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hints", default="82128192,83128192")
    ap.add_argument("--gelu", action="store_true", help="bias + GELU epilogue (the c_fc forward's)")
    ap.add_argument("--shape", default="", help="M,N,K: this product only (e.g. the LM head 8192,50688,768)")
    a = ap.parse_args()
    from nbdistributed_amd import ops

    ops.load_library()
    dev = torch.device("cuda")
    hints = [int(h) for h in a.hints.split(",") if h]
    epi = G.EPI_GELU if a.gelu else G.EPI_NONE
    shapes = SHAPES
    if a.shape:
        M_, N_, K_ = (int(v) for v in a.shape.split(","))
        shapes = (("shape", M_, N_, K_),)
    for name, M, N, K in shapes:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        bias = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16) if a.gelu else None
        flop = 2.0 * M * N * K

        def tfn():
            y = torch.addmm(bias, x, w.t()) if bias is not None else x @ w.t()
            return torch.nn.functional.gelu(y, approximate="tanh") if a.gelu else y

        ref = tfn().float()
        tuned = G.config(False, False, M, N, K, can_split=not a.gelu, epi=epi)
        row = [f"{name:17s} M={M} N={N} K={K}", f"torch {timeit_pipelined(tfn) * 1e3:6.1f}",
               f"tuned{tuned} {timeit_pipelined(lambda: G.matmul(x, w, bias=bias, epi=epi)) * 1e3:6.1f}"]
        for h in hints:
            try:
                def fn():
                    return G.matmul(x, w, bias=bias, epi=epi, tile=h, splits=1)
                out = fn()
                out = out[0] if isinstance(out, tuple) else out
                err = float((out.float() - ref).abs().max() / ref.abs().max())
                t = timeit_pipelined(fn)
                row.append(f"{h} {t * 1e3:6.1f} us ({flop / t / 1e9:6.1f} TF/s, err {err:.1e})")
            except RuntimeError as e:
                row.append(f"{h} n/a ({str(e).splitlines()[0][:60]})")
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
