#!/usr/bin/env python3
"""Linear layers whose row count is off the 64-grid (B·T = 8100): the HIP
GEMMs on zero-padded rows (ops.gemm_linear, NBD_GEMM_PAD_ROWS) against F.linear (hipBLASLt),
forward + backward, interleaved; and the same at the 64-aligned 8192 for reference."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from nbdistributed_amd import ops  # noqa: E402
from nbdistributed_amd.ops import gemm as G  # noqa: E402

ops._require()
dev = torch.device("cuda")


def time_us(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


for M in (8100, 8192):
    for name, N, K in (("c_attn", 2304, 768), ("attn.c_proj", 768, 768), ("c_fc", 3072, 768), ("mlp.c_proj", 768, 3072)):
        x = torch.randn(M, K, device=dev).to(torch.bfloat16).requires_grad_()
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16).requires_grad_()
        b = torch.zeros(N, device=dev, dtype=torch.bfloat16, requires_grad=True)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)

        def hip():
            G.gemm_linear(x, w, b).backward(dy)

        def lib():
            F.linear(x, w, b).backward(dy)

        r = {"hip": [], "lib": []}
        for _ in range(3):
            r["hip"].append(round(time_us(hip), 1))
            r["lib"].append(round(time_us(lib), 1))
        print(f"M={M} {name:12s} N={N:5d} K={K:5d}  hip(padded) fwd+bwd us {r['hip']}  hipBLASLt {r['lib']}", flush=True)


# weight dims off the 64-grid (NBD_GEMM_PAD_DIMS=1 path) against the library
G.PAD_DIMS = True
for (M, N, K) in ((8192, 1000, 768), (8192, 768, 1000), (8192, 3000, 1000)):
    x = torch.randn(M, K, device=dev).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16).requires_grad_()
    b = torch.zeros(N, device=dev, dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(M, N, device=dev).to(torch.bfloat16)

    def hip():
        G.gemm_linear(x, w, b).backward(dy)

    def lib():
        F.linear(x, w, b).backward(dy)

    r = {"hip": [], "lib": []}
    for _ in range(3):
        r["hip"].append(round(time_us(hip), 1))
        r["lib"].append(round(time_us(lib), 1))
    print(f"dims M={M} N={N:5d} K={K:5d}  hip(padded) fwd+bwd us {r['hip']}  hipBLASLt {r['lib']}", flush=True)
