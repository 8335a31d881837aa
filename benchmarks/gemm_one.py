#!/usr/bin/env python3
"""Run one GEMM product repeatedly (for rocprofv3 counter passes).

    python benchmarks/gemm_one.py M N K [--tile T] [--epi 0|1|2] [--layout fwd|dgrad|wgrad] [--iters 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nbdistributed_amd.ops import gemm as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--epi", type=int, default=0)
    ap.add_argument("--layout", default="fwd")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from nbdistributed_amd import ops

    ops.load_library()
    a_km, b_kn = {"fwd": (False, False), "dgrad": (False, True), "wgrad": (True, True)}[a.layout]
    M, N, K = a.M, a.N, a.K
    A = (torch.rand(*((K, M) if a_km else (M, K)), device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(*((K, N) if b_kn else (N, K)), device="cuda") * 0.2 - 0.1).to(torch.bfloat16)
    aux = (torch.rand(M, N, device="cuda") * 2 - 1).to(torch.bfloat16) if a.epi == G.EPI_DGELU else None
    bias = torch.zeros(N, device="cuda", dtype=torch.bfloat16) if a.epi == G.EPI_GELU else None
    fn = lambda: G.matmul(A, B, a_km=a_km, b_kn=b_kn, epi=a.epi, aux=aux, bias=bias, tile=a.tile, splits=1)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    e.synchronize()
    us = s.elapsed_time(e) / a.iters * 1e3
    print(f"{a.layout} {M}x{N}x{K} tile {a.tile} epi {a.epi}: {us:.1f} us, {2.0 * M * N * K / us / 1e6:.0f} TF/s")


if __name__ == "__main__":
    main()
