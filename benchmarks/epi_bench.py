#!/usr/bin/env python3
"""Cost of the fused GEMM epilogues on GPT-2's MLP products (c_fc forward + GELU, c_proj dgrad +
GELU'), vs the plain product, per kernel configuration.  Interleaved rounds, one process.

    python benchmarks/epi_bench.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nbdistributed_amd.ops import gemm as G  # noqa: E402


def bench(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    from nbdistributed_amd import ops

    ops.load_library()
    T, C, F = 8192, 768, 3072
    x = (torch.rand(T, C, device="cuda") * 2 - 1).to(torch.bfloat16)
    w1 = (torch.rand(F, C, device="cuda") * 0.1 - 0.05).to(torch.bfloat16)
    b1 = torch.zeros(F, device="cuda", dtype=torch.bfloat16)
    dy = (torch.rand(T, C, device="cuda") * 2 - 1).to(torch.bfloat16)
    w2 = (torch.rand(C, F, device="cuda") * 0.1 - 0.05).to(torch.bfloat16)
    pre = (torch.rand(T, F, device="cuda") * 2 - 1).to(torch.bfloat16)
    tiles = [int(t) for t in os.environ.get("TILES", "2128128,82128128").split(",")]
    cases = {}
    for t in tiles:
        cases[f"fc fwd none t{t}"] = lambda t=t: G.matmul(x, w1, bias=b1, tile=t, splits=1)
        cases[f"fc fwd gelu t{t}"] = lambda t=t: G.matmul(x, w1, bias=b1, epi=G.EPI_GELU, tile=t, splits=1)
        cases[f"proj dgrad none t{t}"] = lambda t=t: G.matmul(dy, w2, b_kn=True, tile=t, splits=1)
        cases[f"proj dgrad dgelu t{t}"] = lambda t=t: G.matmul(dy, w2, b_kn=True, epi=G.EPI_DGELU, aux=pre, tile=t, splits=1)
    res = {k: [] for k in cases}
    for _ in range(5):
        for k, fn in cases.items():
            res[k].append(bench(fn))
    for k, v in res.items():
        print(f"{k:32s} {statistics.median(v):7.1f} us", flush=True)
    # pure write bandwidth reference: 2 x [T][F] bf16 stores
    o1, o2 = torch.empty(T, F, device="cuda", dtype=torch.bfloat16), torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
    t = statistics.median([bench(lambda: (o1.fill_(1.0), o2.fill_(2.0))) for _ in range(5)])
    print(f"{'fill 2 x [8192][3072] bf16':32s} {t:7.1f} us  ({2 * o1.numel() * 2 / t / 1e6:.2f} TB/s)")


if __name__ == "__main__":
    main()
