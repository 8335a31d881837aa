#!/usr/bin/env python3
"""Column-split forward GEMMs: the columns that make whole rounds of 256x256 tiles (one per CU)
on the 8-phase 256x256 kernel (gemm256.hip), the remaining columns on the 128x128 family — two
launches — against the tuned single kernel and hipBLASLt, for GPT-2 small's q|k|v (N = 2304 =
2048 + 256) and c_fc (+ GELU, N = 3072 = 2048 + 1024) forwards at 8192 tokens.  Back-to-back
launches between two events (GPU time), median of rounds; random bf16 data.

    python benchmarks/gemm_colsplit.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nbdistributed_amd.ops import gemm as G  # noqa: E402

T256 = 86256256


def bench(fn, reps=20, rounds=7, warm=5):
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
    return statistics.median(ts)


def main():
    M, K = 8192, 768
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    for name, N, N0, epi in (("c_attn", 2304, 2048, G.EPI_NONE), ("c_fc", 3072, 2048, G.EPI_GELU),
                             ("c_fc_plain", 3072, 2048, G.EPI_NONE)):
        w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        b = (torch.randn(N, device="cuda") * 0.02).to(torch.bfloat16)
        w0, w1, b0, b1 = w[:N0].contiguous(), w[N0:].contiguous(), b[:N0].contiguous(), b[N0:].contiguous()
        fl = 2.0 * M * N * K
        res = {}
        res["tuned"] = bench(lambda: G.matmul(x, w, bias=b, epi=epi))
        if epi == G.EPI_NONE:
            res["hipblaslt"] = bench(lambda: torch.addmm(b, x, w.t()))
        else:
            res["hipblaslt+gelu"] = bench(lambda: torch.nn.functional.gelu(torch.addmm(b, x, w.t()), approximate="tanh"))
        res["g256_head"] = bench(lambda: G.matmul(x, w0, bias=b0, epi=epi, tile=T256, splits=1))
        for tt in (82128128, 2128128, 2128096 if epi == G.EPI_NONE else 82128128):
            try:
                res[f"tail_{tt}"] = bench(lambda: G.matmul(x, w1, bias=b1, epi=epi, tile=tt, splits=1))
            except Exception as e:  # noqa: BLE001
                res[f"tail_{tt}"] = float("nan")
                print("tail", tt, e)
        for tt in (82128128, 2128128):
            res[f"split_{tt}"] = bench(lambda: (G.matmul(x, w0, bias=b0, epi=epi, tile=T256, splits=1),
                                                G.matmul(x, w1, bias=b1, epi=epi, tile=tt, splits=1)))
        res["g256_full"] = bench(lambda: G.matmul(x, w, bias=b, epi=epi, tile=T256, splits=1)) if N % 256 == 0 else 0
        print(f"{name} M={M} N={N} K={K} (head {N0}):  " + "  ".join(
            f"{k} {v:.1f}us ({fl / v / 1e6:.0f} TF/s)" if "head" not in k and "tail" not in k and v == v and v > 0
            else f"{k} {v:.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
