#!/usr/bin/env python3
"""HIP MFMA GEMM (csrc/kernels/gemm.hip) vs PyTorch/hipBLASLt on the Linear shapes of the
bench workloads: GPT-2 small (8 x 1024 tokens) and SmolLM2-135M (16 x 128 tokens).

    python benchmarks/gemm_bench.py [--json out.json] [--sweep]

For every Linear: forward y = x·Wᵀ, dgrad dx = dy·W, wgrad dW = dyᵀ·x, timed with HIP events
(median of 20 after 5 warm-up) on random bf16 data; TF/s = 2·M·N·K / time.  ``--sweep`` also
times every tile / split-K variant so the heuristic in ops/gemm.py and gemm.hip can be checked.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from nbdistributed_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def timeit_pipelined(fn, reps=20, rounds=7, warm=5):
    """GPU time per call with `reps` launches back to back between two events (each launch's host
    work overlaps the previous kernel: no launch gap inside the window), median over rounds."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / reps)
    return statistics.median(ts)


def linears():
    out = []
    T = 8 * 1024
    for name, n, k in (("gpt2.c_attn", 2304, 768), ("gpt2.attn.c_proj", 768, 768), ("gpt2.c_fc", 3072, 768),
                       ("gpt2.mlp.c_proj", 768, 3072)):
        out.append((name, T, n, k))
    T = 16 * 128
    for name, n, k in (("smollm2.qkv", 960, 576), ("smollm2.o_proj", 576, 576), ("smollm2.gate_up", 3072, 576),
                       ("smollm2.down", 576, 1536)):
        out.append((name, T, n, k))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--pipelined", action="store_true",
                    help="time back-to-back launches (GPU time, no host launch gaps) for both columns")
    ap.add_argument("--tunableop", action="store_true",
                    help="torch column with PyTorch TunableOp: hipBLASLt/rocBLAS solutions searched per shape")
    a = ap.parse_args()
    global timeit
    if a.pipelined:
        timeit = timeit_pipelined  # noqa: F811
    if a.tunableop:
        tun = torch.cuda.tunable
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_filename("/tmp/nbd_gemm_bench_tunableop.csv")
    from nbdistributed_amd import ops

    ops.load_library()
    dev = torch.device("cuda")
    rows = []
    tot = {"torch": 0.0, "nbd": 0.0}
    for name, T, N, K in linears():
        x = torch.randn(T, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        dy = torch.randn(T, N, device=dev).to(torch.bfloat16)
        cases = {
            # product: (torch fn, nbd fn, (M, N, K), a_km, b_kn, A, B)
            "fwd": (lambda: x @ w.t(), (T, N, K), False, False, x, w),
            "dgrad": (lambda: dy @ w, (T, K, N), False, True, dy, w),
            "wgrad": (lambda: dy.t() @ x, (N, K, T), True, True, dy, x),
        }
        for prod, (tfn, (M, NN, KK), a_km, b_kn, A, B) in cases.items():
            flop = 2.0 * M * NN * KK
            if a.tunableop:  # the search runs at the first call of a shape; time the chosen solution
                tfn()
                torch.cuda.synchronize()
            t_torch = timeit(tfn)
            t_nbd = timeit(lambda: G.matmul(A, B, a_km=a_km, b_kn=b_kn))
            ref = tfn().float()
            got = G.matmul(A, B, a_km=a_km, b_kn=b_kn).float()
            err = float((got - ref).abs().max() / ref.abs().max())
            row = {"linear": name, "product": prod, "M": M, "N": NN, "K": KK, "torch_us": t_torch * 1e3,
                   "nbd_us": t_nbd * 1e3, "torch_TFs": flop / t_torch / 1e9, "nbd_TFs": flop / t_nbd / 1e9,
                   "speedup": t_torch / t_nbd, "rel_err": err}
            if a.sweep:
                var = {}
                for tile in (128128, 128064, 64128, 64064):
                    if M % (tile // 1000) or NN % (tile % 1000):
                        continue
                    for wv, stg, ks in ((4, 2, 1), (4, 3, 1), (8, 2, 1), (8, 3, 1), (4, 2, 2), (4, 3, 2)):
                        if ks == 2 and tile == 128128:
                            continue
                        if wv == 8 and tile != 128128:
                            continue
                        for s in (1, 2, 4, 8):
                            if KK % (64 * s * ks) or (s > 1 and KK // s < 256):
                                continue
                            hint = ks * 100000000 + wv * 10000000 + stg * 1000000 + tile
                            var[f"{tile // 1000}x{tile % 1000}/w{wv}p{stg}k{ks}/s{s}"] = round(
                                timeit(lambda: G.matmul(A, B, a_km=a_km, b_kn=b_kn, splits=s, tile=hint)) * 1e3, 1)
                row["variants_us"] = var
            rows.append(row)
            tot["torch"] += t_torch
            tot["nbd"] += t_nbd
            print(f"{name:18s} {prod:5s} M={M:5d} N={NN:5d} K={KK:5d}  torch {t_torch * 1e3:7.1f} us "
                  f"({row['torch_TFs']:6.1f} TF/s)  nbd {t_nbd * 1e3:7.1f} us ({row['nbd_TFs']:6.1f} TF/s)  "
                  f"x{row['speedup']:.2f}  err {err:.1e}" + (f"  {row['variants_us']}" if a.sweep else ""), flush=True)
    print(f"total torch {tot['torch'] * 1e3:.0f} us, nbd {tot['nbd'] * 1e3:.0f} us", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"rows": rows, "total_torch_us": tot["torch"] * 1e3, "total_nbd_us": tot["nbd"] * 1e3,
                       "device": torch.cuda.get_device_name()}, f, indent=1)


if __name__ == "__main__":
    main()
