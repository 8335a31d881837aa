#!/usr/bin/env python3
"""Decode-shaped linear layers: the fused small-M kernel (ops.linear_small) vs the op-by-op path
(norm kernel + hipBLASLt GEMM + activation / residual kernels), and an empty-ish kernel as the
per-launch floor.  Back-to-back launches in one HIP graph per case (the generation loop's mode).

    python benchmarks/smallm_bench.py [--rows 1,8,32,64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def graph_time(fn, reps=20, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / (iters * reps) * 1e3  # us per call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1,8,32,64")
    a = ap.parse_args()
    from nbdistributed_amd import ops

    ops.load_library()
    torch.manual_seed(0)
    C = 768
    bf = dict(device="cuda", dtype=torch.bfloat16)
    W = {"qkv": torch.randn(3 * C, C, **bf) * 0.02, "proj": torch.randn(C, C, **bf) * 0.02,
         "fc": torch.randn(4 * C, C, **bf) * 0.02, "proj2": torch.randn(C, 4 * C, **bf) * 0.02,
         "head": torch.randn(50257, C, **bf) * 0.02}
    b = {k: torch.randn(w.shape[0], **bf) * 0.1 for k, w in W.items()}
    lnw, lnb = torch.ones(C, **bf), torch.zeros(C, **bf)
    out = []
    z = torch.zeros(1, **bf)
    floor = graph_time(lambda: z.add_(1))
    print(json.dumps({"launch_floor_us": round(floor, 2)}), flush=True)
    for M in [int(r) for r in a.rows.split(",")]:
        x = torch.randn(M, C, **bf)
        h = torch.randn(M, 4 * C, **bf)
        cases = {
            "ln+qkv+bias": (lambda: ops.linear_small(x, W["qkv"], b["qkv"], norm=("ln", lnw, lnb, 1e-5)),
                            lambda: F.linear(ops.layer_norm(x, lnw, lnb), W["qkv"], b["qkv"])),
            "proj+bias+res": (lambda: ops.linear_small(x, W["proj"], b["proj"], residual=x),
                              lambda: x + F.linear(x, W["proj"], b["proj"])),
            "ln+fc+gelu": (lambda: ops.linear_small(x, W["fc"], b["fc"], norm=("ln", lnw, lnb, 1e-5), act="gelu"),
                           lambda: F.gelu(F.linear(ops.layer_norm(x, lnw, lnb), W["fc"], b["fc"]), approximate="tanh")),
            "proj2+bias+res": (lambda: ops.linear_small(h, W["proj2"], b["proj2"], residual=x),
                               lambda: x + F.linear(h, W["proj2"], b["proj2"])),
            "ln+head": (lambda: ops.linear_small(x, W["head"], norm=("ln", lnw, lnb, 1e-5)),
                        lambda: F.linear(ops.layer_norm(x, lnw, lnb), W["head"])),
            # the kernel without its norm prologue (what a separate norm kernel would feed)
            "qkv+bias (no norm)": (lambda: ops.linear_small(x, W["qkv"], b["qkv"]),
                                   lambda: F.linear(x, W["qkv"], b["qkv"])),
            "fc+gelu (no norm)": (lambda: ops.linear_small(x, W["fc"], b["fc"], act="gelu"),
                                  lambda: F.gelu(F.linear(x, W["fc"], b["fc"]), approximate="tanh")),
            "head (no norm)": (lambda: ops.linear_small(x, W["head"]), lambda: F.linear(x, W["head"])),
        }
        for name, (fused, ref) in cases.items():
            tf, tr = graph_time(fused), graph_time(ref)
            key = name.split(" ")[0].split("+")
            wbytes = W[key[1] if key[0] == "ln" else key[0]].numel() * 2
            r = dict(rows=M, op=name, fused_us=round(tf, 2), op_by_op_us=round(tr, 2), speedup=round(tr / tf, 2),
                     weight_GBps=round(wbytes / tf / 1e3, 1))
            print(json.dumps(r), flush=True)
            out.append(r)


if __name__ == "__main__":
    main()
