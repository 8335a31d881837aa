#!/usr/bin/env python3
"""Embedding backward (``nbd::embedding_bwd``, csrc/kernels/embed.hip) on the GPT-2 step's shape:
8192 token ids over a 50304-row padded table, C = 768, bf16, accumulating into the tied LM
head's gradient (what ops/embedding.py does in the DDP step) and writing a fresh gradient.
Uniform random ids (mostly distinct) and right-padded batches (one id repeated 2048 times).
Set ``NBD_OPS_LIB`` to time another build (benchmarks/ab_lib.sh).

    python benchmarks/embed_bench.py [--iters 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nbdistributed_amd.ops import _lib  # noqa: E402


def _median_us(fn, iters):
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    assert _lib.load_library(), _lib._load_error
    dev = torch.device("cuda")
    N, V, Vp, C = 8192, 50257, 50304, 768
    g = torch.Generator(device=dev).manual_seed(0)
    dy = torch.randn(N, C, device=dev, generator=g).to(torch.bfloat16)
    grad = torch.zeros(Vp, C, device=dev, dtype=torch.bfloat16)
    res = {"lib": os.environ.get("NBD_OPS_LIB", "in-tree")}
    for name in ("uniform", "padded"):
        idx = torch.randint(0, V, (N,), device=dev, generator=g)
        if name == "padded":
            idx[-2048:] = 50256
        res[name + "_accumulate_us"] = round(_median_us(
            lambda: torch.ops.nbd.embedding_bwd(dy, idx, V, grad, True), a.iters), 1)
        res[name + "_fresh_us"] = round(_median_us(
            lambda: torch.ops.nbd.embedding_bwd(dy, idx, V, None, False), a.iters), 1)
    print(res, flush=True)


if __name__ == "__main__":
    main()
