#!/usr/bin/env python3
"""PyTorch TunableOp (hipBLASLt/rocBLAS solution search) on the GPT-2 LM-head products vs the
default heuristic.  Writes the tuned table to $TUNE_OUT (PYTORCH_TUNABLEOP_FILENAME format)."""
import os
import statistics
import sys
import time

import torch

V = int(os.environ.get("NBD_VOCAB", "50257"))
SHAPES = [("lmhead fwd", lambda h, w, g: torch.mm(h, w.t())),
          ("lmhead dgrad", lambda h, w, g: torch.mm(g, w)),
          ("lmhead wgrad", lambda h, w, g: torch.mm(g.t(), h))]


def bench(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    h = (torch.rand(8192, 768, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(V, 768, device="cuda") * 0.1 - 0.05).to(torch.bfloat16)
    g = (torch.rand(8192, V, device="cuda") * 2e-5 - 1e-5).to(torch.bfloat16)
    base = {n: statistics.median([bench(lambda: f(h, w, g)) for _ in range(3)]) for n, f in SHAPES}
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(os.environ.get("TUNE_OUT", "/tmp/tunableop_results.csv"))
    t0 = time.time()
    for n, f in SHAPES:
        f(h, w, g)
    torch.cuda.synchronize()
    print(f"tuning took {time.time() - t0:.1f} s", flush=True)
    tun.tuning_enable(False)
    tuned = {n: statistics.median([bench(lambda: f(h, w, g)) for _ in range(3)]) for n, f in SHAPES}
    for r in tun.get_results():
        print("result", r)
    for n, _ in SHAPES:
        print(f"{n:14s} default {base[n]:7.1f} us   tuned {tuned[n]:7.1f} us   ({base[n] / tuned[n]:.2f}x)")


if __name__ == "__main__":
    main()
