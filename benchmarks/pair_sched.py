#!/usr/bin/env python3
"""Grouped-backward schedule sweep: every (split count S, dispatch order) of ``nbd::gemm_pair``
on the GPT-2 small and SmolLM2 Linear backward shapes, interleaved rounds, HIP-event timed
(incl. the split-K reduce kernel), each checked against an fp32 reference; marks the schedule
``ops.gemm.pair_schedule`` picks.

    python benchmarks/pair_sched.py [--rounds 3] [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nbdistributed_amd import ops  # noqa: E402
from nbdistributed_amd.ops import gemm as G  # noqa: E402

# dy [M, N], W [N, K], epi1
SHAPES = [("gpt2.qkv", 8192, 2304, 768, 0), ("gpt2.attn_proj", 8192, 768, 768, 0),
          ("gpt2.c_fc", 8192, 3072, 768, 0), ("gpt2.c_proj", 8192, 768, 3072, G.EPI_DGELU),
          ("smollm2.qkv", 2048, 960, 576, 0), ("smollm2.o_proj", 2048, 576, 576, 0),
          ("smollm2.gate_up", 2048, 3072, 576, 0), ("smollm2.down", 2048, 576, 1536, G.EPI_DSWIGLU)]


def _time(fn, iters, flush=False):
    for _ in range(3):
        fn()
    if flush:
        torch.ops.nbd.grad_defer_flush()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    if flush:  # one batched launch for the iters' reduces, like one flush per backward
        torch.ops.nbd.grad_defer_flush()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--deferred", action="store_true",
                    help="queue the split-K reduces (defer.hip) and flush once per timed batch, as a "
                         "DDP backward does for small weight gradients")
    ap.add_argument("--only", default="", help="comma-separated shape name prefixes")
    ap.add_argument("--small-tiles", action="store_true", help="also sweep 64x64 tiles (plan bit 5)")
    a = ap.parse_args()
    ops.load_library()
    if a.deferred:
        torch.ops.nbd.grad_defer_enable(True)
        torch.ops.nbd.grad_defer_force(True)
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, N, K, epi in SHAPES:
        if a.only and not any(name.startswith(p) for p in a.only.split(",")):
            continue
        tile = 128 if M % 128 == 0 and N % 128 == 0 and K % 128 == 0 else 64
        dy = (torch.rand(M, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device="cuda", generator=g) * 0.2 - 0.1).to(torch.bfloat16)
        x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        cols = 2 * K if epi == G.EPI_DSWIGLU else K
        aux = (torch.rand(M, cols, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16) if epi else None
        dx = torch.empty(M, cols, device="cuda", dtype=torch.bfloat16)
        dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        db = torch.empty(N, device="cuda", dtype=torch.bfloat16)
        rdx = dy.float() @ w.float()
        if epi == G.EPI_DGELU:
            rdx = G._dgelu_ref(rdx, aux)
        elif epi == G.EPI_DSWIGLU:
            rdx = G._dswiglu_ref(rdx, aux)
        rdw = dy.float().t() @ x.float()
        scheds = [s | (o << 4) for s in (1, 2, 4, 8) if M % (64 * s) == 0 and M // s >= 256 for o in (0, 1)]
        if tile == 128 and a.small_tiles:  # bit 5: the 64x64 pair kernel on a 128-divisible shape
            scheds += [sc | 32 for sc in scheds]
        pick = G.pair_schedule(M, N, K, tile, epi)

        def run(sc):
            torch.ops.nbd.gemm_pair(dy, w, dx, epi, aux, dy, x, dw, G.EPI_ROWSUM, db, sc)

        times = {sc: [] for sc in scheds}
        for sc in scheds:
            run(sc)
            if a.deferred:
                torch.ops.nbd.grad_defer_flush()
            ew = float((dw.float() - rdw).abs().max() / rdw.abs().max())
            ex = float((dx.float() - rdx).abs().max() / rdx.abs().max())
            assert ew < 2e-2 and ex < 2e-2, (name, sc, ew, ex)
        for _ in range(a.rounds):
            for sc in scheds:
                times[sc].append(_time(lambda: run(sc), a.iters, flush=a.deferred))
        flops = 4.0 * M * N * K
        best = min(scheds, key=lambda sc: min(times[sc]))
        print(f"{name} dy {M}x{N} W {N}x{K} epi {epi} (tile {tile}):", flush=True)
        for sc in scheds:
            t = min(times[sc])
            mark = (" <- model" if sc == pick else "") + (" <- best" if sc == best else "")
            print(f"   S={sc & 15} {'wgrad' if (sc >> 4) & 1 else 'dgrad'}-first{' 64x64' if sc & 32 else ''}  {t:7.1f} us "
                  f"{flops / t / 1e6:5.0f} TF/s  [{' '.join(f'{v:.1f}' for v in times[sc])}]{mark}", flush=True)


if __name__ == "__main__":
    main()
