#!/usr/bin/env python3
"""A/B: the ping-pong GEMM schedule (tile code 89128128: 128x128, 8 waves, 3-buffer ring, wave
groups staggered by one barrier, one workgroup per CU) against the tuned kernels, on the GPT-2
small products (8192 tokens), interleaved rounds in one process, random operands; each result is
checked against an fp32 reference first.

    python benchmarks/gemm_pp_ab.py [--rounds 3] [--iters 30]
    NBD_GEMM_PAIR_PP=0|1 python benchmarks/gemm_pp_ab.py --pair     # the grouped backward launches
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nbdistributed_amd import ops  # noqa: E402
from nbdistributed_amd.ops import gemm as G  # noqa: E402

PP = 89128128
# (layout, M, N, K, epi)
FWD = [("fwd", 8192, 2304, 768, 0), ("fwd", 8192, 3072, 768, 1), ("fwd", 8192, 768, 768, 0),
       ("fwd", 8192, 768, 3072, 0), ("dgrad", 8192, 768, 2304, 0), ("dgrad", 8192, 768, 3072, 0),
       ("dgrad", 8192, 3072, 768, 2), ("fwd", 4096, 4096, 4096, 0)]
# grouped backward: (M tokens, N out, K in, epi1)
PAIRS = [(8192, 2304, 768, 0), (8192, 768, 768, 0), (8192, 3072, 768, 0), (8192, 768, 3072, 2)]


def _time(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def _operands(layout, M, N, K, epi, g):
    a_km, b_kn = {"fwd": (False, False), "dgrad": (False, True), "wgrad": (True, True)}[layout]
    A = (torch.rand(*((K, M) if a_km else (M, K)), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(*((K, N) if b_kn else (N, K)), device="cuda", generator=g) * 0.2 - 0.1).to(torch.bfloat16)
    aux = (torch.rand(M, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16) if epi == G.EPI_DGELU else None
    bias = (torch.rand(N, device="cuda", generator=g) - 0.5).to(torch.bfloat16) if epi == G.EPI_GELU else None
    return a_km, b_kn, A, B, aux, bias


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--pair", action="store_true")
    a = ap.parse_args()
    ops.load_library()
    g = torch.Generator(device="cuda").manual_seed(0)
    if a.pair:
        tag = "pp" if os.environ.get("NBD_GEMM_PAIR_PP") == "1" else "base"
        for M, N, K, epi in PAIRS:
            dy = (torch.rand(M, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
            w = (torch.rand(N, K, device="cuda", generator=g) * 0.2 - 0.1).to(torch.bfloat16)
            x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
            aux = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16) if epi else None
            dx, dw, db = G.backward_pair(dy, w, x, epi, aux, True)
            rdx = dy.float() @ w.float()
            if epi:
                rdx = G._dgelu_ref(rdx, aux)
            rdw = dy.float().t() @ x.float()
            ew = float((dw.float() - rdw).abs().max() / rdw.abs().max())
            ex = float((dx.float() - rdx).abs().max() / rdx.abs().max())
            flops = 4.0 * M * N * K
            ts = [_time(lambda: G.backward_pair(dy, w, x, epi, aux, True), a.iters) for _ in range(a.rounds)]
            print(f"pair[{tag}] dy {M}x{N} W {N}x{K} epi {epi}: " + " ".join(f"{t:.1f}" for t in ts)
                  + f" us  best {flops / min(ts) / 1e6:.0f} TF/s  err dW {ew:.2e} dx {ex:.2e}", flush=True)
        return
    for layout, M, N, K, epi in FWD:
        a_km, b_kn, A, B, aux, bias = _operands(layout, M, N, K, epi, g)
        tuned, _ = G.config(a_km, b_kn, M, N, K, can_split=False, epi=epi)
        ref = (A.float().t() if a_km else A.float()) @ (B.float() if b_kn else B.float().t())
        if bias is not None:
            ref = ref + bias.float()
        if epi == G.EPI_GELU:
            ref = torch.nn.functional.gelu(ref, approximate="tanh")
        if epi == G.EPI_DGELU:
            ref = G._dgelu_ref(ref, aux)
        res = {}
        for name, tile in (("tuned", tuned), ("pp", PP)):
            fn = lambda t=tile: G.matmul(A, B, a_km=a_km, b_kn=b_kn, epi=epi, aux=aux, bias=bias, tile=t, splits=1)  # noqa: E731
            out = fn()
            y = out[0] if isinstance(out, tuple) else out
            err = float((y.float() - ref).abs().max() / ref.abs().max()) if ref is not None else float("nan")
            res[name] = (err, [])
        for _ in range(a.rounds):
            for name, tile in (("tuned", tuned), ("pp", PP)):
                fn = lambda t=tile: G.matmul(A, B, a_km=a_km, b_kn=b_kn, epi=epi, aux=aux, bias=bias, tile=t, splits=1)  # noqa: E731
                res[name][1].append(_time(fn, a.iters))
        flops = 2.0 * M * N * K
        line = f"{layout} {M}x{N}x{K} epi {epi}:"
        for name, tile in (("tuned", tuned), ("pp", PP)):
            err, ts = res[name]
            line += f"  {name}({tile}) best {min(ts):.1f} us {flops / min(ts) / 1e6:.0f} TF/s err {err:.1e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
