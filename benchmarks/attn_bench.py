"""Flash-attention kernel timings (``nbd::attn_fwd`` / ``nbd::attn_bwd``) on the workload shapes.

    python benchmarks/attn_bench.py [--iters 50]

Times the forward and the backward launches separately with HIP events (median of ``iters``
after warm-up) for GPT-2 small (B8 H12 T1024 D64 causal) and the notebook's SmolLM2
(B16 H9/Hkv3 T128 D64 causal), plus non-causal GPT-2 as the no-imbalance reference.
TF/s counts the useful FLOPs: 4·B·Hq·T²·D (½ under a causal mask) forward, 2.5× that backward.
Set ``NBD_OPS_LIB`` to time another build of libnbd_ops.so (A/B in one box session).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nbdistributed_amd.ops import _lib  # noqa: E402

SHAPES = [
    ("gpt2_causal", 8, 12, 12, 1024, True),
    ("gpt2_full", 8, 12, 12, 1024, False),
    ("smollm2_causal", 16, 9, 3, 128, True),
    ("long4k_causal", 2, 12, 12, 4096, True),
]


def _median_ms(fn, iters: int) -> float:
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2]


def _pipelined_ms(fn, iters: int, reps: int = 20) -> float:
    for _ in range(5):
        fn()
    ts = []
    for _ in range(max(3, iters // 10)):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    ts.sort()
    return ts[len(ts) // 2]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="", help="comma-separated shape names")
    ap.add_argument("--shape", action="append", default=[],
                    help="extra shape name,B,H,Hkv,T,causal(0/1) (repeatable)")
    a = ap.parse_args()
    for sh in a.shape:
        nm, B_, H_, K_, T_, c_ = sh.split(",")
        SHAPES.append((nm, int(B_), int(H_), int(K_), int(T_), c_ == "1"))
    assert _lib.load_library(), _lib._load_error
    dev = torch.device("cuda")
    out = {"lib": os.environ.get("NBD_OPS_LIB", "in-tree")}
    for name, B, H, Hkv, T, causal in SHAPES:
        if a.only and name not in a.only.split(","):
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B, H, T, 64, device=dev, dtype=torch.bfloat16, generator=g)
        k, v = (torch.randn(B, Hkv, T, 64, device=dev, dtype=torch.bfloat16, generator=g) for _ in range(2))
        do = torch.randn_like(q)
        scale = 64 ** -0.5
        o, lse = torch.ops.nbd.attn_fwd(q, k, v, causal, scale, None, None)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        t_f = _median_ms(lambda: torch.ops.nbd.attn_fwd(q, k, v, causal, scale, None, None), a.iters)
        t_b = _median_ms(lambda: torch.ops.nbd.attn_bwd(do, q, k, v, o, lse, causal, scale, dq, dk, dv, None, None),
                         a.iters)
        # back-to-back launches (the host's launch work under the previous kernel): GPU time per call
        t_fp = _pipelined_ms(lambda: torch.ops.nbd.attn_fwd(q, k, v, causal, scale, None, None), a.iters)
        t_bp = _pipelined_ms(lambda: torch.ops.nbd.attn_bwd(do, q, k, v, o, lse, causal, scale, dq, dk, dv, None, None),
                             a.iters)
        fl = 4.0 * B * H * T * T * 64 * (0.5 if causal else 1.0)
        out[name] = {"fwd_us": round(t_f * 1e3, 2), "bwd_us": round(t_b * 1e3, 2),
                     "fwd_us_pipelined": round(t_fp * 1e3, 2), "bwd_us_pipelined": round(t_bp * 1e3, 2),
                     "fwd_TFs": round(fl / t_f / 1e9, 1), "bwd_TFs": round(2.5 * fl / t_b / 1e9, 1)}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
