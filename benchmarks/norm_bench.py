"""LayerNorm / RMSNorm kernel timings at the GPT-2 / SmolLM2 step shapes (bf16), with effective
HBM bandwidth.  python benchmarks/norm_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nbdistributed_amd.ops._lib import _require  # noqa: E402


def _time(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    _require()
    dev = torch.device("cuda", 0)
    for rows, C in ((8192, 768), (2048, 576), (16384, 1024)):
        x, d, dy, dr = (torch.randn(rows, C, device=dev, dtype=torch.bfloat16) for _ in range(4))
        w = torch.randn(C, device=dev, dtype=torch.bfloat16)
        b = torch.randn(C, device=dev, dtype=torch.bfloat16)
        y, s, mean, rstd = torch.ops.nbd.ln_fwd(x, d, w, b, 1e-5)
        nb = rows * C * 2
        tf = _time(lambda: torch.ops.nbd.ln_fwd(x, d, w, b, 1e-5))
        tb = _time(lambda: torch.ops.nbd.ln_bwd(s, dy, dr, w, mean, rstd))
        print(json.dumps({"rows": rows, "C": C, "ln_fwd_us": round(tf, 1), "ln_fwd_TBps": round(4 * nb / tf / 1e6, 2),
                          "ln_bwd_us": round(tb, 1), "ln_bwd_TBps": round(4 * nb / tb / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
