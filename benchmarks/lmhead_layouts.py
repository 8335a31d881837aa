"""LM-head weight-gradient layouts on hipBLASLt (torch.mm): dW = dlogitsᵀ·h as [V, C] directly,
or dWᵀ = hᵀ·dlogits as [C, V] (+ the transpose copy the parameter layout then needs).

    python benchmarks/lmhead_layouts.py
"""
import torch


def t_ms(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n


import sys

for V in ([int(v) for v in sys.argv[1:]] or [50257, 50304]):
    N, C = 8192, 768
    dl = torch.randn(N, V, device="cuda", dtype=torch.bfloat16)
    h = torch.randn(N, C, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(V, C, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * N * V * C
    a = t_ms(lambda: torch.mm(dl.t(), h))
    b = t_ms(lambda: torch.mm(h.t(), dl))
    c = t_ms(lambda: torch.mm(h.t(), dl).t().contiguous())
    f = t_ms(lambda: torch.mm(h, w.t()))
    d = t_ms(lambda: torch.mm(dl, w))
    print(f"V={V}: wgrad [V,C] {a*1e3:.0f} us ({fl/a/1e9:.0f} TF)  [C,V] {b*1e3:.0f} us ({fl/b/1e9:.0f} TF)  "
          f"[C,V]+transpose {c*1e3:.0f} us  fwd {f*1e3:.0f} us ({fl/f/1e9:.0f} TF)  dgrad {d*1e3:.0f} us ({fl/d/1e9:.0f} TF)",
          flush=True)
