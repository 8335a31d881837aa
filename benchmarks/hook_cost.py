"""Cost of a Python post-accumulate-grad hook per parameter in a CUDA backward (the autograd
device thread must take the GIL for each call): 183 parameters (SmolLM2-135M), a trivial graph.

    python benchmarks/hook_cost.py
"""
import time

import torch


def main() -> None:
    dev = torch.device("cuda")
    ps = [torch.nn.Parameter(torch.randn(64, device=dev)) for _ in range(183)]
    pend = [0] * 8
    bucket_of = {id(p): i % 8 for i, p in enumerate(ps)}

    def hook(p):
        pend[bucket_of[id(p)]] -= 1

    def run(n=200):
        ts = []
        for _ in range(n):
            loss = torch.stack([p[0] for p in ps]).sum()
            torch.cuda.synchronize()
            t = time.perf_counter()
            loss.backward()
            ts.append(time.perf_counter() - t)
            for p in ps:
                p.grad = None
        ts.sort()
        return ts[len(ts) // 2] * 1e3

    run(20)
    for _ in range(3):
        a = run()
        hs = [p.register_post_accumulate_grad_hook(hook) for p in ps]
        b = run()
        for h in hs:
            h.remove()
        print(f"backward: no hooks {a:.3f} ms, python hooks {b:.3f} ms -> {(b - a) * 1e3 / len(ps):.2f} us/param",
              flush=True)


if __name__ == "__main__":
    main()
