#!/usr/bin/env python3
"""Host (CPU) cost of an eager training step — where the Python / dispatcher time goes when the
step is launch-bound (the SmolLM2 notebook step: 10+ ms eager vs 7 ms as a HIP graph).

    python benchmarks/host_profile.py [--model smollm2|gpt2] [--steps 5]

Prints the step's wall time, the GPU busy time, and the top operators by self CPU time.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="smollm2", choices=["smollm2", "gpt2"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cprofile", action="store_true", help="Python-level cProfile instead of the torch profiler")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dist.init_process_group("nccl", rank=0, world_size=1)
    dev = torch.device("cuda", 0)
    from nbdistributed_amd.optim import FlatAdamW
    from nbdistributed_amd.parallel import DistributedDataParallel as DDP

    torch.manual_seed(0)
    if a.model == "smollm2":
        from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification

        m = LlamaForSequenceClassification(LlamaConfig.smollm2_135m()).to(dev, torch.bfloat16)
        x = torch.randint(1, 49152, (16, 128), device=dev)
        mk = torch.ones_like(x)
        y = torch.randint(0, 2, (16,), device=dev)
        fwd = lambda mod: mod(x, mk, y)[0]  # noqa: E731
    else:
        from nbdistributed_amd.models import GPT2, GPT2Config

        m = GPT2(GPT2Config.small()).to(dev, torch.bfloat16)
        x = torch.randint(0, 50257, (8, 1024), device=dev)
        fwd = lambda mod: mod(x, x, return_logits=False)[1]  # noqa: E731
    ddp = DDP(m, flat_params=True, grad_mode="bucket")
    opt = FlatAdamW(ddp, lr=1e-4)

    def step():
        loss = fwd(ddp)
        loss.backward()
        opt.step()
        opt.zero_grad()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        step()
    host = (time.perf_counter() - t) / a.steps * 1e3  # host time to issue (GPU may lag behind)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t) / a.steps * 1e3
    print(f"{a.model}: wall {wall:.2f} ms/step, host issue {host:.2f} ms/step", flush=True)
    if a.cprofile:
        import cProfile
        import pstats

        pr = cProfile.Profile()
        pr.enable()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(35)
        dist.destroy_process_group()
        return
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
