#!/usr/bin/env python3
"""A/B: the GEMM next-weight warm-up (csrc/kernels/gemm.hip "next-weight warm-up") on the GPT-2
small training step (bf16, 8x1024 tokens, nbd DDP + FlatAdamW), eager and as one HIP graph,
interleaved rounds in one process.  NBD_GEMM_WARM is read at every launch, so the eager arms
toggle it between rounds; each graph arm is captured with its setting.

    python benchmarks/warm_ab.py [--rounds 4] [--steps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    import torch.distributed as dist

    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29737")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from nbdistributed_amd.graphs import GraphedStep
    from nbdistributed_amd.models import GPT2, GPT2Config
    from nbdistributed_amd.optim import FlatAdamW
    from nbdistributed_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = GPT2(GPT2Config.small()).to(dev, torch.bfloat16)
    ddp = DistributedDataParallel(m, flat_params=True, grad_mode="bucket")
    opt = FlatAdamW(ddp, lr=3e-4, capturable=True)
    x = torch.randint(0, 50257, (8, 1024), device=dev)

    def step(inp):
        loss = ddp(inp, inp, return_logits=False)[1]
        loss.backward()
        opt.step()
        opt.zero_grad()
        return loss.detach()

    graphs = {}
    for w in ("0", "1"):
        os.environ["NBD_GEMM_WARM"] = w
        for _ in range(3):  # the launches learn the weight order under this setting
            step(x)
        graphs[w] = GraphedStep(step, (x,), warmup=2, optimizers=[opt])

    def timed(fn):
        for _ in range(3):
            fn(x)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(a.steps):
            fn(x)
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / a.steps

    res = {k: [] for k in ("eager warm=0", "eager warm=1", "graph warm=0", "graph warm=1")}
    for r in range(a.rounds):
        for w in ("0", "1"):
            os.environ["NBD_GEMM_WARM"] = w
            res[f"eager warm={w}"].append(timed(step))
        for w in ("0", "1"):
            res[f"graph warm={w}"].append(timed(graphs[w]))
        print(f"round {r}: " + " | ".join(f"{k} {v[-1]:.3f}" for k, v in res.items()) + " ms", flush=True)
    for k, v in res.items():
        print(f"{k:14s} best {min(v):.3f} ms  median {sorted(v)[len(v) // 2]:.3f} ms", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
