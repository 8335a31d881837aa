#!/usr/bin/env python3
"""Single-process DDP comparison (nbd DDP vs torch DDP vs no DDP) on GPT-2 small, interleaved
rounds so warm-up / clock effects hit both equally.

    python benchmarks/ddp_compare.py [--rounds 3] [--steps 10] [--B 8] [--T 1024]
    torchrun --nproc-per-node N benchmarks/ddp_compare.py
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from nbdistributed_amd.models import GPT2, GPT2Config  # noqa: E402
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP  # noqa: E402
from nbdistributed_amd.parallel.backend import init_data_plane  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warm", type=int, default=3)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--impls", default="none,torch,nbd,nbd32")
    ap.add_argument("--backend", default="rccl")
    a = ap.parse_args()
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    init_data_plane(a.backend, rank, world, dev)
    torch.manual_seed(0)
    base = GPT2(GPT2Config.small()).to(dev)
    x = torch.randint(0, 50257, (a.B, a.T), device=dev)
    models = {}
    import copy

    for impl in a.impls.split(","):
        m = copy.deepcopy(base)
        if impl == "torch":
            w = torch.nn.parallel.DistributedDataParallel(m, device_ids=[local])
        elif impl == "nbd":
            w = NbdDDP(m, comm_dtype=torch.bfloat16)
        elif impl == "nbd32":
            w = NbdDDP(m)
        else:
            w = m
        opt = torch.optim.AdamW(m.parameters(), lr=3e-4, fused=True)
        models[impl] = (w, opt)

    def step(w, opt):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, loss = w(x, x)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)

    res = {k: [] for k in models}
    for r in range(a.rounds):
        for k, (w, opt) in models.items():
            for _ in range(a.warm):
                step(w, opt)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.steps):
                step(w, opt)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t) / a.steps * 1e3)
    if rank == 0:
        for k, v in res.items():
            print(f"{k:8s} ms/step " + " ".join(f"{x:.2f}" for x in v) + f"   tok/s {world * a.B * a.T / (min(v) / 1e3):.0f}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
