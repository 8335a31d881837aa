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
from nbdistributed_amd.optim import FlatAdamW  # noqa: E402
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP  # noqa: E402
from nbdistributed_amd.parallel.backend import init_data_plane  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warm", type=int, default=3)
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--impls", default="none,torch,nbd,nbd32,flat,flatgraph")
    ap.add_argument("--clip", type=float, default=0.0, help="clip_grad_norm_ max norm (0: off)")
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
        amp = True
        if impl.endswith("blas"):  # A/B: Linear layers on hipBLASLt instead of the HIP MFMA GEMM
            for mod in m.modules():
                if hasattr(mod, "hip_gemm"):
                    mod.hip_gemm = False
        kind = impl[:-4] if impl.endswith("blas") else impl
        if kind in ("flat", "flatgraph"):
            # bf16 parameters re-homed into the DDP buckets, fp32 master/moments inside FlatAdamW,
            # one fused HIP AdamW kernel per bucket; no autocast casts in the forward
            m = m.to(torch.bfloat16)
            w = NbdDDP(m, flat_params=True, grad_mode="bucket")
            models[impl] = (w, FlatAdamW(w, lr=3e-4, capturable=kind == "flatgraph"), False)
            continue
        if impl == "torch":
            w = torch.nn.parallel.DistributedDataParallel(m, device_ids=[local])
        elif impl == "nbd":
            w = NbdDDP(m, comm_dtype=torch.bfloat16)
        elif impl == "nbd32":
            w = NbdDDP(m)
        else:
            w = m
        opt = torch.optim.AdamW(m.parameters(), lr=3e-4, fused=True)
        models[impl] = (w, opt, amp)

    def step(w, opt, amp, inp=None):
        inp = x if inp is None else inp
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            _, loss = w(inp, inp, return_logits=False)
        loss.backward()
        if a.clip > 0:
            if isinstance(opt, FlatAdamW):
                opt.clip_grad_norm_(a.clip)
            else:
                torch.nn.utils.clip_grad_norm_(w.parameters(), a.clip)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss.detach()

    graphs = {}
    for gk in ("flatgraph", "flatgraphblas"):
        if gk not in models:
            continue
        from nbdistributed_amd.graphs import GraphedStep

        w, opt, amp = models[gk]
        graphs[gk] = GraphedStep(lambda xx, w=w, opt=opt, amp=amp: step(w, opt, amp, xx), (x,), warmup=3,
                                 optimizers=[opt])

    def run(k, w, opt, amp):
        if k in graphs:
            return graphs[k](x)
        return step(w, opt, amp)

    res = {k: [] for k in models}
    losses = {}
    for r in range(a.rounds):
        for k, (w, opt, amp) in models.items():
            for _ in range(a.warm):
                run(k, w, opt, amp)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.steps):
                loss = run(k, w, opt, amp)
            torch.cuda.synchronize()
            res[k].append((time.perf_counter() - t) / a.steps * 1e3)
            losses[k] = float(loss.detach())
    if rank == 0:
        for k, v in res.items():
            print(f"{k:8s} ms/step " + " ".join(f"{x:.2f}" for x in v) +
                  f"   tok/s {world * a.B * a.T / (min(v) / 1e3):.0f}   loss {losses[k]:.4f}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
