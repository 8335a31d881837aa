#!/usr/bin/env python3
"""Where the device copies and fills of the GPT-2 flat-DDP step come from: one eager step
(after warm-up) under torch.profiler with Python stacks; every aten copy / fill / zero op is
listed with its shapes and the innermost repository frames, grouped and counted.

    python benchmarks/copy_trace.py [--B 8] [--T 1024]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from nbdistributed_amd.models import GPT2, GPT2Config  # noqa: E402
from nbdistributed_amd.optim import FlatAdamW  # noqa: E402
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP  # noqa: E402
from nbdistributed_amd.parallel.backend import init_data_plane  # noqa: E402

OPS = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::clone", "aten::zeros", "aten::zeros_like",
       "aten::cat", "aten::contiguous", "aten::index_put_", "aten::_to_copy")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--T", type=int, default=1024)
    a = ap.parse_args()
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    init_data_plane("rccl", 0, 1, dev)
    torch.manual_seed(0)
    m = GPT2(GPT2Config.small()).to(dev).to(torch.bfloat16)
    w = NbdDDP(m, flat_params=True, grad_mode="bucket")
    opt = FlatAdamW(w, lr=3e-4, capturable=True)
    x = torch.randint(0, 50257, (a.B, a.T), device=dev)

    def step():
        _, loss = w(x, x, return_logits=False)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    groups = collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        # only top-level calls of these ops (a clone's inner copy_ is counted once, as the clone)
        if ev.cpu_parent is not None and ev.cpu_parent.name in OPS:
            continue
        frames = [f for f in (ev.stack or []) if repo in f or "torch/autograd" in f]
        where = " <- ".join(f.replace(repo + "/", "") for f in frames[:3]) or "(no python frame: autograd engine / C++)"
        groups[(ev.name, str(ev.input_shapes)[:90], where)] += 1
    print(f"{sum(groups.values())} copy/fill ops in one step")
    for (name, shapes, where), n in groups.most_common():
        print(f"{n:4d}  {name:18s} {shapes:90s}  {where}")


if __name__ == "__main__":
    main()
