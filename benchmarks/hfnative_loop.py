#!/usr/bin/env python3
"""The reference notebook's training loop with the one-line swap, standalone (for rocprofv3 and
host/GPU phase timing): SmolLM2-135M-cls (random init), accelerate ``prepare`` (torch DDP on a
one-rank ``rccl`` group), ``nbd.models.native(model)``, torch AdamW (native()'s fused default),
linear warm-up schedule, bs 16 x seq 128 synthetic MRPC-shaped batches.

    python benchmarks/hfnative_loop.py [--steps 20] [--warm 5] [--no-accelerate] [--phases]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warm", type=int, default=5)
    ap.add_argument("--no-accelerate", action="store_true")
    ap.add_argument("--phases", action="store_true")
    a = ap.parse_args()
    for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29543"), ("RANK", "0"), ("WORLD_SIZE", "1"),
                 ("LOCAL_RANK", "0")):
        os.environ.setdefault(k, v)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from nbdistributed_amd.parallel.backend import init_data_plane

    init_data_plane("rccl", 0, 1, dev)
    from torch.utils.data import DataLoader, TensorDataset
    from transformers import get_linear_schedule_with_warmup

    from nbdistributed_amd.models import native, smollm2_135m_classifier, synthetic_mrpc

    bs = 16
    n = bs * (a.steps + a.warm + 2)
    ids, mask, labels = synthetic_mrpc(n=n, seq_len=128)
    torch.manual_seed(42)
    model = native(smollm2_135m_classifier().to(dev))
    opt = torch.optim.AdamW(model.parameters(), lr=2e-5)
    dl = DataLoader(TensorDataset(ids, mask, labels), batch_size=bs, shuffle=True)
    sched = get_linear_schedule_with_warmup(opt, 100, 3 * len(dl))
    if not a.no_accelerate:
        from accelerate import Accelerator

        acc = Accelerator()
        model, opt, dl, sched = acc.prepare(model, opt, dl, sched)
        backward = acc.backward
    else:
        backward = lambda loss: loss.backward()  # noqa: E731
        dl = [(x.to(dev), m.to(dev), y.to(dev)) for x, m, y in dl]
    it = iter(dl)
    marks = []

    def mark():
        if a.phases:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            marks[-1].append((time.perf_counter(), e))

    def step():
        x, m, y = next(it)
        if a.phases:
            marks.append([])
        mark()
        out = model(input_ids=x, attention_mask=m, labels=y)
        mark()
        backward(out.loss)
        mark()
        opt.step()
        sched.step()
        opt.zero_grad()
        mark()
        return out.loss.detach()

    for _ in range(a.warm):
        step()
    torch.cuda.synchronize()
    marks.clear()
    t = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / a.steps * 1e3
    extra = ""
    if marks:
        names = ("forward", "backward", "optimizer")
        host, gpu = [0.0] * 3, [0.0] * 3
        for mk in marks:
            for j in range(3):
                host[j] += (mk[j + 1][0] - mk[j][0]) * 1e3
                gpu[j] += mk[j][1].elapsed_time(mk[j + 1][1])
        extra = "  phases (host enqueue ms / GPU span ms): " + ", ".join(
            f"{nm} {h / len(marks):.2f} / {g / len(marks):.2f}" for nm, h, g in zip(names, host, gpu))
    print(f"hfnative{'' if not a.no_accelerate else '-noacc'} {ms:.2f} ms/step  loss {float(loss):.4f}{extra}",
          flush=True)
    import torch.distributed as dist

    dist.destroy_process_group()


if __name__ == "__main__":
    main()
