#!/usr/bin/env python3
"""Staged HIP-graph capture probe (which part of a training step breaks capture?)."""
import faulthandler
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29555")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
from nbdistributed_amd.models import GPT2, GPT2Config  # noqa: E402
from nbdistributed_amd.optim import FlatAdamW  # noqa: E402
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP  # noqa: E402
from nbdistributed_amd.parallel.backend import init_data_plane  # noqa: E402

stage = sys.argv[1] if len(sys.argv) > 1 else "all"
if os.environ.get("PROBE_SMALL"):  # the bench shapes: GPT-2 small, 8 x 1024 tokens
    cfg = GPT2Config()
    x = torch.randint(0, 50257, (8, 1024), device=dev)
else:
    cfg = GPT2Config(vocab_size=1024, n_positions=256, n_embd=256, n_layer=2, n_head=4)
    x = torch.randint(0, 1024, (2, 256), device=dev)


def capture(name, fn):
    print(f"[{name}] warmup", flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    print(f"[{name}] capture", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        out = fn()
    torch.cuda.synchronize()
    print(f"[{name}] replay", flush=True)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print(f"[{name}] OK {out}", flush=True)


if stage in ("ar", "ar_async", "side"):
    init_data_plane(os.environ.get("PROBE_BACKEND", "rccl"), 0, 1, dev)
    t = torch.ones(1 << 20, device=dev)
    if stage == "ar":
        capture("all_reduce", lambda: dist.all_reduce(t) or t.sum())
    elif stage == "ar_async":
        def f():
            w = dist.all_reduce(t, async_op=True)
            w.wait()
            return t.sum()
        capture("all_reduce async", f)
    else:
        side = torch.cuda.Stream()

        def f():
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                t.mul_(1.0)
                w = dist.all_reduce(t, async_op=True)
                w.wait()
                t.mul_(1.0)
            torch.cuda.current_stream().wait_stream(side)
            return t.sum()
        capture("side-stream all_reduce", f)
    dist.destroy_process_group()
    sys.exit(0)
m = GPT2(cfg).to(dev, torch.bfloat16)
if stage in ("fwd", "all"):
    capture("fwd", lambda: m(x, x, return_logits=False)[1].detach())
if stage in ("bwd", "all"):
    def fb():
        loss = m(x, x, return_logits=False)[1]
        loss.backward()
        return loss.detach()
    capture("fwd+bwd", fb)
if stage in ("ddp", "opt", "all"):
    init_data_plane(os.environ.get("PROBE_BACKEND", "rccl"), 0, 1, dev)
    d = NbdDDP(GPT2(cfg).to(dev, torch.bfloat16), flat_params=True, grad_mode="bucket")

    def ddp_step():
        loss = d(x, x, return_logits=False)[1]
        loss.backward()
        return loss.detach()
    if stage in ("ddp", "all"):
        capture("ddp fwd+bwd", ddp_step)
    if stage in ("opt", "all"):
        o = FlatAdamW(d, lr=1e-3, capturable=True)

        def full():
            loss = ddp_step()
            o.clip_grad_norm_(1.0)
            o.step()
            o.zero_grad()
            return loss
        capture("ddp+opt", full)
    dist.destroy_process_group()
