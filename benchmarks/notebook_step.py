#!/usr/bin/env python3
"""The reference notebook's training step (SmolLM2-135M sequence classifier, bs 16, seq 128)
in one process on one GPU, in several recipes, for profiling:

    python benchmarks/notebook_step.py [--modes fp32,bf16flat,graph] [--steps 20]

fp32      : HF model, fp32 params, torch AdamW (the notebook's recipe, minus accelerate/DDP wrappers)
bf16flat  : HF model, bf16 params in nbd DDP buckets (world 1) + FlatAdamW
nbd       : native Llama (models/llama.py, HIP kernels), bf16 flat DDP + FlatAdamW
nbdgraph  : nbd captured once into a HIP graph (nbdistributed_amd.graphs) and replayed
nbdbg     : nbd eager with one HIP graph per decoder block's forward (ops.block_graphs(1))
nbdbg2    : nbdbg with each block's backward graphed too (ops.block_graphs(2))
hfnative  : HF model + the one-line swap nbd.models.native(model) (fp32 master weights, bf16
            compute), torch AdamW — the notebook's loop minus accelerate's wrappers
hfnativebg: hfnativedefault with per-block forward graphs (ops.block_graphs(1))
hfnativefused: hfnative with torch.optim.AdamW(..., fused=True)
hfnativedefault: hfnative with the notebook's optimizer line unchanged (native() makes it fused)
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
    ap.add_argument("--modes", default="fp32,bf16flat")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warm", type=int, default=5)
    ap.add_argument("--bs", type=int, default=16)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--phases", action="store_true",
                    help="eager modes: per-phase host time vs GPU time (HIP events) of forward / backward / step")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from nbdistributed_amd.parallel.backend import init_data_plane

    init_data_plane("rccl", 0, 1, dev)
    from nbdistributed_amd.models import smollm2_135m_classifier, synthetic_mrpc
    from nbdistributed_amd.optim import FlatAdamW
    from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP

    ids, mask, labels = synthetic_mrpc(n=a.bs * 8, seq_len=a.seq)
    ids, mask, labels = ids.to(dev), mask.to(dev), labels.to(dev)
    for mode in a.modes.split(","):
        torch.manual_seed(42)
        native = mode in ("nbd", "nbdgraph", "nbdbg", "nbdbg2")
        if native:
            from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification

            model = LlamaForSequenceClassification(LlamaConfig.smollm2_135m())
        else:
            model = smollm2_135m_classifier()
        if mode == "fp32":
            model = model.to(dev)
            opt = torch.optim.AdamW(model.parameters(), lr=2e-5)
            fwd = model
        elif mode.startswith("hfnative"):
            from nbdistributed_amd.models import native as _native

            model = _native(model.to(dev))
            if mode in ("hfnativedefault", "hfnativebg"):  # the notebook's line as written (native(): fused)
                opt = torch.optim.AdamW(model.parameters(), lr=2e-5)
            else:
                opt = torch.optim.AdamW(model.parameters(), lr=2e-5, fused=mode == "hfnativefused")
            print(f"{mode}: AdamW fused={opt.defaults.get('fused')}", flush=True)
            fwd = model
        else:
            fwd = NbdDDP(model.to(dev, torch.bfloat16), flat_params=True, grad_mode="bucket")
            opt = FlatAdamW(fwd, lr=2e-5, capturable=mode == "nbdgraph")  # overlap: NBD_ADAMW_OVERLAP
        batches = [(ids[i * a.bs:(i + 1) * a.bs], mask[i * a.bs:(i + 1) * a.bs], labels[i * a.bs:(i + 1) * a.bs])
                   for i in range(8)]

        marks = []  # (--phases) per step: [(host s, event)] at start / after fwd / bwd / optimizer

        def mark():
            if a.phases and mode != "nbdgraph":
                e = torch.cuda.Event(enable_timing=True)
                e.record()
                marks[-1].append((time.perf_counter(), e))

        def step(x, m, y):
            if a.phases and mode != "nbdgraph":
                marks.append([])
            mark()
            if native:
                loss = fwd(x, m, y)[0]
            else:
                loss = fwd(input_ids=x, attention_mask=m, labels=y).loss
            mark()
            loss.backward()
            mark()
            opt.step()
            opt.zero_grad(set_to_none=True)
            mark()
            return loss.detach()

        from nbdistributed_amd import ops

        if native or mode.startswith("hfnative"):
            ops.block_graphs({"nbdbg": 1, "nbdbg2": 2, "hfnativebg": 1}.get(mode, 0))
        if mode == "nbdgraph":
            from nbdistributed_amd.graphs import GraphedStep

            call = GraphedStep(step, batches[0], warmup=3, optimizers=[opt])
        else:
            call = step
        for i in range(a.warm):
            call(*batches[i % 8])
        torch.cuda.synchronize()
        marks.clear()
        if os.environ.get("NBD_HOST_TIMING") == "1" and native:
            torch.ops.nbd.host_timing(True)
        t = time.perf_counter()
        for i in range(a.steps):
            loss = call(*batches[i % 8])
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / a.steps * 1e3
        extra = f"  {ops.block_graphs_stats()}" if mode.startswith("nbdbg") or mode == "hfnativebg" else ""
        if marks:  # host enqueue time vs GPU time per phase; GPU idle = the step's GPU span minus busy
            names = ("forward", "backward", "optimizer")
            host = [0.0] * 3
            gpu = [0.0] * 3
            for mk in marks:
                for j in range(3):
                    host[j] += (mk[j + 1][0] - mk[j][0]) * 1e3
                    gpu[j] += mk[j][1].elapsed_time(mk[j + 1][1])
            n = len(marks)
            extra += "\n  phases (host enqueue ms / GPU span ms): " + ", ".join(
                f"{nm} {h / n:.2f} / {g / n:.2f}" for nm, h, g in zip(names, host, gpu))
        if os.environ.get("NBD_HOST_TIMING") == "1" and native:
            extra += "\n" + torch.ops.nbd.host_timing(True)
        print(f"{mode:9s} {ms:8.2f} ms/step  {a.bs / ms * 1e3:8.1f} samples/s  loss {float(loss.detach()):.4f}{extra}",
              flush=True)
        del model, opt, fwd
        torch.cuda.empty_cache()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
