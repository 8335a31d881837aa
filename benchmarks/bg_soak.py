#!/usr/bin/env python3
"""Soak run of the eager SmolLM2 notebook step with block / stack graphs (ops.block_graphs(1)):
600 steps in windows of 100, a differently sized batch every 150 steps (another shape: its own
per-block graphs, the stack keeps serving the main shape), an eval forward under no_grad every 50.
Prints per-window ms/step, allocated / reserved GiB and the graph counters — memory must stay flat
and the stack must keep serving.

    python benchmarks/bg_soak.py [--steps 600]
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
    ap.add_argument("--steps", type=int, default=600)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29571")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from nbdistributed_amd import ops
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification
    from nbdistributed_amd.optim import FlatAdamW
    from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
    from nbdistributed_amd.parallel.backend import init_data_plane

    init_data_plane("rccl", 0, 1, dev)
    torch.manual_seed(0)
    model = LlamaForSequenceClassification(LlamaConfig.smollm2_135m()).to(dev, torch.bfloat16)
    model.model.block_graphs = 1
    fwd = NbdDDP(model, flat_params=True, grad_mode="bucket")
    opt = FlatAdamW(fwd, lr=2e-5)
    g = torch.Generator(device=dev).manual_seed(1)
    main_b = [(torch.randint(1, 49152, (16, 128), device=dev, generator=g), torch.randint(0, 2, (16,), device=dev,
                                                                                           generator=g)) for _ in range(4)]
    odd = (torch.randint(1, 49152, (8, 256), device=dev, generator=g), torch.randint(0, 2, (8,), device=dev, generator=g))
    t0 = time.perf_counter()
    for i in range(1, a.steps + 1):
        ids, lab = odd if i % 150 == 0 else main_b[i % 4]
        loss = fwd(ids, torch.ones_like(ids), lab)[0]
        loss.backward()
        opt.step()
        opt.zero_grad()
        if i % 50 == 0:
            with torch.no_grad():
                fwd(main_b[0][0], torch.ones_like(main_b[0][0]), main_b[0][1])
        if i % 100 == 0:
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 100 * 1e3
            st = ops.block_graphs_stats()
            print(f"steps {i - 99}-{i}: {dt:.2f} ms/step  allocated {torch.cuda.memory_allocated() / 2**30:.2f} GiB "
                  f"reserved {torch.cuda.memory_reserved() / 2**30:.2f} GiB  live {st['live']} "
                  f"stack replays {st['stack_replays']} served {st['stack_served']} dropped {st['stacks_dropped']} "
                  f"eager {st['eager']}  loss {float(loss):.4f}", flush=True)
            t0 = time.perf_counter()


if __name__ == "__main__":
    main()
