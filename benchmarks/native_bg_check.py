#!/usr/bin/env python3
"""native() with block_graphs=1 (eager backward) vs 2 (backward block graphs) on the notebook's
recipe with torch AdamW: per-step loss and the largest gradient / weight difference.

    python benchmarks/native_bg_check.py [--steps 12] [--layers 30]
"""
from __future__ import annotations

import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--layers", type=int, default=30)
    ap.add_argument("--lr", type=float, default=2e-5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    import transformers

    import nbdistributed_amd as nbd
    from nbdistributed_amd import ops
    from nbdistributed_amd.models import SMOLLM2_135M, synthetic_mrpc

    cfg = dict(SMOLLM2_135M)
    cfg.update(num_hidden_layers=a.layers)
    torch.manual_seed(0)
    hf = transformers.LlamaForSequenceClassification(transformers.LlamaConfig(num_labels=2, pad_token_id=0, **cfg))
    ms = [nbd.models.native(copy.deepcopy(hf).to(dev), block_graphs=g) for g in (1, 2)]
    opts = [torch.optim.AdamW(m.parameters(), lr=a.lr) for m in ms]
    ids, mask, labels = synthetic_mrpc(n=16 * a.steps, seq_len=128)
    names = [n for n, _ in ms[0].named_parameters()]
    for s in range(a.steps):
        sl = slice(16 * s, 16 * s + 16)
        x, mk, y = ids[sl].to(dev), mask[sl].to(dev), labels[sl].to(dev)
        losses, grads = [], []
        for m, o in zip(ms, opts):
            out = m(input_ids=x, attention_mask=mk, labels=y)
            out.loss.backward()
            losses.append(float(out.loss))
            grads.append([p.grad.detach().clone() for p in m.parameters()])
            o.step()
            o.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        gd = [(float((g1 - g2).abs().max()), n) for g1, g2, n in zip(*grads, names)]
        worst = max(gd)
        wd = max(float((p1 - p2).abs().max()) for p1, p2 in zip(ms[0].parameters(), ms[1].parameters()))
        print(f"step {s}: loss {losses[0]:.6f} / {losses[1]:.6f}  max |grad diff| {worst[0]:.3e} ({worst[1]})  "
              f"max |weight diff| {wd:.3e}  unequal grads {sum(d > 0 for d, _ in gd)}/{len(gd)}", flush=True)
    print("block graph stats", ops.block_graphs_stats(), flush=True)


if __name__ == "__main__":
    main()
