#!/usr/bin/env python3
"""Why do the HIP GEMMs run slower inside the GPT-2 step than alone?  Times the q|k|v forward
product (8192 x 2304 x 768, + bias) in one process under four conditions:

  1. random operands, back to back (the A/B benchmarks' condition)
  2. the model's real operands (layer-0 LayerNorm output, c_attn weight and bias), back to back
  3. (2) right after 20 replays of the graphed training step (the chip hot, caches holding the
     step's working set)
  4. (2) with one graphed step replayed between every two GEMMs (per-GEMM events): the
     in-step condition minus the GEMM's own neighbours

    python benchmarks/gemm_context.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nbdistributed_amd import ops  # noqa: E402
from nbdistributed_amd.ops import gemm as G  # noqa: E402


def _loop(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29731")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from nbdistributed_amd.graphs import GraphedStep
    from nbdistributed_amd.models import GPT2, GPT2Config
    from nbdistributed_amd.optim import FlatAdamW
    from nbdistributed_amd.parallel import DistributedDataParallel

    ops.load_library()
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

    g = GraphedStep(step, (x,), warmup=3, optimizers=[opt])
    blk = m.h[0]
    with torch.no_grad():
        emb = m.wte.weight[x] + m.wpe.weight[:1024]
        h = ops.layer_norm(emb, blk.ln_1.weight, blk.ln_1.bias, blk.ln_1.eps).reshape(-1, 768).contiguous()
    W, b = blk.attn.c_attn.weight.detach(), blk.attn.c_attn.bias.detach()
    tile, _ = G.config(False, False, 8192, 2304, 768, can_split=False)
    gq = torch.Generator(device="cuda").manual_seed(1)
    Ar = (torch.rand(8192, 768, device=dev, generator=gq) * 2 - 1).to(torch.bfloat16)
    Br = (torch.rand(2304, 768, device=dev, generator=gq) * 0.2 - 0.1).to(torch.bfloat16)
    real = lambda: G.matmul(h, W, bias=b, tile=tile, splits=1)  # noqa: E731
    rand = lambda: G.matmul(Ar, Br, tile=tile, splits=1)  # noqa: E731
    flops = 2.0 * 8192 * 2304 * 768
    for rnd in range(2):
        r1 = _loop(rand)
        r2 = _loop(real)
        for _ in range(20):
            g(x)
        r3 = _loop(real)
        ts = []
        for _ in range(10):
            g(x)
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            real()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        ts.sort()
        r4 = ts[len(ts) // 2]
        # which cold operand costs: touch (read) W, h or both right before the GEMM
        touched = {}
        for name, pre in (("W", lambda: W.view(-1).max()), ("h", lambda: h.view(-1).max()),
                          ("W+h", lambda: (W.view(-1).max(), h.view(-1).max()))):
            tt = []
            for _ in range(10):
                g(x)
                pre()
                s, e = torch.cuda.Event(True), torch.cuda.Event(True)
                s.record()
                real()
                e.record()
                e.synchronize()
                tt.append(s.elapsed_time(e) * 1e3)
            tt.sort()
            touched[name] = tt[len(tt) // 2]
        print(f"round {rnd}: random b2b {r1:.1f} us ({flops / r1 / 1e6:.0f} TF/s) | real b2b {r2:.1f} | real after "
              f"20 graph steps {r3:.1f} | real between graph steps (median of 10) {r4:.1f} us | after touching "
              + ", ".join(f"{k} {v:.1f}" for k, v in touched.items()), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
