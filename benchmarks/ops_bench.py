#!/usr/bin/env python3
"""Microbenchmarks of the HIP hot-path kernels vs the PyTorch eager equivalents.

    python benchmarks/ops_bench.py [--json out.json]

Bytes counted = bytes each op must read + write (compulsory traffic); GB/s = bytes / median time
(HIP events, 5 warm-up + 20 timed).  HBM roof on MI355X ≈ 6.3 TB/s measured for a float4 copy
(MI355X_MICROARCH.md).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from nbdistributed_amd import ops  # noqa: E402


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def host_us(fn, n=50):
    """CPU wall time of one call (launch + argument marshalling), no device sync inside."""
    import time

    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    return dt


def gpt2_like_shapes(total_params: int = 124_439_808):
    # GPT-2 small parameter tensors (wte, wpe, 12 x block, ln_f); used as the bucket contents
    d, v, ctx = 768, 50257, 1024
    shapes = [(v, d), (ctx, d)]
    for _ in range(12):
        shapes += [(d,), (d,), (d, 3 * d), (3 * d,), (d, d), (d,), (d,), (d,), (d, 4 * d), (4 * d,), (4 * d, d), (d,)]
    shapes += [(d,), (d,)]
    return shapes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default="", help="comma list of: flatten,unflatten,prereduce,summary,adamw,xent,attn")
    a = ap.parse_args()
    only = set(filter(None, a.only.split(",")))

    def want(k):
        return not only or k in only

    dev = torch.device("cuda", 0)
    assert ops.native_available(), ops._load_error
    res = {}

    if want("flatten") or want("unflatten"):
        bench_bucket(res, dev)
    if want("prereduce"):
        bench_prereduce(res, dev)
    if want("summary"):
        bench_summary(res, dev)
    if want("adamw"):
        bench_adamw(res, dev)
    if want("xent"):
        bench_xent(res, dev)
    if want("attn"):
        bench_attn(res, dev)
    torch.cuda.synchronize()
    for k, v in res.items():
        print(f"{k:28s} " + " ".join(f"{kk}={vv:.4g}" if isinstance(vv, float) else f"{kk}={vv}" for kk, vv in v.items()))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


def bench_bucket(res, dev):
    # K1: flatten 124M fp32 grads (GPT-2 small) -> bf16 bucket, scale 1/8
    grads = [torch.randn(s, device=dev) for s in gpt2_like_shapes()]
    numel = sum(g.numel() for g in grads)
    offs, total = ops.plan_offsets([g.numel() for g in grads])
    bucket = torch.empty(total, device=dev, dtype=torch.bfloat16)
    byts = numel * 4 + numel * 2
    t_hip = timeit(lambda: ops.bucket_flatten(grads, bucket, offs, scale=0.125))

    def torch_flat():
        return torch.cat([g.reshape(-1) for g in grads]).to(torch.bfloat16).mul_(0.125)

    t_torch = timeit(torch_flat)
    res["flatten_fp32_to_bf16"] = {"numel": numel, "hip_ms": t_hip, "torch_ms": t_torch,
                                   "hip_GBps": byts / t_hip / 1e6, "torch_GBps": byts / t_torch / 1e6,
                                   "speedup": t_torch / t_hip,
                                   "host_us": host_us(lambda: ops.bucket_flatten(grads, bucket, offs, scale=0.125))}

    # same bytes as ONE tensor: isolates the per-block chunk->tensor lookup and tensor-tail cost
    one = torch.randn(numel, device=dev)
    t_one = timeit(lambda: ops.bucket_flatten([one], bucket, [0], scale=0.125))
    res["flatten_single_tensor"] = {"hip_ms": t_one, "hip_GBps": byts / t_one / 1e6}
    # 148 tensors that are views into that one allocation: same lookup work, contiguous memory
    views, pos = [], 0
    for g in grads:
        views.append(one[pos:pos + g.numel()])
        pos += (g.numel() + 63) // 64 * 64 if pos + (g.numel() + 63) // 64 * 64 <= one.numel() else g.numel()
    t_views = timeit(lambda: ops.bucket_flatten(views, bucket, offs, scale=0.125))
    res["flatten_views_one_alloc"] = {"hip_ms": t_views, "hip_GBps": byts / t_views / 1e6}
    del one, views

    # K2: unflatten bf16 bucket -> fp32 grads, x 1/8 (DDP average) ; torch: per-tensor copy_
    def torch_unflat():
        for g, o in zip(grads, offs):
            g.view(-1).copy_(bucket[o:o + g.numel()].float().mul_(0.125))

    t_hip = timeit(lambda: ops.bucket_unflatten(bucket, grads, offs, scale=0.125))
    t_torch = timeit(torch_unflat)
    res["unflatten_bf16_to_fp32"] = {"hip_ms": t_hip, "torch_ms": t_torch, "hip_GBps": byts / t_hip / 1e6,
                                     "torch_GBps": byts / t_torch / 1e6, "speedup": t_torch / t_hip}
    t_hip = timeit(lambda: ops.bucket_unflatten(bucket, grads, offs, scale=0.125, accumulate=True))
    res["unflatten_accumulate"] = {"hip_ms": t_hip, "hip_GBps": (numel * 2 + numel * 8) / t_hip / 1e6}


def bench_prereduce(res, dev):
    # K3: pre-reduce 4 bf16 buffers of 128 Mi elements -> bf16
    n = 128 << 20
    xs = [torch.randn(n, device=dev, dtype=torch.bfloat16) for _ in range(4)]
    out = torch.empty(n, device=dev, dtype=torch.bfloat16)
    byts = n * 2 * 5
    t_hip = timeit(lambda: ops.local_prereduce(xs, out, scale=0.25))

    def torch_pre():
        acc = xs[0].float()
        for x in xs[1:]:
            acc += x
        out.copy_(acc.mul_(0.25))

    t_torch = timeit(torch_pre)
    res["prereduce_4x_bf16"] = {"numel": n, "hip_ms": t_hip, "torch_ms": t_torch, "hip_GBps": byts / t_hip / 1e6,
                                "torch_GBps": byts / t_torch / 1e6, "speedup": t_torch / t_hip}
    del xs, out
    # K3 on DDP's no_sync path (parallel/ddp.py _prereduce_local, buckets without gradient views):
    # one micro-batch's bf16 gradients summed into a 64 MiB bf16 bucket (fp32 math, one rounding),
    # GPT-2 block shapes filling the bucket; bytes = gradients read + bucket read + bucket written
    d = 768
    block = [(d,), (d,), (d, 3 * d), (3 * d,), (d, d), (d,), (d,), (d,), (d, 4 * d), (4 * d,), (4 * d, d), (d,)]
    shapes, numel = [], 0
    while True:
        for s in block:
            k = 1
            for x in s:
                k *= x
            if (numel + k) * 2 > (64 << 20):
                break
            shapes.append(s)
            numel += k
        else:
            continue
        break
    grads = [torch.randn(s, device=dev, dtype=torch.bfloat16) for s in shapes]
    offs, total = ops.plan_offsets([g.numel() for g in grads])
    bucket = torch.zeros(total, device=dev, dtype=torch.bfloat16)
    t_acc = timeit(lambda: ops.prereduce_into_bucket(grads, bucket, offs))

    def torch_acc():
        for g, o in zip(grads, offs):
            bucket[o:o + g.numel()].add_(g.view(-1))

    t_torch = timeit(torch_acc)
    # the same launches back to back (10 per event pair): the host's table build and launch (58
    # tensors -> a 9 KiB argument block) overlap the previous launch's GPU time, as they do inside
    # a no_sync backward — the GPU time per launch, not host latency + GPU time
    t_acc_b = timeit(lambda: [ops.prereduce_into_bucket(grads, bucket, offs) for _ in range(10)]) / 10
    t_torch_b = timeit(lambda: [torch_acc() for _ in range(10)]) / 10
    res["nosync_prereduce_64MiB"] = {"tensors": len(grads), "numel": numel, "hip_ms": t_acc, "torch_ms": t_torch,
                                     "hip_GBps": numel * 6 / t_acc / 1e6, "torch_GBps": numel * 6 / t_torch / 1e6,
                                     "speedup": t_torch / t_acc, "hip_ms_pipelined": t_acc_b,
                                     "hip_GBps_pipelined": numel * 6 / t_acc_b / 1e6, "torch_ms_pipelined": t_torch_b,
                                     "host_us": host_us(lambda: ops.prereduce_into_bucket(grads, bucket, offs))}


def bench_summary(res, dev):
    # K4: summary of 1 GiB bf16 and 512 MiB f32 vs torch's separate reductions
    for name, dt, numel in (("summary_bf16_1GiB", torch.bfloat16, 512 << 20), ("summary_f32_512MiB", torch.float32, 128 << 20)):
        x = torch.randn(numel, device=dev, dtype=dt)
        byts = x.numel() * x.element_size()
        t_hip = timeit(lambda: ops.tensor_summary_raw(x))

        def torch_sum():
            xf = x.float()
            return torch.stack([xf.sum(), xf.mean(), xf.std(), xf.norm(), xf.min(), xf.max(), xf.abs().max(),
                                torch.isnan(xf).sum().float(), torch.isinf(xf).sum().float()])

        t_torch = timeit(torch_sum)
        res[name] = {"numel": numel, "hip_ms": t_hip, "torch_ms": t_torch, "hip_GBps": byts / t_hip / 1e6,
                     "torch_GBps": byts / t_torch / 1e6, "speedup": t_torch / t_hip}
        del x


def bench_adamw(res, dev):
    # K5: one AdamW step over GPT-2 small.  HIP: one flat bucket (bf16 grad + bf16 param, fp32
    # master/m/v: 28 B/param).  torch: fused AdamW over the 148 fp32 parameters (fp32 grads;
    # also 28 B/param) — the mixed-precision recipe the flat path replaces.
    shapes = gpt2_like_shapes()
    numels = [int(torch.Size(s).numel()) for s in shapes]
    offs, total = ops.plan_offsets(numels)
    grad = torch.randn(total, device=dev, dtype=torch.bfloat16)
    param = torch.randn(total, device=dev, dtype=torch.bfloat16)
    master = param.float()
    m, v = torch.zeros_like(master), torch.zeros_like(master)
    step = [0]

    def hip_step():
        step[0] += 1
        ops.adamw_flat(grad, param, master, m, v, 1e-4, 0.9, 0.999, 1e-8, 0.1, step[0])

    t_hip = timeit(hip_step)
    byts = total * 28
    ps = [torch.nn.Parameter(torch.randn(s, device=dev)) for s in shapes]
    for p in ps:
        p.grad = torch.randn_like(p)
    opt = torch.optim.AdamW(ps, lr=1e-4, weight_decay=0.1, fused=True)
    t_torch = timeit(opt.step)
    res["adamw_gpt2_small"] = {"numel": total, "hip_ms": t_hip, "torch_fused_ms": t_torch,
                               "hip_GBps": byts / t_hip / 1e6, "torch_GBps": byts / t_torch / 1e6,
                               "speedup": t_torch / t_hip}



def bench_xent(res, dev):
    # K6: GPT-2 small LM-head loss, logits [8192, 50257] bf16: forward + backward.
    # HIP: logsumexp pass + gradient pass (2 reads + 1 write of the logits);  torch: the model's
    # previous path F.cross_entropy(logits.float()) + backward (fp32 copy, log_softmax, ...).
    import torch.nn.functional as F

    N, V = 8192, 50257
    base = (torch.randn(N, V, device=dev) * 2).to(torch.bfloat16)
    tgt = torch.randint(0, V, (N,), device=dev)

    def hip():
        x = base.detach().requires_grad_(True)
        ops.cross_entropy(x, tgt).backward()

    def hip_inplace():
        x = base.detach().requires_grad_(True)
        y = x.view(N, V)  # non-leaf alias: the gradient is written over y's storage (copy of base)
        ops.cross_entropy(y * 1, tgt, inplace_backward=True).backward()

    def eager():
        x = base.detach().requires_grad_(True)
        F.cross_entropy(x.float(), tgt).backward()

    t_hip = timeit(hip)
    t_eager = timeit(eager)
    fb = timeit(lambda: torch.ops.nbd.xent_fwd(base, tgt, -100))
    byts = N * V * 2
    res["xent_gpt2_fwd_bwd"] = {"rows": N, "vocab": V, "hip_ms": t_hip, "torch_ms": t_eager, "speedup": t_eager / t_hip,
                                "fwd_ms": fb, "fwd_GBps": byts / fb / 1e6,
                                "bwd_GBps_est": 2 * byts / max(t_hip - fb, 1e-6) / 1e6}


def bench_attn(res, dev):
    # K7: GPT-2 small attention, B=8 H=12 T=1024 D=64 causal, bf16: HIP flash vs torch SDPA
    import torch.nn.functional as F

    B, H, T, D = 8, 12, 1024, 64
    q, k, v, do = (torch.randn(B, H, T, D, device=dev, dtype=torch.bfloat16) for _ in range(4))
    flops_fwd = 4 * B * H * T * T * D / 2  # causal: half the score matrix
    for name, fn in (("hip", lambda a, b, c: ops.flash_attention(a, b, c, causal=True)),
                     ("sdpa", lambda a, b, c: F.scaled_dot_product_attention(a, b, c, is_causal=True))):
        t_f = timeit(lambda: fn(q, k, v))
        qq, kk, vv = (t.detach().requires_grad_(True) for t in (q, k, v))

        def fb():
            fn(qq, kk, vv).backward(do)

        t_fb = timeit(fb)
        res.setdefault("attn_gpt2_causal", {}).update({
            f"{name}_fwd_ms": t_f, f"{name}_fwd_bwd_ms": t_fb, f"{name}_fwd_TFs": flops_fwd / t_f / 1e9,
            f"{name}_bwd_TFs": 2.5 * flops_fwd / (t_fb - t_f) / 1e9})
    r = res["attn_gpt2_causal"]
    r["speedup_fwd"] = r["sdpa_fwd_ms"] / r["hip_fwd_ms"]
    r["speedup_fwd_bwd"] = r["sdpa_fwd_bwd_ms"] / r["hip_fwd_bwd_ms"]


if __name__ == "__main__":
    main()
