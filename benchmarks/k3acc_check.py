#!/usr/bin/env python3
"""Correctness of the accumulating bucket flatten (bucket[slice] += scale * t) under the current
NBD_K3ACC_VARIANT against a PyTorch fp32 reference: mixed sizes (chunk tails, < 8-element
tails, a misaligned tensor), bf16 and fp32 buckets.  Prints OK or raises."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from nbdistributed_amd import ops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
for bdt in (torch.bfloat16, torch.float32):
    sizes = [1, 7, 8, 8191, 8192, 8193, 16383, 16384, 16385, 40000, 3, 70001, 123457]
    ts = [torch.randn(n, device=dev, generator=g).to(bdt) for n in sizes]
    ts.append(torch.randn(1001, device=dev, generator=g).to(bdt)[1:])  # misaligned source
    offs, o = [], 0
    for t in ts:
        offs.append(o)
        o += t.numel() + 8
    bucket = torch.randn(o, device=dev, generator=g).to(bdt)
    ref = bucket.float().clone()
    for t, off in zip(ts, offs):
        ref[off:off + t.numel()] += 0.5 * t.float()
    ops.bucket_flatten(ts, bucket, offs, scale=0.5, accumulate=True)
    torch.cuda.synchronize()
    err = (bucket.float() - ref).abs().max().item()
    tol = 1e-5 if bdt == torch.float32 else 0.02 * ref.abs().max().item()
    assert err <= tol, (bdt, err)
print("OK variant", os.environ.get("NBD_K3ACC_VARIANT", "0"))
