#!/usr/bin/env python3
"""torch.matmul (hipBLASLt) on the GPT-2 forward shapes the HIP GEMM loses (c_attn, c_fc, mlp.c_proj)
— run under rocprofv3 --kernel-trace --stats to see which library kernels (macro tile, stream-K)
win there."""
import torch

dev = torch.device("cuda")
for n, k in ((2304, 768), (3072, 768), (768, 3072)):
    x = torch.randn(8192, k, device=dev).to(torch.bfloat16)
    w = (torch.randn(n, k, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(n, device=dev).to(torch.bfloat16)
    for _ in range(30):
        torch.nn.functional.linear(x, w, b)
    torch.cuda.synchronize()
print("done")
