#!/usr/bin/env python3
"""Does the GPT-2 attention -> c_proj backward skip the δ pre-pass (gemm.hip EPI_ADELTA)?  Run
under rocprofv3 --kernel-trace --stats and count attn::bwd_pre_kernel: one GPT-2 small block's
attention at B8 T1024 through the model's own fast path, 3 backward passes."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from nbdistributed_amd.models import GPT2, GPT2Config  # noqa: E402

torch.manual_seed(0)
m = GPT2(GPT2Config(n_layer=1)).cuda().to(torch.bfloat16)
idx = torch.randint(0, 50257, (8, 1024), device="cuda")
for _ in range(3):
    loss = m(idx, idx, return_logits=False)[1]
    loss.backward()
torch.cuda.synchronize()
print("done", float(loss))
