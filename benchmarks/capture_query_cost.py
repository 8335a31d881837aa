#!/usr/bin/env python3
"""Host cost of asking HIP whether the current stream is capturing (hipStreamIsCapturing through
torch.cuda.is_current_stream_capturing), as the GEMM launches do once per call."""
import time

import torch

torch.cuda.init()
s = torch.cuda.current_stream()
for _ in range(1000):
    torch.cuda.is_current_stream_capturing()
n = 20000
t = time.perf_counter()
for _ in range(n):
    torch.cuda.is_current_stream_capturing()
print(f"is_current_stream_capturing: {(time.perf_counter() - t) / n * 1e6:.3f} us/call")
