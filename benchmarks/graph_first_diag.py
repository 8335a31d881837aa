#!/usr/bin/env python3
"""The bench's GPT-2 phases in one plain process (no coordinator): eager 'flat', then the graphed
step several times — to find out why the FIRST graphed phase on a box can run ~12 % slower
(docs/FINDINGS.md "open at the end of round 3").  Prints one line per phase."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from nbdistributed_amd import benchmarking as B  # noqa: E402
from nbdistributed_amd.parallel.backend import init_data_plane  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
init_data_plane("rccl", 0, 1, dev)
ns = {"torch": torch, "dist": dist, "device": dev, "rank": 0, "world_size": 1}
exec(B.AR_SETUP, ns)
exec(B.DDP_SETUP, ns)
seq = sys.argv[1].split(",") if len(sys.argv) > 1 else ["flat", "flatgraph", "flatgraph", "flat", "flatgraph"]
for impl in seq:
    t = time.time()
    ms, loss = ns["_nbd_gpt2_bench"](20, 5, 8, 1024, impl)
    print(f"{impl:10s} {ms:8.3f} ms/step  (phase {time.time() - t:.1f} s)", flush=True)
