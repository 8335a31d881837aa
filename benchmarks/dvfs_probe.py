import os, sys, statistics, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from nbdistributed_amd.ops import gemm as G
from nbdistributed_amd import ops
ops.load_library()
T, C, F = 8192, 768, 3072
x = (torch.rand(T, C, device="cuda") * 2 - 1).to(torch.bfloat16)
w1 = (torch.rand(F, C, device="cuda") * 0.1 - 0.05).to(torch.bfloat16)
big = [torch.empty(300 << 20, dtype=torch.uint8, device="cuda") for _ in range(2)]
def run(n, flush=False):
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(n):
        if flush: big[0].copy_(big[1])
        G.matmul(x, w1, tile=82128128, splits=1)
    e.record(); e.synchronize()
    return s.elapsed_time(e) / n * 1e3
for n in (20, 200, 2000):
    print("iters", n, "us/gemm", round(run(n), 1), flush=True)
# with a 300 MB copy between GEMMs (evicts L2/MALL): time the pair, minus the copy alone
s, e = torch.cuda.Event(True), torch.cuda.Event(True)
s.record()
for _ in range(50): big[0].copy_(big[1])
e.record(); e.synchronize(); cp = s.elapsed_time(e) / 50 * 1e3
print("copy 300MB us", round(cp, 1), "gemm after flush us", round(run(50, True) - cp, 1))
# sustained: 3 s of back-to-back GEMMs, then 20
import time
t0 = time.time()
while time.time() - t0 < 3: run(100)
print("after 3 s sustained: us/gemm", round(run(200), 1))
