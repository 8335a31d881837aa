"""GPU, ring attention at world size 4: with n >= 3 the ring's next and previous neighbours are
different peers, so the backward's two batched P2P groups in flight at once (the dK/dV
accumulators travelling with their block, and the next K/V block) go to different ranks — an
ordering that two ranks cannot exercise.

* four ranks sharing GPU 0 over gloo (what a one-GPU box can run): the HIP flash blocks, the HIP
  LSE merge and the n = 4 zigzag schedule, with P2P staged through host memory;
* four ranks on four GPUs over RCCL (the xGMI P2P path): runs on a box with >= 4 GPUs, skipped
  otherwise.

Both compare the per-rank output and q/k/v gradients with flash attention on the unsplit
sequence (causal, grouped-query, zigzag and contiguous layouts)."""
import pytest

from nbdistributed_amd.session import Session

pytestmark = pytest.mark.gpu

RING4 = """
from nbdistributed_amd.parallel.context import ring_attention, shard_context
torch.manual_seed(8)
T = 1024                                   # 4 ranks x 2 zigzag chunks x 128 tokens
q = torch.randn(1, 4, T, 64, device=device, dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(1, 2, T, 64, device=device, dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(1, 2, T, 64, device=device, dtype=torch.bfloat16, requires_grad=True)
w = torch.randn(1, 4, T, 64, device=device, dtype=torch.bfloat16)
ref = nbd.ops.flash_attention(q, k, v, causal=True)
(ref.float() * w.float()).sum().backward()
def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
oks = []
for layout in ("contiguous", "zigzag"):
    sh = lambda t: shard_context(t, dim=2, layout=layout)
    ql, kl, vl = (sh(t.detach()).clone().requires_grad_() for t in (q, k, v))
    out = ring_attention(ql, kl, vl, causal=True, layout=layout)
    (out.float() * sh(w).float()).sum().backward()
    torch.cuda.synchronize()
    oks.append(_rel(out, sh(ref.detach())) < 2e-2 and _rel(ql.grad, sh(q.grad)) < 5e-2
               and _rel(kl.grad, sh(k.grad)) < 5e-2 and _rel(vl.grad, sh(v.grad)) < 5e-2)
(world_size, tuple(oks))
"""


def _run(backend, gpu_ids):
    s = Session(writer=lambda t: None)
    s.start(4, backend=backend, gpu_ids=gpu_ids, startup_timeout=600, timeout=300)
    try:
        r = s.execute(RING4, render=False)
        for rank in range(4):
            assert r.results[rank]["echo"] == "(4, (True, True))", r.results[rank]
    finally:
        s.shutdown()


def test_ring_attention_four_ranks_gloo_on_gpu0(require_gpu):
    _run("gloo", [0, 0, 0, 0])


def test_ring_attention_four_ranks_rccl(require_gpu):
    import torch

    if torch.cuda.device_count() < 4:
        pytest.skip("needs 4 GPUs (RCCL refuses two ranks on one device)")
    _run("rccl", [0, 1, 2, 3])
