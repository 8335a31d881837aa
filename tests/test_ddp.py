"""nbd DistributedDataParallel vs torch DDP (CPU/gloo, 2 ranks, run through notebook cells)."""
import pytest

from nbdistributed_amd.session import Session

SETUP = """
import contextlib
import copy
import torch.nn as nn
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from torch.nn.parallel import DistributedDataParallel as TorchDDP

class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(32, 64)
        self.b = nn.Linear(64, 64)
        self.unused = nn.Linear(64, 64)   # never used in forward
        self.c = nn.Linear(64, 8)
        self.register_buffer("steps", torch.zeros(1))
    def forward(self, x):
        return self.c(torch.relu(self.b(torch.relu(self.a(x)))))

torch.manual_seed(1234 + rank)        # different init per rank: DDP must broadcast rank 0's
base = Net()
ref = TorchDDP(copy.deepcopy(base), find_unused_parameters=True)
ours = NbdDDP(copy.deepcopy(base), bucket_cap_mb=0.01, first_bucket_mb=0.005)
len(ours.buckets)
"""

STEP = """
def run(model, accum):
    g = torch.Generator().manual_seed(99 + rank)
    for p in model.parameters():
        p.grad = None
    for i in range(accum):
        x = torch.randn(16, 32, generator=g)
        ctx = model.no_sync() if i < accum - 1 else contextlib.nullcontext()
        with ctx:
            model(x).square().mean().backward()
    return [None if p.grad is None else p.grad.clone() for p in model.module.parameters()]

import contextlib
ok = []
for accum in (1, 3):
    gr = run(ref, accum)
    go = run(ours, accum)
    for a, b in zip(gr, go):
        if a is None:
            ok.append(b is None or float(b.abs().max()) == 0.0)
        else:
            ok.append(bool(torch.allclose(a, b, atol=1e-6, rtol=1e-5)))
same_init = all(torch.equal(p, q) for p, q in zip(ref.module.parameters(), ours.module.parameters()))
(all(ok), same_init, len(ok))
"""


@pytest.fixture(scope="module")
def sess():
    s = Session(writer=lambda t: None)
    s.start(2, backend="gloo")
    s.execute(SETUP, render=False)  # every test can run alone (pytest -k / xdist splits the module)
    yield s
    s.shutdown()


def test_nbd_ddp_matches_torch_ddp(sess):
    r = sess.execute(SETUP, render=False)
    assert int(r.results[0]["output"]) > 1  # several buckets
    r = sess.execute(STEP, render=False)
    for rank in (0, 1):
        assert r.results[rank]["output"] == "(True, True, 16)", r.results[rank]


def test_bf16_wire_dtype_close_to_fp32(sess):
    code = """
m32 = NbdDDP(copy.deepcopy(base))
m16 = NbdDDP(copy.deepcopy(base), comm_dtype=torch.bfloat16)
x = torch.randn(16, 32, generator=torch.Generator().manual_seed(rank))
for m in (m32, m16):
    m(x).square().mean().backward()
errs = [float((p.grad - q.grad).abs().max() / (p.grad.abs().max() + 1e-12))
        for p, q in zip(m32.module.parameters(), m16.module.parameters()) if p.grad is not None]
max(errs) < 1e-2
"""
    r = sess.execute(code, render=False)
    assert r.results[0]["output"] == "True" and r.results[1]["output"] == "True"


def test_torch_ddp_with_fused_comm_hooks(sess):
    code = """
from nbdistributed_amd.parallel import bf16_compress_hook, allreduce_hook
torch.manual_seed(0)
net = nn.Sequential(nn.Linear(32, 256), nn.ReLU(), nn.Linear(256, 4))
outs = []
for hook in (None, allreduce_hook, bf16_compress_hook):
    m = TorchDDP(copy.deepcopy(net))
    if hook is not None:
        m.register_comm_hook(None, hook)
    x = torch.randn(8, 32, generator=torch.Generator().manual_seed(rank))
    m(x).sum().backward()
    outs.append(torch.cat([p.grad.flatten() for p in m.parameters()]))
(bool(torch.allclose(outs[0], outs[1], atol=1e-6)), bool(torch.allclose(outs[0], outs[2], atol=2e-2, rtol=2e-2)))
"""
    r = sess.execute(code, render=False)
    assert r.results[0]["output"] == "(True, True)", r.results[0]


def test_models_forward_backward_tiny(sess):
    code = """
from nbdistributed_amd.models import GPT2, GPT2Config, synthetic_mrpc
m = NbdDDP(GPT2(GPT2Config.tiny()))
idx = torch.randint(0, 512, (2, 32))
logits, loss = m(idx, idx)
loss.backward()
ids, mask, labels = synthetic_mrpc(n=8, seq_len=16, vocab=100)
(tuple(logits.shape), bool(torch.isfinite(loss)), tuple(ids.shape), int(labels.numel()))
"""
    r = sess.execute(code, render=False)
    assert r.results[0]["output"] == "((2, 32, 512), True, (8, 16), 8)"


def test_broadcast_params_coalesced(sess):
    code = """
from nbdistributed_amd.parallel import broadcast_params
torch.manual_seed(rank)
net = nn.Sequential(nn.Linear(8, 8), nn.BatchNorm1d(8), nn.Linear(8, 3).to(torch.bfloat16))
net[1].num_batches_tracked += 5 * rank
broadcast_params(net, src=1)
sig = torch.cat([t.detach().float().reshape(-1) for t in list(net.parameters()) + list(net.buffers())])
ref = sig.clone(); dist.broadcast(ref, src=1)
(bool(torch.equal(sig, ref)), int(net[1].num_batches_tracked))
"""
    r = sess.execute(code, render=False)
    for rank in (0, 1):
        assert r.results[rank]["output"] == "(True, 5)", r.results[rank]


def test_no_sync_accumulation_matches_torch_ddp_exactly(sess):
    """k micro-batches under no_sync() then one synchronised backward: the local pre-reduce into
    the bucket (K3, accumulate="bucket") gives torch DDP's gradients bit for bit (fp32: the same
    additions in the same order; the average is exact at world 2), as does accumulate="grad"."""
    code = """
def _acc(model, k):
    g = torch.Generator().manual_seed(7 + rank)
    for p in model.parameters():
        p.grad = None
    seen_none = True
    for i in range(k):
        x = torch.randn(16, 32, generator=g)
        ctx = model.no_sync() if i < k - 1 else contextlib.nullcontext()
        with ctx:
            model(x).square().mean().backward()
        if i < k - 1 and isinstance(model, NbdDDP) and model.accumulate == "bucket":
            seen_none &= all(p.grad is None for p in model.module.parameters())
    return [None if p.grad is None else p.grad.clone() for p in model.module.parameters()], seen_none

tref = TorchDDP(copy.deepcopy(base), find_unused_parameters=True)
res = []
for mode in ("bucket", "grad"):
    mine = NbdDDP(copy.deepcopy(base), bucket_cap_mb=0.01, first_bucket_mb=0.005, accumulate=mode)
    for k in (1, 2, 4):
        gr, _ = _acc(tref, k)
        go, released = _acc(mine, k)
        same = all((a is None and (b is None or not b.any())) or (a is not None and torch.equal(a, b))
                   for a, b in zip(gr, go))
        res.append(same and released)
res
"""
    r = sess.execute(code, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "[True, True, True, True, True, True]", r.results[rank]


def test_cpp_bucket_hooks_match_torch_ddp(sess):
    """Bucket readiness counted by the C++ post-accumulate hooks (csrc/kernels/ddp_hooks.cpp):
    same gradients as torch DDP with an unused parameter and no_sync accumulation; a hook the
    user registers later still fires and DDP keeps working; a dropped DDP removes its hooks."""
    code = """
import gc
ours_c = NbdDDP(copy.deepcopy(base), bucket_cap_mb=0.01, first_bucket_mb=0.005, cpp_hooks=True)
assert ours_c._hook_handle is not None and not ours_c._hooks
ok = []
for accum in (1, 3, 1):
    gr = run(ref, accum)
    go = run(ours_c, accum)
    ok += [(b is None or float(b.abs().max()) == 0.0) if a is None else bool(torch.allclose(a, b, atol=1e-6, rtol=1e-5))
           for a, b in zip(gr, go)]
seen = []
h = ours_c.module.a.weight.register_post_accumulate_grad_hook(lambda p: seen.append(1))
gr, go = run(ref, 1), run(ours_c, 1)
ok += [bool(torch.allclose(a, b, atol=1e-6, rtol=1e-5)) for a, b in zip(gr, go) if a is not None]
intact = int(torch.ops.nbd.ddp_hooks_intact(ours_c._hook_handle, ours_c.params)) == len(ours_c.params)
h.remove()
handle, params = ours_c._hook_handle, ours_c.params
del ours_c
gc.collect()
gone = int(torch.ops.nbd.ddp_hooks_intact(handle, params)) == 0
(all(ok), seen == [1], intact, gone)
"""
    sess.execute(SETUP, render=False)
    sess.execute(STEP, render=False)  # defines run()
    r = sess.execute(code, render=False)
    for rank in (0, 1):
        assert r.results[rank]["output"] == "(True, True, True, True)", r.results[rank]


def test_rerun_cell_ddp_leaves_no_dead_hook_layers(sess):
    """A notebook cell that builds DDP over the same module again: the new DDP's hooks wrap the
    old ones (the old DDP is still alive then); once the old one is collected its hook layer is
    spliced out of the chain — one BucketHook per parameter, gradients still torch DDP's."""
    code = """
import gc
m = copy.deepcopy(base)
d1 = NbdDDP(m, bucket_cap_mb=0.01, first_bucket_mb=0.005, cpp_hooks=True)
d2 = NbdDDP(m, bucket_cap_mb=0.01, first_bucket_mb=0.005, cpp_hooks=True)   # the re-run cell
p0 = m.a.weight
both = int(torch.ops.nbd.ddp_hooks_depth(p0))
del d1
gc.collect()
after = int(torch.ops.nbd.ddp_hooks_depth(p0))
gr, go = run(ref, 1), run(d2, 1)
same = all(torch.allclose(a, b, atol=1e-6, rtol=1e-5) for a, b in zip(gr, go) if a is not None)
h2 = d2._hook_handle
del d2
gc.collect()
(both, after, same, int(torch.ops.nbd.ddp_hooks_depth(p0)))
"""
    sess.execute(SETUP, render=False)
    sess.execute(STEP, render=False)
    r = sess.execute(code, render=False)
    for rank in (0, 1):
        assert r.results[rank]["output"] == "(2, 1, True, 0)", r.results[rank]


def test_cpp_bucket_hook_callback_error_reaches_backward():
    """A failure inside the bucket callback (called from the C++ hook on the autograd engine's
    thread) surfaces as an exception from backward(), and the DDP is usable afterwards."""
    import os

    import torch
    import torch.distributed as dist

    from nbdistributed_amd import ops
    from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP

    if not ops.native_available():
        pytest.skip("native ops unavailable")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29641")
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        m = NbdDDP(torch.nn.Linear(8, 4), cpp_hooks=True)
        orig = m._bucket_event

        def boom(i):
            if i >= 0:
                raise ValueError("injected")
            orig(i)

        m._bucket_event = boom
        with pytest.raises(RuntimeError, match="injected"):
            m(torch.randn(3, 8)).sum().backward()
        m._bucket_event = orig
        m(torch.randn(3, 8)).sum().backward()  # rearmed by forward: works again
        assert all(p.grad is not None for p in m.module.parameters())
    finally:
        if own:
            dist.destroy_process_group()
