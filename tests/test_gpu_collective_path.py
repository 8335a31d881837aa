"""GPU: the multi-GPU code paths exercised on ONE MI355X, from notebook cells over the registered
``rccl`` backend.

* every collective flavour a cell may type (reference ``README.md:106-124``,
  ``worker.py:151``): all_reduce ops, reduce_scatter_tensor / all_gather_into_tensor (also in
  place, as ZeRO-2 issues them), all_to_all_single, reduce / gather / scatter, object
  collectives, barrier(device_ids=...), point-to-point to this rank, new_group and ParallelMesh
  subgroups through the ``rccl`` creator;
* DistributedDataParallel with ``force_collectives=True``: the world > 1 path (per-bucket
  collectives on the side stream, per-bucket events, in-place ZeRO-2 reduce-scatter / all-gather,
  RCCL inside a captured HIP graph, FlatAdamW updating each bucket once its all-reduce landed)
  against the world-1 path, which issues no collective;
* no_sync gradient accumulation with a weight used twice per pass;
* the GEMM next-weight warm-up under graph capture: a graph whose warm-up
  reads another model's weight keeps that storage alive, and replays bit-identically to a graph
  captured with the warm-up off after that model is deleted and the cache emptied.
"""
import pytest

from nbdistributed_amd.session import Session

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sess(require_gpu):
    s = Session(writer=lambda t: None)
    s.start(1, startup_timeout=600, timeout=600)
    yield s
    s.shutdown()


def _echo(r):
    assert r.ok, r.errors
    return r.results[0]["echo"]


CODE_SURFACE = """
import torch.distributed as dist
from nbdistributed_amd.parallel import ParallelMesh, batch_isend_irecv
ok = {}
n, dv = world_size, device
ok['backend'] = dist.get_backend() == 'rccl'
x = torch.full((1024,), 2.0, device=dv, dtype=torch.bfloat16)
dist.all_reduce(x, op=dist.ReduceOp.SUM); ok['ar_sum'] = bool((x == 2.0 * n).all())
dist.all_reduce(x, op=dist.ReduceOp.AVG); ok['ar_avg'] = bool((x == 2.0 * n).all())
y = torch.full((64,), float(rank), device=dv)
dist.all_reduce(y, op=dist.ReduceOp.MAX); ok['ar_max'] = bool((y == n - 1).all())
inp = torch.arange(8 * n, device=dv, dtype=torch.float32)
out = torch.empty(8, device=dv)
dist.reduce_scatter_tensor(out, inp); ok['rs'] = torch.equal(out, inp[rank * 8:(rank + 1) * 8] * n)
# in place, as ZeRO-2 issues it: the output is this rank's slice of the input buffer
buf = torch.arange(8 * n, device=dv, dtype=torch.bfloat16)
ref = buf.clone()
dist.reduce_scatter_tensor(buf[rank * 8:(rank + 1) * 8], buf); ok['rs_inplace'] = torch.equal(buf[rank * 8:(rank + 1) * 8], ref[rank * 8:(rank + 1) * 8] * n)
full = torch.zeros(16 * n, device=dv, dtype=torch.bfloat16)
full[rank * 16:(rank + 1) * 16] = rank + 1
dist.all_gather_into_tensor(full, full[rank * 16:(rank + 1) * 16]); ok['ag_inplace'] = all(bool((full[r * 16:(r + 1) * 16] == r + 1).all()) for r in range(n))
g = torch.empty(4 * n, device=dv)
dist.all_gather_into_tensor(g, torch.full((4,), float(rank), device=dv)); ok['ag'] = torch.equal(g, torch.arange(n, device=dv).repeat_interleave(4).float())
a2a_in = torch.arange(4 * n, device=dv, dtype=torch.float32) + 100 * rank
a2a_out = torch.empty_like(a2a_in)
dist.all_to_all_single(a2a_out, a2a_in); ok['a2a'] = torch.equal(a2a_out.view(n, 4)[0], (torch.arange(4, device=dv) + rank * 4).float())
r_ = torch.ones(32, device=dv); dist.reduce(r_, dst=0); ok['reduce'] = rank != 0 or bool((r_ == n).all())
gl = [torch.empty(8, device=dv) for _ in range(n)] if rank == 0 else None
dist.gather(torch.full((8,), float(rank), device=dv), gl, dst=0); ok['gather'] = rank != 0 or all(bool((t == i).all()) for i, t in enumerate(gl))
sc = torch.empty(8, device=dv)
dist.scatter(sc, [torch.full((8,), float(i), device=dv) for i in range(n)] if rank == 0 else None, src=0); ok['scatter'] = bool((sc == rank).all())
objs = [None] * n; dist.all_gather_object(objs, {'rank': rank}); ok['ag_object'] = objs == [{'rank': i} for i in range(n)]
ol = [{'k': 'v'} if rank == 0 else None]; dist.broadcast_object_list(ol, src=0); ok['bcast_object'] = ol[0] == {'k': 'v'}
dist.barrier(device_ids=[device.index]); ok['barrier'] = True
s_ = torch.randn(256, device=dv); r2 = torch.empty(256, device=dv)
ws = batch_isend_irecv([dist.P2POp(dist.isend, s_, rank), dist.P2POp(dist.irecv, r2, rank)])
for w in ws: w.wait()
ok['p2p_self'] = torch.equal(s_, r2)
# torch's own batch_isend_irecv also takes a self-peer on RCCL (one ncclGroup with the send and
# the receive); gloo refuses it, which is what parallel.p2p serves
r3 = torch.zeros(256, device=dv)
for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, s_, rank), dist.P2POp(dist.irecv, r3, rank)]): w.wait()
ok['torch_p2p_self_rccl'] = torch.equal(s_, r3)
sub = dist.new_group([0]); t = torch.ones(16, device=dv)
dist.all_reduce(t, group=sub); ok['subgroup'] = bool((t == 1).all()) and dist.get_backend(sub) == 'rccl'
mesh = ParallelMesh(dp=n); t2 = torch.ones(16, device=dv); dist.all_reduce(t2, group=mesh.group('dp')); ok['mesh'] = bool((t2 == n).all())
torch.cuda.synchronize()
sorted(k for k, v in ok.items() if not v)
"""


def test_rccl_collective_surface_from_a_cell(sess):
    assert _echo(sess.execute(CODE_SURFACE, render=False)) == "[]"


CODE_FORCED = """
import copy
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
from nbdistributed_amd.graphs import GraphedStep
cfg = GPT2Config(vocab_size=4096, n_positions=256, n_embd=256, n_layer=2, n_head=4)
torch.manual_seed(0)
base = GPT2(cfg).to(device, torch.bfloat16)
ids = torch.randint(0, 4096, (4, 256), generator=torch.Generator().manual_seed(1)).to(device)
def run(force, shard=False, graph=False, steps=4, overlap=False):
    m = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", shard=shard, bucket_cap_mb=1.0,
               first_bucket_mb=0.25, force_collectives=force)
    opt = FlatAdamW(m, lr=1e-3, capturable=graph, overlap=overlap)
    assert opt.overlap == overlap
    def step(x):
        _, loss = m(x, x, return_logits=False)
        loss.backward()
        opt.step(); opt.zero_grad()
        return loss.detach()
    fn = GraphedStep(step, (ids,), warmup=2, optimizers=[opt]) if graph else step
    losses = [fn(ids).float().item() for _ in range(steps)]
    params = torch.cat([b.param_flat.float() for b in m.buckets])
    return losses, params, m._collectives, len(m.buckets)
l0, p0, c0, nb = run(False)
l1, p1, c1, _ = run(True)
l2, p2, _, _ = run(True, shard=True)
l3, p3, _, _ = run(True, graph=True)
l4, p4, _, _ = run(False, graph=True)
l5, p5, _, _ = run(True, overlap=True)   # each bucket updated on the update stream once its all-reduce landed
def close(a, b):
    return (a - b).abs().max().item() <= 1e-6 + 1e-3 * b.abs().max().item()
def lclose(a, b):
    return max(abs(x - y) for x, y in zip(a, b)) <= 1e-3
(c0, c1, nb > 2, l0[0] == l1[0], lclose(l1, l0), lclose(l2, l0), lclose(l3, l4), close(p1, p0), close(p2, p0), close(p3, p4),
 l5 == l1, torch.equal(p5, p1))
"""


def test_forced_collective_path_matches_world1_path(sess):
    """The world>1 DDP path on one GPU: side-stream all-reduce per bucket, ZeRO-2 in-place
    reduce-scatter/all-gather, and the same inside a captured HIP graph, all match the
    collective-free world-1 path."""
    out = _echo(sess.execute(CODE_FORCED, render=False))
    assert out == "(False, True, True, True, True, True, True, True, True, True, True, True)", out


CODE_NOSYNC_TWICE = """
import contextlib, copy
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from torch.nn.parallel import DistributedDataParallel as TorchDDP
class Twice(torch.nn.Module):
    # self.a is used twice per forward: the engine sums its two gradient contributions
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(256, 256)
        self.b = torch.nn.Linear(256, 128)
    def forward(self, x):
        return self.b(torch.relu(self.a(torch.relu(self.a(x)))))
res = []
for dt in (torch.float32, torch.bfloat16):
    torch.manual_seed(3)
    base = Twice().to(device, dt)
    xs = [torch.randn(512, 256, device=device, dtype=dt) for _ in range(3)]
    ref = copy.deepcopy(base).float()
    rd = TorchDDP(ref, device_ids=[device.index])
    nd = NbdDDP(copy.deepcopy(base), force_collectives=False)
    for m, cast in ((rd, torch.float32), (nd, dt)):
        for i, x in enumerate(xs):
            ctx = m.no_sync() if i < len(xs) - 1 else contextlib.nullcontext()
            with ctx:
                m(x.to(cast)).float().square().mean().backward()
    torch.cuda.synchronize()
    err = max(float((p.grad.float() - q.grad).abs().max() / q.grad.abs().max())
              for p, q in zip(nd.module.parameters(), ref.parameters()))
    res.append((nd.stats["fused_linears"], err < (1e-5 if dt == torch.float32 else 3e-2)))
    del rd, nd
res
"""


def test_no_sync_weight_used_twice_matches_torch_ddp(sess):
    """k=3 micro-batches (two under no_sync) of a module that applies one nn.Linear twice:
    gradients written in place into the bucket must equal torch DDP's (no micro-batch lost,
    none counted twice)."""
    out = _echo(sess.execute(CODE_NOSYNC_TWICE, render=False))
    assert out == "[(2, True), (2, True)]", out


CODE_WARM = """
import copy, gc, os
from nbdistributed_amd import ops
assert ops.native_available()
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
from nbdistributed_amd.graphs import GraphedStep
cfg = GPT2Config(vocab_size=4096, n_positions=256, n_embd=512, n_layer=2, n_head=8)
ids = torch.randint(0, 4096, (4, 256), generator=torch.Generator().manual_seed(2)).to(device)
def make(seed):
    torch.manual_seed(seed)
    m = NbdDDP(GPT2(cfg).to(device, torch.bfloat16), flat_params=True, grad_mode="bucket")
    opt = FlatAdamW(m, lr=1e-3, capturable=True)
    def step(x):
        _, loss = m(x, x, return_logits=False)
        loss.backward()
        opt.step(); opt.zero_grad()
        return loss.detach()
    return m, opt, step
def capture(warm):
    os.environ["NBD_GEMM_WARM"] = "1" if warm else "0"
    torch.ops.nbd.gemm_warm_reset()
    a, oa, sa = make(0)
    b, ob, sb = make(1)
    for _ in range(3):          # interleave A and B: A's last product -> B's first weight is learned
        sa(ids); sb(ids)
    torch.cuda.synchronize()
    ga = GraphedStep(sa, (ids,), warmup=1, optimizers=[oa])
    refs = len(ga._warm_refs)
    del b, ob, sb                # B goes away while A's graph may have warmed B's weights
    gc.collect(); torch.cuda.synchronize(); torch.cuda.empty_cache()
    losses = [ga(ids).float().item() for _ in range(5)]
    params = torch.cat([bk.param_flat.float() for bk in a.buckets])
    del ga, a, oa, sa
    gc.collect(); torch.cuda.empty_cache()
    return refs, losses, params
r_on, l_on, p_on = capture(True)
r_off, l_off, p_off = capture(False)
os.environ["NBD_GEMM_WARM"] = "1"
(r_on > 0, r_off == 0, l_on == l_off, torch.equal(p_on, p_off))
"""


def test_gemm_warmup_is_capture_safe(sess):
    out = _echo(sess.execute(CODE_WARM, render=False))
    assert out == "(True, True, True, True)", out


CODE_LIFETIME = """
import gc
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
from nbdistributed_amd.ops import graddst
torch.manual_seed(0)
net = torch.nn.Sequential(torch.nn.Linear(256, 512), torch.nn.GELU(), torch.nn.Linear(512, 256)).to(device, torch.bfloat16)
x = torch.randn(64, 256, device=device, dtype=torch.bfloat16)
gc.collect()
c0 = graddst.count()  # registrations of other cells' models still alive in this worker
counts = []
for i in range(4):   # a notebook re-running the cell that wraps the same module
    d = NbdDDP(net, flat_params=True, grad_mode="bucket")
    d(x).float().square().mean().backward()
    counts.append(graddst.count() - c0)
    patched = sum("forward" in m.__dict__ for m in net.modules())
    del d
    gc.collect()
after = graddst.count() - c0
unpatched = sum("forward" in m.__dict__ for m in net.modules())
# FlatAdamW(overlap=True) updates during backward: clipping afterwards must refuse, and leave no
# stale coefficient behind (the next step still runs)
d = NbdDDP(net, flat_params=True, grad_mode="bucket")
o = FlatAdamW(d, lr=1e-3, overlap=True)
d(x).float().square().mean().backward()
try:
    o.clip_grad_norm_(1.0)
    clip = "no error"
except RuntimeError:
    clip = "refused"
o.step(); o.zero_grad()
d(x).float().square().mean().backward()
o.step()
torch.cuda.synchronize()
(counts, after, patched, unpatched, clip, o._clip_coef is None)
"""


def test_ddp_lifetime_and_overlap_clip(sess):
    """Re-creating DDP on the same module keeps one set of gradient-destination registrations
    (the dropped DDP's finalizer removes its own), and FlatAdamW(overlap=True) refuses
    clip_grad_norm_ without leaving a stale coefficient."""
    out = _echo(sess.execute(CODE_LIFETIME, render=False))
    assert out == "([4, 4, 4, 4], 0, 2, 0, 'refused', True)", out
