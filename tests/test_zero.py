"""ZeRO-2 sharding (``DistributedDataParallel(shard=True)`` + ``FlatAdamW``) on the CPU/gloo data
plane: reduce-scattered gradient slices, optimizer state for this rank's slice only, parameters
rebuilt by async all-gathers waited in the pre-forward hooks — must train exactly like the
unsharded DDP + FlatAdamW (and so like torch DDP + AdamW: tests/test_optim.py)."""
import pytest

from nbdistributed_amd.session import Session

SETUP = """
import copy
import torch.nn as nn
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW

class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(32, 64)
        self.b = nn.Linear(64, 64)
        self.c = nn.Linear(64, 8)
    def forward(self, x):
        return self.c(torch.relu(self.b(torch.relu(self.a(x)))))

torch.manual_seed(7 + rank)
base = Net()
kw = dict(bucket_cap_mb=0.01, first_bucket_mb=0.005, flat_params=True, grad_mode="bucket")
full = NbdDDP(copy.deepcopy(base), **kw)
zero = NbdDDP(copy.deepcopy(base), shard=True, **kw)
opt_full = FlatAdamW(full, lr=3e-3, betas=(0.9, 0.95), weight_decay=0.05)
opt_zero = FlatAdamW(zero, lr=3e-3, betas=(0.9, 0.95), weight_decay=0.05)
state_full = sum(st["master"].numel() for st in opt_full.flat_state)
state_zero = sum(st["master"].numel() for st in opt_zero.flat_state)
(len(zero.buckets) > 1, state_zero * world_size >= state_full, state_zero < state_full or world_size == 1,
 all(b.numel % world_size == 0 and b.lo == rank * b.shard for b in zero.buckets))
"""

TRAIN = """
g = torch.Generator().manual_seed(1000 + rank)
norms = []
for step in range(5):
    x = torch.randn(16, 32, generator=g)
    with full.no_sync() if step == 1 else contextlib.nullcontext(), \\
         zero.no_sync() if step == 1 else contextlib.nullcontext():
        for model, o in ((full, opt_full), (zero, opt_zero)):
            if step != 1:  # step 1 accumulates into step 2 (no_sync)
                o.zero_grad(set_to_none=True)
            model(x).square().mean().backward()
    if step == 1:
        continue
    for o in (opt_full, opt_zero):
        if step >= 3:
            norms.append(float(o.clip_grad_norm_(0.05)))
        o.step()
zero.wait_params()
err = max(float((p - q).detach().abs().max()) for p, q in zip(full.module.parameters(), zero.module.parameters()))
norm_ok = all(abs(a - b) <= 1e-5 * max(1.0, abs(a)) for a, b in zip(norms[0::2], norms[1::2]))
# every rank holds the same full parameters
flat = torch.cat([p.detach().reshape(-1) for p in zero.module.parameters()])
same = [torch.zeros_like(flat) for _ in range(world_size)]
dist.all_gather(same, flat)
(err < 1e-6, norm_ok, len(norms), all(torch.equal(same[0], t) for t in same))
"""

STATE = """
opt_zero.step(); opt_zero.step()  # back-to-back steps (no forward between): gathers are joined first
opt_full.step(); opt_full.step()
zero.wait_params()
err2 = max(float((p - q).detach().abs().max()) for p, q in zip(full.module.parameters(), zero.module.parameters()))
assert err2 < 1e-6, err2
sd = opt_zero.state_dict()
opt2 = FlatAdamW(zero, lr=1.0)
opt2.load_state_dict(sd)
bad = dict(sd, shard={"rank": rank, "world": world_size + 1})
try:
    opt2.load_state_dict(bad)
    refused = False
except ValueError:
    refused = True
(sd["shard"] == {"rank": rank, "world": world_size}, opt2.step_count == opt_zero.step_count, refused,
 all(torch.equal(a["exp_avg"], b["exp_avg"]) for a, b in zip(opt_zero.flat_state, opt2.flat_state)))
"""


@pytest.fixture(scope="module", params=[2, 4])
def sess(request):
    s = Session(writer=lambda t: None)
    s.start(request.param, backend="gloo")
    s.execute("import contextlib", render=False)
    yield s
    s.shutdown()


def test_zero2_trains_like_unsharded_ddp(sess):
    r = sess.execute(SETUP, render=False)
    assert r.ok, r.errors
    for res in r.results.values():
        assert res["output"] == "(True, True, True, True)", res
    r = sess.execute(TRAIN, render=False)
    assert r.ok, r.errors
    for res in r.results.values():
        assert res["output"] == "(True, True, 4, True)", res
    r = sess.execute(STATE, render=False)
    assert r.ok, r.errors
    assert r.results[0]["output"] == "(True, True, True, True)", r.results[0]


def test_zero2_requires_flat_bucket_mode(sess):
    code = "NbdDDP(copy.deepcopy(base), shard=True)"
    r = sess.execute(SETUP, render=False)
    r = sess.execute(code, render=False, raise_on_error=False)
    assert not r.ok and "flat_params=True" in str(r.errors)
