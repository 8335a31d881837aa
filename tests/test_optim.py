"""FlatAdamW (bucket-resident fused AdamW) vs torch.optim.AdamW — CPU reference path and
2-rank gloo DDP through notebook cells.  The GPU kernel is checked in test_gpu_ops.py."""
import pytest
import torch

from nbdistributed_amd import ops
from nbdistributed_amd.session import Session


@pytest.mark.parametrize("wd", [0.0, 0.1])
def test_reference_adamw_matches_torch(wd):
    torch.manual_seed(0)
    p_ref = torch.nn.Parameter(torch.randn(1001))
    opt = torch.optim.AdamW([p_ref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=wd)
    param = p_ref.detach().clone()
    master, m, v = param.clone(), torch.zeros_like(param), torch.zeros_like(param)
    for step in range(1, 6):
        g = torch.randn(1001)
        p_ref.grad = g.clone()
        opt.step()
        ops.adamw_flat(g, param, master, m, v, 1e-2, 0.9, 0.95, 1e-8, wd, step)
    assert torch.allclose(param, p_ref.detach(), atol=1e-6, rtol=1e-5)
    st = opt.state[p_ref]
    assert torch.allclose(m, st["exp_avg"], atol=1e-7) and torch.allclose(v, st["exp_avg_sq"], atol=1e-8)


def test_reference_adamw_bf16_param_keeps_fp32_master():
    param = torch.zeros(64, dtype=torch.bfloat16)
    master = torch.zeros(64)
    m, v = torch.zeros(64), torch.zeros(64)
    for step in range(1, 4):
        ops.adamw_flat(torch.full((64,), 1.0, dtype=torch.bfloat16), param, master, m, v, 1e-4, 0.9, 0.999, 1e-8, 0.0,
                       step)
    assert torch.allclose(master, torch.full((64,), -3e-4), atol=1e-7)
    assert param.dtype == torch.bfloat16 and torch.equal(param, master.to(torch.bfloat16))


def test_reference_adamw_device_scale_tensor():
    g = torch.randn(100)
    outs = []
    for scale, t in ((0.5, None), (1.0, torch.tensor([0.5]))):
        p = torch.zeros(100)
        mm, m, v = p.clone(), torch.zeros(100), torch.zeros(100)
        ops.adamw_flat(g, p, mm, m, v, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1, grad_scale=scale, grad_scale_t=t)
        outs.append((m.clone(), p.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


SETUP = """
import copy
import torch.nn as nn
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
from torch.nn.parallel import DistributedDataParallel as TorchDDP

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
ref = TorchDDP(copy.deepcopy(base))
ours = NbdDDP(copy.deepcopy(base), bucket_cap_mb=0.01, first_bucket_mb=0.005, flat_params=True, grad_mode="bucket")
opt_ref = torch.optim.AdamW(ref.parameters(), lr=3e-3, betas=(0.9, 0.95), weight_decay=0.05)
opt = FlatAdamW(ours, lr=3e-3, betas=(0.9, 0.95), weight_decay=0.05)
views = all(p.data_ptr() >= b.param_flat.data_ptr() for b in ours.buckets for p in b.params)
(len(ours.buckets), views)
"""

TRAIN = """
g = torch.Generator().manual_seed(1000 + rank)
norms = []
for step in range(4):
    x = torch.randn(16, 32, generator=g)
    for model, o in ((ref, opt_ref), (ours, opt)):
        o.zero_grad(set_to_none=True)
        model(x).square().mean().backward()
        if step >= 2:
            if o is opt:
                norms.append(float(o.clip_grad_norm_(0.05)))
            else:
                norms.append(float(torch.nn.utils.clip_grad_norm_(model.parameters(), 0.05)))
        o.step()
err = max(float((p - q).detach().abs().max()) for p, q in zip(ref.module.parameters(), ours.module.parameters()))
grads_released = all(p.grad is None for p in ours.module.parameters())
norm_ok = all(abs(a - b) <= 1e-5 * max(1.0, abs(a)) for a, b in zip(norms[0::2], norms[1::2]))
(err < 1e-5, grads_released, norm_ok, len(norms))
"""

STATE = """
sd = opt.state_dict()
opt2 = FlatAdamW(ours, lr=1.0)
opt2.load_state_dict(sd)
(opt2.step_count == opt.step_count, opt2.param_groups[0]["lr"] == 3e-3,
 all(torch.equal(a["exp_avg"], b["exp_avg"]) for a, b in zip(opt.flat_state, opt2.flat_state)))
"""


@pytest.fixture(scope="module")
def sess():
    s = Session(writer=lambda t: None)
    s.start(2, backend="gloo")
    # every test can run alone (pytest-xdist spreads a module's tests over processes)
    assert s.execute(SETUP, render=False).ok
    yield s
    s.shutdown()


def test_flat_adamw_ddp_matches_torch_ddp_adamw(sess):
    r = sess.execute(SETUP, render=False)
    assert r.ok, r.errors
    nb, views = eval(r.results[0]["output"])
    assert nb > 1 and views
    r = sess.execute(TRAIN, render=False)
    assert r.ok, r.errors
    for rank in (0, 1):
        assert r.results[rank]["output"] == "(True, True, True, 4)", r.results[rank]
    r = sess.execute(STATE, render=False)
    assert r.results[0]["output"] == "(True, True, True)", r.results[0]


def test_flat_adamw_drives_lr_scheduler(sess):
    code = ("sch = torch.optim.lr_scheduler.LambdaLR(opt, lambda s: 0.5)\n"
            "sch.step()\n"
            "(isinstance(opt, torch.optim.Optimizer), opt.param_groups[0]['lr'])")
    r = sess.execute(code, render=False)
    assert r.results[0]["echo"] == "(True, 0.0015)", r.results[0]


def test_flat_adamw_requires_bucket_mode(sess):
    r = sess.execute("FlatAdamW(NbdDDP(copy.deepcopy(base)))", render=False, raise_on_error=False)
    assert not r.ok and "flat_params=True" in str(r.errors)


def test_fast_adamw_falls_back_to_torch_off_gpu_and_survives_an_lr_scheduler():
    """optim.install_fast_adamw binds the HIP step to the instance: an LR scheduler wraps it as it
    wraps torch's (it reads ``step.__func__``), and off the GPU the update is torch's own."""
    from nbdistributed_amd.optim import install_fast_adamw

    torch.manual_seed(0)
    a = torch.nn.Linear(16, 8)
    b = torch.nn.Linear(16, 8)
    b.load_state_dict(a.state_dict())
    oa = torch.optim.AdamW(a.parameters(), lr=1e-2, weight_decay=0.1)
    ob = torch.optim.AdamW(b.parameters(), lr=1e-2, weight_decay=0.1)
    installed = install_fast_adamw(ob)
    assert installed == ops.native_available()
    sa = torch.optim.lr_scheduler.StepLR(oa, 2, 0.5)
    sb = torch.optim.lr_scheduler.StepLR(ob, 2, 0.5)
    x = torch.randn(4, 16)
    for _ in range(4):
        for m, o, s in ((a, oa, sa), (b, ob, sb)):
            o.zero_grad()
            m(x).square().mean().backward()
            o.step()
            s.step()
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)
    assert ob.state_dict()["state"].keys() == oa.state_dict()["state"].keys()
