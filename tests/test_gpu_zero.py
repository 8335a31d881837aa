"""ZeRO-2 on one MI355X over RCCL (world 1): the reduce-scatter / all-gather path inside a
captured HIP graph (GraphedStep) replays like the eager unsharded step."""
import pytest

from nbdistributed_amd.session import Session

pytestmark = pytest.mark.gpu

CODE = """
import copy
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
from nbdistributed_amd.graphs import GraphedStep
torch.manual_seed(3)
cfg = GPT2Config(vocab_size=2048, n_positions=256, n_embd=256, n_layer=2, n_head=4)
base = GPT2(cfg).to(device, torch.bfloat16)
mf = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", bucket_cap_mb=1.0)
mz = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", bucket_cap_mb=1.0, shard=True)
of, oz = FlatAdamW(mf, lr=1e-3), FlatAdamW(mz, lr=1e-3, capturable=True)
idx = torch.randint(0, 2048, (2, 256), generator=torch.Generator().manual_seed(0)).to(device)
def step_z(x):
    loss = mz(x, x, return_logits=False)[1]
    loss.backward()
    oz.step()
    oz.zero_grad()
    return loss.detach()
g = GraphedStep(step_z, (idx,), warmup=2, optimizers=[oz])
lf = []
for _ in range(2 + 3):   # the sharded one: 2 eager warm-up steps, the capture (records, runs nothing), 3 replays
    loss = mf(idx, idx, return_logits=False)[1]; loss.backward(); of.step(); of.zero_grad()
    lf.append(float(loss.detach()))
lz = [float(g(idx)) for _ in range(3)]
mz.wait_params(); torch.cuda.synchronize()
err = max(float((p.float() - q.float()).abs().max()) for p, q in zip(mf.module.parameters(), mz.module.parameters()))
(dist.get_backend(), err < 1e-2, all(abs(a - b) < 1e-2 for a, b in zip(lf[2:], lz)))
"""


@pytest.fixture(scope="module")
def sess(require_gpu):
    s = Session(writer=lambda t: None)
    s.start(1, startup_timeout=600, timeout=600)
    yield s
    s.shutdown()


def test_zero2_graphed_step_on_rccl(sess):
    r = sess.execute(CODE, render=False)
    assert r.ok, r.errors
    assert r.results[0]["echo"] == "('rccl', True, True)", r.results[0]
