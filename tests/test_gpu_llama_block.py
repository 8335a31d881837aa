"""GPU: the fused Llama decoder block (one autograd node, csrc/kernels/autograd.hip LlamaBlockFn)
against the per-op path (NBD_FUSED_BLOCK=0 behaviour) — same kernels in the same order, so the
loss, logits and every parameter gradient must be bit-identical; plus DDP with the gradients in
their bucket slices (graddst) and the fp32 PyTorch reference of the whole model."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

from nbdistributed_amd import ops  # noqa: E402
from nbdistributed_amd.ops import gemm as G  # noqa: E402
from nbdistributed_amd.session import Session  # noqa: E402


@pytest.fixture(scope="module")
def dev(require_gpu):
    assert ops.native_available(), ops._load_error
    return torch.device("cuda")


def _run(model, ids, labels, fused: bool):
    prev = G.FUSED_BLOCK
    G.FUSED_BLOCK = fused
    try:
        for p in model.parameters():
            p.grad = None
        loss, logits = model(ids, torch.ones_like(ids), labels)
        loss.backward()
        torch.cuda.synchronize()
        return loss.detach(), logits.detach(), {n: p.grad.clone() for n, p in model.named_parameters()}
    finally:
        G.FUSED_BLOCK = prev


@pytest.mark.parametrize("qkv_bias", [False, True])
def test_fused_block_bit_identical_to_per_op_path(dev, qkv_bias):
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification

    torch.manual_seed(0)
    cfg = LlamaConfig.smollm2_135m(num_hidden_layers=3, qkv_bias=qkv_bias)
    m = LlamaForSequenceClassification(cfg).to(dev, torch.bfloat16)
    if qkv_bias:
        for layer in m.model.layers:
            torch.nn.init.normal_(layer.self_attn.qkv_proj.bias, std=0.02)
    ids = torch.randint(1, cfg.vocab_size, (4, 128), device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    labels = torch.tensor([0, 1, 1, 0], device=dev)
    lf, logf, gf = _run(m, ids, labels, True)
    lu, logu, gu = _run(m, ids, labels, False)
    assert torch.equal(lf, lu) and torch.equal(logf, logu)
    bad = [n for n in gu if not torch.equal(gf[n], gu[n])]
    assert not bad, bad


def test_fused_block_matches_fp32_reference(dev):
    """The fused bf16 model against the same weights in fp32 through plain PyTorch ops."""
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification

    torch.manual_seed(2)
    cfg = LlamaConfig.smollm2_135m(num_hidden_layers=2)
    m = LlamaForSequenceClassification(cfg).to(dev, torch.bfloat16)
    ref = copy.deepcopy(m).float()
    ids = torch.randint(1, cfg.vocab_size, (2, 128), device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    labels = torch.tensor([1, 0], device=dev)
    _, logits, _ = _run(m, ids, labels, True)
    prev = G.ENABLED  # fp32 weights take the PyTorch path of every op
    try:
        _, ref_logits = ref(ids, torch.ones_like(ids), labels)
    finally:
        G.ENABLED = prev
    err = (logits.float() - ref_logits).abs().max().item()
    assert err <= 0.05 * ref_logits.abs().max().item() + 0.02, err


CODE = """
import copy
from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.ops import gemm as G
torch.manual_seed(4)
base = LlamaForSequenceClassification(LlamaConfig.smollm2_135m(num_hidden_layers=2)).to(device, torch.bfloat16)
m = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket")
ids = torch.randint(1, 49152, (8, 128), generator=torch.Generator().manual_seed(0)).to(device)
lab = torch.zeros(8, dtype=torch.long, device=device)
out = []
for fused in (True, False):
    G.FUSED_BLOCK = fused
    for k in (1, 2):
        for p in m.parameters():
            p.grad = None
        for i in range(k):
            with (m.no_sync() if i < k - 1 else contextlib.nullcontext()):
                m(ids, torch.ones_like(ids), lab)[0].backward()
        torch.cuda.synchronize()
        out.append(torch.cat([b.buffer.float() for b in m.buckets]))
G.FUSED_BLOCK = True
(torch.equal(out[0], out[2]), torch.equal(out[1], out[3]), bool(out[0].abs().sum() > 0))
"""


@pytest.fixture(scope="module")
def sess(require_gpu):
    s = Session(writer=lambda t: None)
    s.start(1, startup_timeout=600, timeout=600)
    yield s
    s.shutdown()


def test_fused_block_ddp_buckets_bit_identical(sess):
    r = sess.execute("import contextlib\n" + CODE, render=False)
    assert r.ok, r.errors
    assert r.results[0]["echo"] == "(True, True, True)", r.results[0]


CODE_OVERLAP = """
import copy
from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
from nbdistributed_amd.graphs import GraphedStep
torch.manual_seed(6)
base = LlamaForSequenceClassification(LlamaConfig.smollm2_135m(num_hidden_layers=2)).to(device, torch.bfloat16)
ids = torch.randint(1, 49152, (8, 128), generator=torch.Generator().manual_seed(1)).to(device)
lab = torch.ones(8, dtype=torch.long, device=device)
res = []
for graphed in (False, True):
    outs = []
    for overlap in (False, True):
        m = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", bucket_cap_mb=4.0)
        o = FlatAdamW(m, lr=1e-3, capturable=graphed, overlap=overlap)
        def step(x, y):
            loss = m(x, torch.ones_like(x), y)[0]
            loss.backward()
            o.step()
            o.zero_grad()
            return loss.detach()
        call = GraphedStep(step, (ids, lab), warmup=2, optimizers=[o]) if graphed else step
        for _ in range(4):
            call(ids, lab)
        torch.cuda.synchronize()
        outs.append(torch.cat([b.param_flat.float() for b in m.buckets]))
        m.unpatch()
    res.append(torch.equal(outs[0], outs[1]))
tuple(res)
"""


def test_flat_adamw_overlap_matches_step(sess):
    """FlatAdamW(overlap=True) (buckets updated on a side stream during backward) leaves exactly
    the parameters of the update in step(), eager and as a HIP graph."""
    r = sess.execute(CODE_OVERLAP, render=False)
    assert r.ok, r.errors
    assert r.results[0]["echo"] == "(True, True)", r.results[0]
