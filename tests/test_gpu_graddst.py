"""Gradients written straight into their DDP bucket slices (ops.graddst, csrc/kernels/graddst.cpp):
the accumulating GEMM epilogue, the C++ Linear / MLP nodes, the LM head + tied embedding, and
DistributedDataParallel(grad_views=True) against the flatten path and torch DDP — each checked
against an fp32 (or flatten-path) reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from nbdistributed_amd import ops  # noqa: E402
from nbdistributed_amd.session import Session  # noqa: E402

EPI_NONE, EPI_ROWSUM = 0, 3


@pytest.fixture(scope="module")
def dev(require_gpu):
    assert ops.native_available(), ops._load_error
    return torch.device("cuda")


def _r(*s, g, scale=1.0):
    return (torch.randn(*s, device="cuda", generator=g) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("tile,splits", [(128128, 1), (64064, 1), (128128, 2), (3128128, 1), (80128128, 1)])
def test_gemm_accumulate_epilogue(dev, tile, splits):
    """c += dyᵀ·x (wgrad layout) and rowsum += Σ dy in the epilogue / split-K reduce."""
    g = torch.Generator(device="cuda").manual_seed(tile + splits)
    M, N, K = 256, 384, 512  # dW [M=out, N=in], K = tokens
    a = _r(K, M, g=g)
    b = _r(K, N, g=g)
    c0 = _r(M, N, g=g)
    rs0 = _r(M, g=g)
    c, rs = c0.clone(), rs0.clone()
    torch.ops.nbd.gemm(a, b, c, True, True, None, EPI_ROWSUM, None, rs, splits, tile, 3)
    ref = c0.float() + a.float().t() @ b.float()
    ref_rs = rs0.float() + a.float().sum(0)
    assert (c.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    assert (rs.float() - ref_rs).abs().max().item() < 2e-2 * ref_rs.abs().max().item()
    # accum=0 still overwrites
    c2 = c0.clone()
    torch.ops.nbd.gemm(a, b, c2, True, True, None, EPI_NONE, None, None, splits, tile, 0)
    assert (c2.float() - a.float().t() @ b.float()).abs().max().item() < 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("bias_grad", [False, True])
def test_gemm_pair_accumulate(dev, bias_grad):
    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, K = 512, 256, 384  # dy [M, N], W [N, K], x [M, K]
    dy, w, x = _r(M, N, g=g), _r(N, K, g=g), _r(M, K, g=g)
    dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    dw0, db0 = _r(N, K, g=g), _r(N, g=g)
    dw, db = dw0.clone(), db0.clone()
    torch.ops.nbd.gemm_pair(dy, w, dx, 0, None, dy, x, dw, EPI_ROWSUM if bias_grad else EPI_NONE,
                            db if bias_grad else None, 2, 1 | (2 if bias_grad else 0))
    ref = dw0.float() + dy.float().t() @ x.float()
    assert (dw.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    assert (dx.float() - dy.float() @ w.float()).abs().max().item() < 2e-2 * (dy.float() @ w.float()).abs().max().item()
    if bias_grad:
        rb = db0.float() + dy.float().sum(0)
        assert (db.float() - rb).abs().max().item() < 2e-2 * rb.abs().max().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_linear_node_writes_into_registered_destination(dev, dtype):
    """The C++ Linear node writes dW / db into the registered slice (``p.grad`` *is* the slice),
    bit-identical to its normal output, and accumulates there on a second backward."""
    from nbdistributed_amd.ops import gemm as G
    from nbdistributed_amd.ops import graddst

    torch.manual_seed(0)
    x = torch.randn(256, 512, device="cuda", dtype=dtype)
    lin = torch.nn.Linear(512, 384, device="cuda", dtype=dtype)
    dy = torch.randn(256, 384, device="cuda", dtype=dtype)
    # reference: no destination
    G.linear_any(x, lin.weight, lin.bias).backward(dy)
    gw, gb = lin.weight.grad.clone(), lin.bias.grad.clone()
    lin.weight.grad = lin.bias.grad = None
    home = torch.zeros(384 * 512 + 384 + 64, device="cuda", dtype=dtype)
    vw = home[:384 * 512].view(384, 512)
    vb = home[384 * 512 + 64:].view(384)
    graddst.register(lin.weight, vw)
    graddst.register(lin.bias, vb)
    try:
        graddst.new_pass()
        G.linear_any(x, lin.weight, lin.bias).backward(dy)
        assert lin.weight.grad.data_ptr() == vw.data_ptr() and lin.bias.grad.data_ptr() == vb.data_ptr()
        assert torch.equal(vw, gw) and torch.equal(vb, gb)
        graddst.new_pass()
        G.linear_any(x, lin.weight, lin.bias).backward(dy)  # accumulate: grad = g + g = 2g exactly
        assert lin.weight.grad.data_ptr() == vw.data_ptr()
        assert torch.equal(vw, 2 * gw) and torch.equal(vb, 2 * gb)
        # a parameter used twice in one pass: only the first writer takes the slice
        lin.weight.grad = lin.bias.grad = None
        graddst.new_pass()
        (G.linear_any(x, lin.weight, lin.bias) + G.linear_any(x, lin.weight, lin.bias)).backward(dy)
        tol = 0 if dtype == torch.float32 else 1e-2
        assert (lin.weight.grad.float() - 2 * gw.float()).abs().max().item() <= tol * gw.float().abs().max().item() + 1e-6
    finally:
        graddst.register(lin.weight, None)
        graddst.register(lin.bias, None)


CODE_DDP = """
import copy
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
torch.manual_seed(3)
cfg = GPT2Config(vocab_size=5000, n_positions=256, n_embd=256, n_layer=2, n_head=4)  # padded vocab 5120
base = GPT2(cfg).to(device, torch.bfloat16)
mv = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", bucket_cap_mb=1.0)
mf = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", bucket_cap_mb=1.0, grad_views=False)
idx = torch.randint(0, 5000, (2, 256), generator=torch.Generator().manual_seed(0)).to(device)
def grads(m, k=1):
    for i in range(k):
        ctx = m.no_sync() if i < k - 1 else contextlib.nullcontext()
        with ctx:
            m(idx, idx, return_logits=False)[1].backward()
    torch.cuda.synchronize()
    return torch.cat([b.buffer.float() for b in m.buckets])
import contextlib
a, b = grads(mv), grads(mf)
rel1 = float((a - b).abs().max() / b.abs().max())
a2, b2 = grads(mv, 3), grads(mf, 3)
rel3 = float((a2 - b2).abs().max() / b2.abs().max())
pad_zero = bool((mv.module.wte.weight[5000:] == 0).all())
(mv.stats["grad_views"] == len(list(mv.module.parameters())), rel1 < 2e-2, rel3 < 3e-2, pad_zero)
"""

CODE_DDP_LLAMA = """
import copy
import contextlib
from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification, LlamaForCausalLM
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
res = []
for cls in (LlamaForSequenceClassification, LlamaForCausalLM):
    torch.manual_seed(4)
    cfg = LlamaConfig(vocab_size=1000, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                      num_attention_heads=2, num_key_value_heads=1, tie_word_embeddings=cls is LlamaForCausalLM)
    base = cls(cfg).to(device, torch.bfloat16)
    mv = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", bucket_cap_mb=1.0)
    mf = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", bucket_cap_mb=1.0, grad_views=False)
    ids = torch.randint(1, 1000, (2, 128), generator=torch.Generator().manual_seed(1)).to(device)
    lab = torch.tensor([0, 1], device=device) if cls is LlamaForSequenceClassification else ids
    def grads(m, k=1):
        for i in range(k):
            ctx = m.no_sync() if i < k - 1 else contextlib.nullcontext()
            with ctx:
                m(ids, labels=lab).loss.backward()
        torch.cuda.synchronize()
        return torch.cat([b.buffer.float() for b in m.buckets])
    a, b = grads(mv), grads(mf)
    a3, b3 = grads(mv, 3), grads(mf, 3)
    res += [float((a - b).abs().max() / b.abs().max()) < 2e-2, float((a3 - b3).abs().max() / b3.abs().max()) < 3e-2]
tuple(res)
"""

CODE_LINEAR = """
import copy
import contextlib
from torch.nn.parallel import DistributedDataParallel as TorchDDP
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
torch.manual_seed(0)
lin = torch.nn.Linear(1024, 1024).to(device)
mt = TorchDDP(copy.deepcopy(lin), device_ids=[device.index])
mn = NbdDDP(copy.deepcopy(lin))
x = torch.randn(2048, 1024, device=device)
out = []
for k in (1, 2):
    for m in (mt, mn):
        for p in m.parameters():
            p.grad = None
        for i in range(k):
            ctx = m.no_sync() if i < k - 1 else contextlib.nullcontext()
            with ctx:
                m(x * (i + 1)).square().mean().backward()
    gt = [p.grad for p in mt.module.parameters()]
    gn = [p.grad for p in mn.module.parameters()]
    out.append(max(float((a - b).abs().max() / a.abs().max()) for a, b in zip(gt, gn)))
home = any(v.data_ptr() == mn.module.weight.grad.data_ptr() for bk in mn.buckets for v in (bk.views or []))
(mn.stats["fused_linears"], home, out[0] < 1e-5, out[1] < 1e-5)
"""


@pytest.fixture(scope="module")
def sess(require_gpu):
    s = Session(writer=lambda t: None)
    s.start(1, startup_timeout=600, timeout=600)
    yield s
    s.shutdown()


def test_ddp_gpt2_grad_views_match_flatten_path(sess):
    r = sess.execute(CODE_DDP, render=False)
    assert r.ok, r.errors
    assert r.results[0]["echo"] == "(True, True, True, True)", r.results[0]


def test_ddp_llama_embedding_grad_in_bucket_matches_flatten_path(sess):
    """Llama under nbd DDP with gradients as bucket views — the token embedding + first norm node
    (its table gradient written into the bucket slice) and the blocks — against the flatten path,
    untied (sequence classifier) and tied to the LM head, incl. no_sync accumulation."""
    r = sess.execute(CODE_DDP_LLAMA, render=False)
    assert r.ok, r.errors
    assert r.results[0]["echo"] == str((True,) * 4), r.results[0]


def test_ddp_fp32_linear_in_place_matches_torch_ddp(sess):
    r = sess.execute(CODE_LINEAR, render=False)
    assert r.ok, r.errors
    assert r.results[0]["echo"] == "(1, True, True, True)", r.results[0]


def test_deferred_splitk_reduce_matches_immediate(dev):
    """A split-K weight gradient written into its slice is queued (graddst.h ``defer``) and summed
    by one flush launch bit-identically to the immediate reduce — the flush registered with the
    running backward has run when ``backward()`` returns (no DDP here); a second use of the slice
    in the same pass flushes first."""
    from nbdistributed_amd.ops import gemm as G
    from nbdistributed_amd.ops import graddst

    torch.manual_seed(1)
    M, N, K = 2048, 576, 576  # SmolLM2 o_proj: the grouped backward splits the weight gradient
    assert G.pair_schedule(M, N, K, 64) & 15 > 1
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)  # the grouped launch
    lin = torch.nn.Linear(K, N, bias=False, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    home = torch.zeros(N * K, device="cuda", dtype=torch.bfloat16)
    vw = home.view(N, K)
    graddst.register(lin.weight, vw)
    try:
        ref = []
        for on in (False, True):
            graddst.defer_enable(on)
            lin.weight.grad = None
            home.fill_(7.0)  # stale contents must be overwritten
            graddst.new_pass()
            seen = []
            y = G.linear_any(x, lin.weight)
            # a hook on the input's gradient runs after the weight node, before backward() returns
            h = x.register_hook(lambda g: seen.append(graddst.defer_pending()))
            y.backward(dy)
            h.remove()
            assert lin.weight.grad.data_ptr() == vw.data_ptr()
            assert seen == [1 if on else 0] and graddst.defer_pending() == 0
            ref.append(vw.clone())
            # accumulate (grad already the slice): the queued reduce adds
            graddst.new_pass()
            G.linear_any(x, lin.weight).backward(dy)
            assert graddst.defer_pending() == 0
            ref.append(vw.clone())
        assert torch.equal(ref[0], ref[2]) and torch.equal(ref[1], ref[3])
        assert torch.equal(ref[1], 2 * ref[0])
        # used twice in one pass: the second claim flushes the first writer's reduce
        graddst.defer_enable(True)
        lin.weight.grad = None
        graddst.new_pass()
        (G.linear_any(x, lin.weight) + G.linear_any(x, lin.weight)).backward(dy)
        graddst.defer_flush()
        assert (lin.weight.grad.float() - 2 * ref[0].float()).abs().max().item() <= 1e-2 * ref[0].float().abs().max().item()
    finally:
        graddst.defer_enable(False)
        graddst.register(lin.weight, None)


CODE_DEFER = """
import copy
import contextlib
from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.ops import graddst
res = []
for kind in ("llama", "gpt2"):
    torch.manual_seed(5)
    if kind == "llama":
        base = LlamaForSequenceClassification(LlamaConfig.smollm2_135m(num_hidden_layers=2)).to(device, torch.bfloat16)
        ids = torch.randint(1, 49152, (16, 128), generator=torch.Generator().manual_seed(0)).to(device)
        fwd = lambda m: m(ids, torch.ones_like(ids), torch.zeros(16, dtype=torch.long, device=device))[0]
    else:
        base = GPT2(GPT2Config(vocab_size=5000, n_positions=256, n_embd=256, n_layer=2, n_head=4)).to(device, torch.bfloat16)
        ids = torch.randint(0, 5000, (4, 256), generator=torch.Generator().manual_seed(0)).to(device)
        fwd = lambda m: m(ids, ids, return_logits=False)[1]
    m = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket")
    out = []
    for on in (True, False):
        graddst.defer_enable(on)
        for k in (1, 3):
            for p in m.parameters():
                p.grad = None
            for i in range(k):
                ctx = m.no_sync() if i < k - 1 else contextlib.nullcontext()
                with ctx:
                    fwd(m).backward()
            torch.cuda.synchronize()
            out.append(torch.cat([b.buffer.float() for b in m.buckets]))
    graddst.defer_enable(True)
    res.append(torch.equal(out[0], out[2]) and torch.equal(out[1], out[3]) and graddst.defer_pending() == 0)
tuple(res)
"""


def test_ddp_deferred_reduces_bit_identical(sess):
    r = sess.execute(CODE_DEFER, render=False)
    assert r.ok, r.errors
    assert r.results[0]["echo"] == "(True, True)", r.results[0]
