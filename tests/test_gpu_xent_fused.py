"""GPU numerics: the one-pass LM-head loss (``nbd::xent_fused`` in csrc/kernels/xent.hip and
``ops.linear_cross_entropy``) against a plain fp32 PyTorch reference of the same bf16 inputs —
loss, and dh / dW through autograd; every register-chunk instance (8, 16, 25, 32), odd vocabularies
(unaligned rows: scalar head and tail lanes), ignore_index rows, sum reduction, grad_out ≠ 1."""
import pytest
import torch
import torch.nn.functional as F

from nbdistributed_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(require_gpu):
    assert ops.native_available(), ops._load_error
    return torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("V", [7, 1000, 2048, 4001, 32000, 50257, 65536])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_xent_fused_op_matches_reference(dev, V, dtype):
    torch.manual_seed(V)
    N = 96
    logits = (torch.randn(N, V, device=dev) * 3).to(dtype)
    tgt = torch.randint(0, V, (N,), device=dev)
    tgt[::7] = -100
    ref = logits.float().requires_grad_()
    loss_ref = F.cross_entropy(ref, tgt, ignore_index=-100, reduction="none")
    F.cross_entropy(ref, tgt, ignore_index=-100).backward()
    n_valid = (tgt != -100).sum().float()
    scale = (1.0 / n_valid).reshape(1)
    work = logits.clone()
    loss_rows, lse = torch.ops.nbd.xent_fused(work, tgt, -100, scale)
    torch.cuda.synchronize()
    assert _rel(loss_rows, loss_ref) < 1e-3
    assert _rel(lse, torch.logsumexp(logits.float(), -1)) < 1e-4
    assert _rel(work, ref.grad) < 2e-2          # the gradient, in place, in the logits' dtype
    assert bool((work[::7] == 0).all())         # ignored rows: zero gradient


@pytest.mark.parametrize("chunk", [0, 128, 200])
@pytest.mark.parametrize("reduction", ["mean", "sum"])
@pytest.mark.parametrize("V,C", [(50257, 768), (4000, 256)])
def test_linear_cross_entropy_autograd(dev, reduction, V, C, chunk, monkeypatch):
    """chunk > 0: the row-chunked head (GEMM -> in-place loss gradient -> input-gradient GEMM per
    chunk; 200 leaves a ragged last chunk)."""
    from nbdistributed_amd.ops import loss as L

    monkeypatch.setattr(L, "LM_HEAD_CHUNK", chunk)
    monkeypatch.setattr(L, "LM_HEAD_HIP", False)  # the library head (its row-chunked form included)
    torch.manual_seed(1)
    N = 512
    h = (torch.randn(N, C, device=dev) * 0.5).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(V, C, device=dev) * 0.05).to(torch.bfloat16).requires_grad_()
    tgt = torch.randint(0, V, (N,), device=dev)
    tgt[5] = -100
    loss = ops.linear_cross_entropy(h, w, tgt, reduction=reduction)
    (loss * 3.0).backward()                      # grad_out = 3 goes to the small operands only
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    lr = F.cross_entropy(hr @ wr.t(), tgt, ignore_index=-100, reduction=reduction)
    (lr * 3.0).backward()
    assert abs(float(loss) - float(lr)) < 2e-2 * max(1.0, abs(float(lr)))
    assert _rel(h.grad, hr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2


def test_gpt2_fused_head_matches_logits_path(dev):
    """GPT-2's return_logits=False path (fused head) = the return_logits=True path (logits, then
    the two-kernel loss) on the same bf16 model: loss and the tied embedding's gradient."""
    from nbdistributed_amd.models import GPT2, GPT2Config

    torch.manual_seed(2)
    cfg = GPT2Config(vocab_size=50257, n_positions=256, n_embd=256, n_layer=2, n_head=4)
    m = GPT2(cfg).to(dev, torch.bfloat16)
    idx = torch.randint(0, 50257, (2, 256), device=dev)
    _, l1 = m(idx, idx, return_logits=False)
    l1.backward()
    g1 = m.wte.weight.grad.clone()
    m.zero_grad(set_to_none=True)
    logits, l2 = m(idx, idx, return_logits=True)
    assert logits is not None
    l2.backward()
    assert abs(float(l1) - float(l2)) < 1e-2
    assert _rel(g1, m.wte.weight.grad) < 3e-2


@pytest.mark.parametrize("reduction", ["mean", "sum"])
# (38400, 512, 512): 300 weight-gradient tiles on 256 CUs — one whole round unsplit plus 44 tiles
# split 4 ways along the tokens, the second launch reading a column block of the logits
@pytest.mark.parametrize("V,C,N", [(50257, 768, 512), (5000, 256, 512), (4200, 256, 384), (38400, 512, 512)])
def test_linear_cross_entropy_hand_written_products(dev, reduction, V, C, N, monkeypatch):
    """NBD_LMHEAD_HIP: the head's forward, input- and weight-gradient products on the hand-written
    kernels (256x256 forward when tokens and padded vocabulary are multiples of 256 — 5000 -> 5120
    — else 128x128; split-K input gradient; 128x128 weight gradient) against fp32 torch
    F.linear + F.cross_entropy: loss, dh and dW."""
    from nbdistributed_amd.ops import loss as L

    monkeypatch.setattr(L, "LM_HEAD_HIP", True)
    monkeypatch.setattr(L, "HEAD_PRODUCTS", {"fwd": True, "dgrad": True, "wgrad": True})
    torch.manual_seed(3)
    h = (torch.randn(N, C, device=dev) * 0.5).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(V, C, device=dev) * 0.05).to(torch.bfloat16).requires_grad_()
    tgt = torch.randint(0, V, (N,), device=dev)
    tgt[3] = -100
    loss = ops.linear_cross_entropy(h, w, tgt, reduction=reduction)
    (loss * 2.0).backward()
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    lr = F.cross_entropy(F.linear(hr, wr), tgt, ignore_index=-100, reduction=reduction)
    (lr * 2.0).backward()
    assert abs(float(loss) - float(lr)) < 2e-2 * max(1.0, abs(float(lr)))
    assert _rel(h.grad, hr.grad) < 3e-2
    assert _rel(w.grad, wr.grad) < 3e-2


def test_hand_written_head_runs_no_library_gemm(dev, monkeypatch):
    """With NBD_LMHEAD_HIP=1 the head issues only nbd kernels: torch.mm is never called."""
    from nbdistributed_amd.ops import loss as L

    monkeypatch.setattr(L, "LM_HEAD_HIP", True)
    monkeypatch.setattr(L, "HEAD_PRODUCTS", {"fwd": True, "dgrad": True, "wgrad": True})
    calls = []
    real_mm = torch.mm

    def spy(*a, **k):
        calls.append(a[0].shape)
        return real_mm(*a, **k)

    monkeypatch.setattr(torch, "mm", spy)
    h = torch.randn(256, 256, device=dev).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(4096, 256, device=dev) * 0.05).to(torch.bfloat16).requires_grad_()
    tgt = torch.randint(0, 4096, (256,), device=dev)
    ops.linear_cross_entropy(h, w, tgt).backward()
    torch.cuda.synchronize()
    assert calls == []
    assert h.grad is not None and w.grad is not None


@pytest.mark.parametrize("products", [{"fwd": False, "dgrad": True, "wgrad": False},
                                      {"fwd": True, "dgrad": False, "wgrad": True}])
def test_linear_cross_entropy_mixed_products(dev, products, monkeypatch):
    """The head's products chosen one by one (the default "auto" plan: the input gradient
    hand-written, forward and weight gradient on the library) give the same loss / gradients as
    fp32 torch, and the library is called for exactly the library products."""
    from nbdistributed_amd.ops import loss as L

    monkeypatch.setattr(L, "LM_HEAD_HIP", True)
    monkeypatch.setattr(L, "HEAD_PRODUCTS", products)
    calls = []
    real_mm = torch.mm
    monkeypatch.setattr(torch, "mm", lambda *a, **k: calls.append(1) or real_mm(*a, **k))
    torch.manual_seed(5)
    V, C, N = 50257, 768, 512
    h = (torch.randn(N, C, device=dev) * 0.5).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(V, C, device=dev) * 0.05).to(torch.bfloat16).requires_grad_()
    tgt = torch.randint(0, V, (N,), device=dev)
    loss = ops.linear_cross_entropy(h, w, tgt)
    loss.backward()
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    F.cross_entropy(F.linear(hr, wr), tgt).backward()
    assert _rel(h.grad, hr.grad) < 3e-2 and _rel(w.grad, wr.grad) < 3e-2
    assert len(calls) == sum(not v for v in products.values())


@pytest.mark.parametrize("n", [1, 96, 8192, 70001])
def test_loss_scalar_ops(dev, n):
    """xent_mean_scale / xent_loss_total (the mean reduction's two one-launch scalars) and
    scale_pair_ (the backward's dh *= g, h·g) against fp32 PyTorch."""
    torch.manual_seed(n)
    tgt = torch.randint(0, 50, (n,), device=dev)
    tgt[::3] = -100
    valid = int((tgt != -100).sum())
    s = torch.ops.nbd.xent_mean_scale(tgt, -100)
    assert s.shape == (1,) and s.dtype == torch.float32
    assert (float(s) == float("inf")) if valid == 0 else abs(float(s) * valid - 1.0) < 1e-6  # fp32 reciprocal
    rows = torch.randn(n, device=dev)
    tot = torch.ops.nbd.xent_loss_total(rows, s if valid else torch.ones(1, device=dev))
    ref = rows.double().sum() * (float(s) if valid else 1.0)
    assert tot.dim() == 0 and abs(float(tot) - float(ref)) <= 1e-5 * max(1.0, abs(float(ref)))
    a = torch.randn(n * 8, device=dev).to(torch.bfloat16)
    b = torch.randn(n * 8, device=dev).to(torch.bfloat16)
    g = torch.tensor([0.37], device=dev)
    a_ref, b_ref = (a.float() * 0.37).to(torch.bfloat16), (b.float() * 0.37).to(torch.bfloat16)
    out = torch.ops.nbd.scale_pair_(a, b, g)
    assert torch.equal(a, a_ref) and torch.equal(out, b_ref)


def test_mean_scale_all_ignored(dev):
    tgt = torch.full((64,), -100, device=dev)
    assert float(torch.ops.nbd.xent_mean_scale(tgt, -100)) == float("inf")
