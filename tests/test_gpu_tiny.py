"""GPU: the tiny-linear kernels (``csrc/kernels/tiny.hip``, classifier heads such as SmolLM2's
``score``) against an fp32 PyTorch reference of the same Linear: output, input / weight / bias
gradients; and the sequence classifier's head runs on them (no library GEMM)."""
import pytest
import torch
import torch.nn.functional as F

from nbdistributed_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture
def dev(require_gpu):
    return torch.device("cuda", 0)


def _rel(a, r):
    a, r = a.detach().float(), r.detach().float()
    return float((a - r).abs().max() / r.abs().max().clamp_min(1e-6))


@pytest.mark.parametrize("M,N,K,bias", [(16, 2, 576, False), (16, 2, 576, True), (1, 1, 8, True), (33, 7, 200, True),
                                        (300, 64, 1024, False), (4096, 3, 576, True)])
def test_linear_tiny_matches_fp32(require_gpu, M, N, K, bias):
    torch.manual_seed(M * 131 + N * 7 + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_()
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_() if bias else None
    assert ops.tiny.supported(x, w, b)
    y = ops.linear_tiny(x, w, b)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    y.backward(dy)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    bf = b.detach().float().requires_grad_() if bias else None
    yf = torch.nn.functional.linear(xf, wf, bf)
    yf.backward(dy.float())

    def rel(a, r):
        return float((a.float() - r).abs().max() / r.abs().max().clamp_min(1e-6))

    assert y.dtype == torch.bfloat16 and rel(y, yf) < 1e-2
    assert rel(x.grad, xf.grad) < 1e-2 and rel(w.grad, wf.grad) < 1e-2
    if bias:
        assert rel(b.grad, bf.grad) < 1e-2


def test_seqcls_head_uses_tiny_kernels(require_gpu, monkeypatch):
    """Without labels the sequence classifier's score head calls nbd.linear_tiny on the GPU (never
    F.linear / a library GEMM)."""
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification

    torch.manual_seed(0)
    m = LlamaForSequenceClassification(LlamaConfig.tiny()).cuda().to(torch.bfloat16)
    calls = []
    real = torch.ops.nbd.linear_tiny
    monkeypatch.setattr(torch.ops.nbd, "linear_tiny", lambda *a: calls.append(1) or real(*a), raising=False)
    ids = torch.randint(1, 100, (4, 128), device="cuda")
    mask = torch.ones_like(ids)
    out = m(input_ids=ids, attention_mask=mask)  # (with labels the fused tail runs: below)
    F.cross_entropy(out.logits.float(), torch.tensor([0, 1, 1, 0], device="cuda")).backward()
    assert calls, "the score head did not run on the tiny-linear kernel"
    assert m.score.weight.grad is not None and torch.isfinite(m.score.weight.grad.float()).all()


@pytest.mark.parametrize("B,T,C,N", [(16, 128, 576, 2), (3, 40, 64, 5), (64, 16, 256, 16)])
def test_seqcls_head_loss_matches_reference(dev, B, T, C, N):
    """The fused classifier tail (pooled gather -> score -> mean cross-entropy) against fp32
    PyTorch: loss, logits, dh (zero except the pooled rows) and dW, with an ignored label and a
    gradient arriving at the logits too."""
    from nbdistributed_amd.ops import tiny

    g = torch.Generator(device="cpu").manual_seed(B * 1000 + N)
    h = torch.randn(B, T, C, generator=g).to(dev, torch.bfloat16).requires_grad_()
    w = (torch.randn(N, C, generator=g) * 0.05).to(dev, torch.bfloat16).requires_grad_()
    last = torch.randint(0, T, (B,), generator=g).to(dev)
    labels = torch.randint(0, N, (B,), generator=g).to(dev)
    labels[1] = -100
    assert tiny.seqcls_ok(h, w, labels)
    loss, logits = tiny.seqcls_head_loss(h, last, w, labels)
    glog = torch.randn(B, N, generator=g).to(dev, torch.bfloat16)
    (2.5 * loss + (logits.float() * glog.float()).sum()).backward()
    hr, wr = h.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    pooled = hr[torch.arange(B, device=dev), last]
    lr = (pooled @ wr.t())
    ref_logits = lr.to(torch.bfloat16)
    assert torch.equal(logits, ref_logits) or _rel(logits, lr) < 1e-2
    loss_r = F.cross_entropy(ref_logits.float(), labels, ignore_index=-100)
    assert abs(float(loss) - float(loss_r)) < 1e-4 * max(1.0, abs(float(loss_r)))
    # gradient reference through the fp32 logits (the kernel differentiates its rounded logits)
    lr2 = pooled @ wr.t()
    (2.5 * F.cross_entropy(lr2, labels, ignore_index=-100) + (lr2 * glog.float()).sum()).backward()
    assert _rel(h.grad, hr.grad) < 3e-2 and _rel(w.grad, wr.grad) < 3e-2
    mask = torch.ones(B, T, dtype=torch.bool, device=dev)
    mask[torch.arange(B, device=dev), last] = False
    assert float(h.grad[mask].float().abs().max()) == 0.0


def test_llama_seqcls_uses_fused_tail(dev, monkeypatch):
    """LlamaForSequenceClassification with labels runs the fused tail (no torch cross-entropy)."""
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification
    from nbdistributed_amd.ops import tiny

    calls = []
    real = tiny.seqcls_head_loss
    monkeypatch.setattr(tiny, "seqcls_head_loss", lambda *a, **k: calls.append(1) or real(*a, **k))
    torch.manual_seed(0)
    c = LlamaConfig.smollm2_135m(num_hidden_layers=2, hidden_size=64, intermediate_size=128, num_attention_heads=4,
                                 num_key_value_heads=2, vocab_size=512)
    m = LlamaForSequenceClassification(c).to(dev, torch.bfloat16)
    ids = torch.randint(1, 512, (4, 128), device=dev)
    mask = torch.ones_like(ids)
    y = torch.randint(0, 2, (4,), device=dev)
    out = m(ids, mask, y)
    out[0].backward()
    assert calls and torch.isfinite(out[0]) and m.score.weight.grad is not None
    with torch.no_grad():
        ref = F.cross_entropy(out[1].float(), y)
    assert abs(float(out[0]) - float(ref)) < 1e-4
