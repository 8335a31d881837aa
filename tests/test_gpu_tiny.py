"""GPU: the tiny-linear kernels (``csrc/kernels/tiny.hip``, classifier heads such as SmolLM2's
``score``) against an fp32 PyTorch reference of the same Linear: output, input / weight / bias
gradients; and the sequence classifier's head runs on them (no library GEMM)."""
import pytest
import torch

from nbdistributed_amd import ops

pytestmark = pytest.mark.gpu


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
    """The sequence classifier's score head calls nbd.linear_tiny on the GPU (never F.linear /
    a library GEMM), and its logits and gradient match the module path."""
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification

    torch.manual_seed(0)
    m = LlamaForSequenceClassification(LlamaConfig.tiny()).cuda().to(torch.bfloat16)
    calls = []
    real = torch.ops.nbd.linear_tiny
    monkeypatch.setattr(torch.ops.nbd, "linear_tiny", lambda *a: calls.append(1) or real(*a), raising=False)
    ids = torch.randint(1, 100, (4, 128), device="cuda")
    mask = torch.ones_like(ids)
    out = m(input_ids=ids, attention_mask=mask, labels=torch.tensor([0, 1, 1, 0], device="cuda"))
    out.loss.backward()
    assert calls, "the score head did not run on the tiny-linear kernel"
    assert m.score.weight.grad is not None and torch.isfinite(m.score.weight.grad.float()).all()
