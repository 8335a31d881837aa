"""GPU numerics: HIP flash attention (csrc/kernels/attn.hip) against a plain fp32 PyTorch
reference of the same bf16 inputs — forward output, and dq/dk/dv through autograd."""
import pytest
import torch

from nbdistributed_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(require_gpu):
    assert ops.native_available(), ops._load_error
    return torch.device("cuda", 0)


def ref_attn(q, k, v, causal, scale):
    q, k, v = q.float(), k.float(), v.float()
    s = (q @ k.transpose(-1, -2)) * scale
    if causal:
        T = q.shape[-2]
        s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return torch.softmax(s, -1) @ v


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("B,H,T", [(1, 1, 128), (2, 3, 256), (1, 2, 384), (1, 2, 640), (2, 2, 1024)])
def test_flash_forward_backward(dev, causal, B, H, T):
    """T >= 256 causal: the forward's heavier query blocks run split along the keys
    (fwd_split_kernel, merged through LDS); odd block counts (384, 640) leave an uneven split."""
    g = torch.Generator(device="cpu").manual_seed(T + H)
    q, k, v, do = (torch.randn(B, H, T, 64, generator=g).to(dev, torch.bfloat16) for _ in range(4))
    scale = 0.125
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = ref_attn(qr, kr, vr, causal, scale)
    ref.backward(do.float())
    qh, kh, vh = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    out = ops.flash_attention(qh, kh, vh, causal=causal, scale=scale)
    out.backward(do)
    torch.cuda.synchronize()
    assert out.shape == (B, H, T, 64) and out.dtype == torch.bfloat16
    assert _rel(out, ref) < 2e-2, _rel(out, ref)
    for name, a, b in (("dq", qh.grad, qr.grad), ("dk", kh.grad, kr.grad), ("dv", vh.grad, vr.grad)):
        assert _rel(a, b) < 3e-2, (name, _rel(a, b))


_GQA_CASES = [(2, 9, 3, 128), (4, 8, 2, 256), (1, 6, 1, 384), (16, 9, 3, 128), (64, 9, 3, 128), (4, 9, 3, 256),
              (3, 9, 3, 384)]


def _gqa_case(dev, B, H, Hkv, T, causal):
    g = torch.Generator(device="cpu").manual_seed(B * 100 + H * 10 + Hkv + T)
    q, do = (torch.randn(B, H, T, 64, generator=g).to(dev, torch.bfloat16) for _ in range(2))
    k, v = (torch.randn(B, Hkv, T, 64, generator=g).to(dev, torch.bfloat16) for _ in range(2))
    qh, kh, vh = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    out = ops.flash_attention(qh, kh, vh, causal=causal, scale=0.125)
    out.backward(do)
    torch.cuda.synchronize()
    return (q, k, v, do), (out, qh.grad, kh.grad, vh.grad)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("B,H,Hkv,T", _GQA_CASES)
def test_flash_gqa_backward(dev, causal, B, H, Hkv, T):
    """Grouped-query backward, incl. the query-head groups split over workgroups and summed by
    gqa_reduce_kernel (B·Hkv·T/128 < 128 — fused δ at T ≤ 256, the δ pre-pass at 384), and one
    workgroup per key/value head sweeping its group (B64: 192), against fp32 attention on repeated
    K/V."""
    (q, k, v, do), (out, dq, dk, dv) = _gqa_case(dev, B, H, Hkv, T, causal)
    rep = H // Hkv
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = ref_attn(qr, kr.repeat_interleave(rep, 1), vr.repeat_interleave(rep, 1), causal, 0.125)
    ref.backward(do.float())
    assert _rel(out, ref) < 2e-2
    for name, a, b in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        assert _rel(a, b) < 3e-2, (name, _rel(a, b))


@pytest.mark.parametrize("causal", [True, False])
def test_flash_deferred_rescale_branch(dev, causal):
    """Scores that grow along the keys, by a different rate per query: some waves rescale O at
    every 64-key tile (growth > 2^4 per tile), others keep a stale running max for several tiles
    (the forward's deferred-rescale branch is data-dependent: random data rarely takes it)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    B, H, T = 1, 2, 512
    u = torch.nn.functional.normalize(torch.randn(64, generator=g), dim=0)
    a_q = torch.linspace(0.0, 4.0, T).repeat(B, H, 1)[..., None]  # per-query alignment
    q = 0.3 * torch.randn(B, H, T, 64, generator=g) + a_q * u
    k = 0.3 * torch.randn(B, H, T, 64, generator=g) + (0.1 * torch.arange(T, dtype=torch.float32))[:, None] * u
    v, do = (torch.randn(B, H, T, 64, generator=g) for _ in range(2))
    q, k, v, do = (t.to(dev, torch.bfloat16) for t in (q, k, v, do))
    scale = 0.125
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = ref_attn(qr, kr, vr, causal, scale)
    ref.backward(do.float())
    qh, kh, vh = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    out = ops.flash_attention(qh, kh, vh, causal=causal, scale=scale)
    out.backward(do)
    torch.cuda.synchronize()
    assert _rel(out, ref) < 2e-2, _rel(out, ref)
    _, lse = torch.ops.nbd.attn_fwd(q, k, v, causal, scale)
    s = (q.float() @ k.float().transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=dev).triu(1), float("-inf"))
    assert torch.allclose(lse, torch.logsumexp(s, -1), atol=2e-3, rtol=1e-4)
    # dq = scale·Σ dS·k with keys of magnitude ~50 here: dS rounded to bf16 for the MFMA does not
    # cancel the keys' common component exactly (Σ dS = 0), so dq gets a looser bound than dk/dv
    for name, a, b, tol in (("dq", qh.grad, qr.grad, 8e-2), ("dk", kh.grad, kr.grad, 3e-2),
                            ("dv", vh.grad, vr.grad, 3e-2)):
        assert _rel(a, b) < tol, (name, _rel(a, b))


def test_flash_lse_matches_reference(dev):
    q, k, v = (torch.randn(2, 2, 256, 64, device=dev).to(torch.bfloat16) for _ in range(3))
    o, lse = torch.ops.nbd.attn_fwd(q, k, v, True, 0.125)
    s = (q.float() @ k.float().transpose(-1, -2)) * 0.125
    s = s.masked_fill(torch.ones(256, 256, dtype=torch.bool, device=dev).triu(1), float("-inf"))
    assert torch.allclose(lse, torch.logsumexp(s, -1), atol=2e-3, rtol=1e-4)


def test_attention_qkv_packed_matches_sdpa_path(dev):
    """GPT-2 layout: packed c_attn output [B, T, 3C] in, [B, T, C] out, packed dqkv back."""
    B, T, H = 2, 256, 4
    C = H * 64
    g = torch.Generator(device="cpu").manual_seed(5)
    qkv = torch.randn(B, T, 3 * C, generator=g).to(dev, torch.bfloat16)
    dy = torch.randn(B, T, C, generator=g).to(dev, torch.bfloat16)
    a = qkv.detach().clone().requires_grad_(True)
    y = ops.attention_qkv(a, H, causal=True)
    y.backward(dy)
    r = qkv.detach().float().requires_grad_(True)
    q, k, v = (r[:, :, i * C:(i + 1) * C].view(B, T, H, 64).transpose(1, 2) for i in range(3))
    yr = ref_attn(q, k, v, True, 0.125).transpose(1, 2).reshape(B, T, C)
    yr.backward(dy.float())
    torch.cuda.synchronize()
    assert _rel(y, yr) < 2e-2
    assert _rel(a.grad, r.grad) < 3e-2
    assert a.grad.is_contiguous() and a.grad.shape == qkv.shape


def test_gpt2_small_step_fused_matches_sdpa(dev):
    from nbdistributed_amd.models import GPT2, GPT2Config

    torch.manual_seed(0)
    cfg = GPT2Config(n_layer=2)
    m1 = GPT2(cfg).to(dev, torch.bfloat16)
    cfg2 = GPT2Config(n_layer=2, fused_attn=False)
    m2 = GPT2(cfg2).to(dev, torch.bfloat16)
    m2.load_state_dict(m1.state_dict())
    idx = torch.randint(0, 50257, (2, 256), device=dev)
    l1 = m1(idx, idx, return_logits=False)[1]
    l2 = m2(idx, idx, return_logits=False)[1]
    l1.backward()
    l2.backward()
    torch.cuda.synchronize()
    assert abs(float(l1.detach()) - float(l2.detach())) < 2e-2
    g1 = m1.h[0].attn.c_attn.weight.grad
    g2 = m2.h[0].attn.c_attn.weight.grad
    assert _rel(g1, g2) < 5e-2


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("H,Hkv", [(4, 4), (4, 2)])
def test_ring_attention_zigzag_single_rank_hip_blocks(dev, causal, H, Hkv):
    """parallel.context on one rank with the zigzag layout: two 128-token HIP flash blocks per
    query chunk merged through their log-sum-exps, and the backward given the merged output/LSE —
    vs the fp32 reference on the whole sequence."""
    from nbdistributed_amd.parallel.context import ring_attention

    g = torch.Generator(device="cpu").manual_seed(H * 7 + Hkv)
    B, T = 2, 256
    q, do = (torch.randn(B, H, T, 64, generator=g).to(dev, torch.bfloat16) for _ in range(2))
    k, v = (torch.randn(B, Hkv, T, 64, generator=g).to(dev, torch.bfloat16) for _ in range(2))
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    rep = H // Hkv
    ref = ref_attn(qr, kr.repeat_interleave(rep, 1), vr.repeat_interleave(rep, 1), causal, 0.125)
    ref.backward(do.float())
    qh, kh, vh = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    out = ring_attention(qh, kh, vh, causal=causal, scale=0.125, layout="zigzag")
    out.backward(do)
    assert _rel(out, ref) < 2e-2
    assert _rel(qh.grad, qr.grad) < 3e-2
    assert _rel(kh.grad, kr.grad) < 3e-2
    assert _rel(vh.grad, vr.grad) < 3e-2


@pytest.mark.parametrize("last", [False, True])
def test_attn_merge_kernel(dev, last):
    """nbd::attn_merge_ (csrc/kernels/ring.hip) vs the fp32 log-sum-exp merge, on a strided bf16
    block (the [B, T, H, D]-stored output of attn_fwd)."""
    g = torch.Generator(device="cpu").manual_seed(5)
    B, H, T = 2, 3, 256
    acc = torch.randn(B, H, T, 64, generator=g).to(dev)
    la = (torch.randn(B, H, T, generator=g) * 3).to(dev)
    ob = torch.randn(B, T, H, 64, generator=g).to(dev, torch.bfloat16).transpose(1, 2)
    lb = (torch.randn(B, H, T, generator=g) * 3).to(dev)
    l_ref = torch.logaddexp(la, lb)
    o_ref = acc * torch.exp(la - l_ref).unsqueeze(-1) + ob.float() * torch.exp(lb - l_ref).unsqueeze(-1)
    out = torch.empty(B, H, T, 64, device=dev, dtype=torch.bfloat16) if last else None
    acc0 = acc.clone()
    torch.ops.nbd.attn_merge_(acc, la, ob, lb, out)
    assert (la - l_ref).abs().max().item() < 1e-4
    if last:
        assert _rel(out, o_ref) < 1e-2
        assert torch.equal(acc, acc0)
    else:
        assert _rel(acc, o_ref) < 1e-5


def test_gqa_split_sum_repeatable(dev):
    """The query-head split of the GQA backward (partials summed by gqa_reduce_kernel in a fixed
    order): bit-identical over repeated calls, and equal to fp32 attention on repeated K/V."""
    g = torch.Generator(device="cpu").manual_seed(11)
    B, H, Hkv, T = 16, 9, 3, 128
    q, do = (torch.randn(B, H, T, 64, generator=g).to(dev, torch.bfloat16) for _ in range(2))
    k, v = (torch.randn(B, Hkv, T, 64, generator=g).to(dev, torch.bfloat16) for _ in range(2))
    o, lse = torch.ops.nbd.attn_fwd(q, k, v, True, 0.125, None, None)
    outs = []
    for _ in range(3):
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        torch.ops.nbd.attn_bwd(do, q, k, v, o, lse, True, 0.125, dq, dk, dv, None, None)
        torch.cuda.synchronize()
        outs.append((dq, dk, dv))
    for a in outs[1:]:
        assert all(torch.equal(x, y) for x, y in zip(outs[0], a))
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = ref_attn(qr, kr.repeat_interleave(H // Hkv, 1), vr.repeat_interleave(H // Hkv, 1), True, 0.125)
    ref.backward(do.float())
    for name, a, b in (("dq", outs[0][0], qr.grad), ("dk", outs[0][1], kr.grad), ("dv", outs[0][2], vr.grad)):
        assert _rel(a, b) < 3e-2, (name, _rel(a, b))


@pytest.mark.parametrize("T", [512, 1024])
def test_attention_out_projection_delta_epilogue(dev, T):
    """GPT-2's attention -> c_proj on the native nodes: at T > 256 the projection's grouped
    backward launch computes the flash backward's δ in its epilogue (gemm.hip EPI_ADELTA, no
    pre-pass); q|k|v, weight and bias gradients against fp32 SDPA + Linear."""
    import torch.nn.functional as F

    B, H, D = 2, 4, 64
    C = H * D
    g = torch.Generator(device="cpu").manual_seed(T)
    qkv = (torch.randn(B, T, 3 * C, generator=g) * 0.5).to(dev, torch.bfloat16).requires_grad_()
    w = (torch.randn(C, C, generator=g) * 0.05).to(dev, torch.bfloat16).requires_grad_()
    b = (torch.randn(C, generator=g) * 0.1).to(dev, torch.bfloat16).requires_grad_()
    dy = torch.randn(B, T, C, generator=g).to(dev, torch.bfloat16)
    y = ops.gemm_linear(ops.attention_qkv(qkv, H, causal=True), w, b)
    y.backward(dy)
    qr, wr, br = (t.detach().float().requires_grad_() for t in (qkv, w, b))
    q, k, v = (t.view(B, T, H, D).transpose(1, 2) for t in qr.split(C, dim=-1))
    a = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, C)
    yr = F.linear(a, wr, br)
    yr.backward(dy.float())
    torch.cuda.synchronize()
    assert _rel(y, yr) < 2e-2
    for name, x, r in (("dqkv", qkv.grad, qr.grad), ("dW", w.grad, wr.grad), ("db", b.grad, br.grad)):
        assert _rel(x, r) < 3e-2, (name, _rel(x, r))
