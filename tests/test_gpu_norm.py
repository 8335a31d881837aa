"""GPU numerics: HIP LayerNorm (+ fused residual add), column sums and the bias-grad Linear
(csrc/kernels/norm.hip) against plain fp32 PyTorch references."""
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


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("C", [8, 64, 256, 512, 768, 1000, 1536, 2048])  # 256·k: the 16-B half-wave backward
@pytest.mark.parametrize("res", [False, True])
def test_layer_norm_fwd_bwd(dev, dt, C, res):
    g = torch.Generator(device="cpu").manual_seed(C)
    rows = 333
    x = (torch.randn(rows, C, generator=g) * 2 + 0.5).to(dev, dt)
    d = torch.randn(rows, C, generator=g).to(dev, dt)
    w = (1 + 0.1 * torch.randn(C, generator=g)).to(dev, dt)
    b = (0.1 * torch.randn(C, generator=g)).to(dev, dt)
    dy = torch.randn(rows, C, generator=g).to(dev, dt)
    ds = torch.randn(rows, C, generator=g).to(dev, dt)
    xs, ds_, ws, bs = (t.detach().clone().requires_grad_(True) for t in (x, d, w, b))
    xr, dr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, d, w, b))
    if res:
        s, y = ops.add_layer_norm(xs, ds_, ws, bs)
        (y.float() * dy.float()).sum().add_((s.float() * ds.float()).sum()).backward()
        sr = (xr + dr).to(dt).float()  # the kernel normalises the stored (rounded) sum
        sr = xr + dr + (sr - (xr + dr)).detach()
        yr = F.layer_norm(sr, (C,), wr, br, 1e-5)
        ((yr * dy.float()).sum() + (sr * ds.float()).sum()).backward()
        assert _rel(s, sr) < 1e-2
    else:
        y = ops.layer_norm(xs, ws, bs)
        (y.float() * dy.float()).sum().backward()
        yr = F.layer_norm(xr, (C,), wr, br, 1e-5)
        (yr * dy.float()).sum().backward()
    torch.cuda.synchronize()
    tol = {torch.bfloat16: 2e-2, torch.float16: 4e-3}.get(dt, 1e-4)
    assert _rel(y, yr) < tol
    assert _rel(xs.grad, xr.grad) < 2 * tol, _rel(xs.grad, xr.grad)
    assert _rel(ws.grad, wr.grad) < 2 * tol and _rel(bs.grad, br.grad) < 2 * tol
    if res:
        assert _rel(ds_.grad, dr.grad) < 2 * tol


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,C", [(1, 8), (67, 768), (8192, 2304), (100, 3072)])
def test_colsum(dev, dt, rows, C):
    x = torch.randn(rows, C, device=dev).to(dt)
    got = ops.colsum(x, torch.float32)
    assert torch.allclose(got, x.float().sum(0), atol=1e-3 * max(1.0, rows ** 0.5), rtol=1e-4)


def test_linear_bias_grad(dev):
    x = torch.randn(4, 128, 768, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(3072, 768, device=dev, dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(3072, device=dev, dtype=torch.bfloat16, requires_grad=True)
    dy = torch.randn(4, 128, 3072, device=dev, dtype=torch.bfloat16)
    ops.linear(x, w, b).backward(dy)
    g1 = [t.grad.clone() for t in (x, w, b)]
    for t in (x, w, b):
        t.grad = None
    F.linear(x, w, b).backward(dy)
    for a, r in zip(g1, (x.grad, w.grad, b.grad)):
        assert _rel(a, r) < 1e-2


def test_gpt2_fused_path_matches_reference(dev):
    from nbdistributed_amd.models import GPT2, GPT2Config

    torch.manual_seed(0)
    m1 = GPT2(GPT2Config(n_layer=2)).to(dev, torch.bfloat16)
    m2 = GPT2(GPT2Config(n_layer=2, fused_norm=False, fused_attn=False, fused_ce=False)).to(dev, torch.bfloat16)
    m2.load_state_dict(m1.state_dict())
    idx = torch.randint(0, 50257, (2, 256), device=dev)
    l1 = m1(idx, idx, return_logits=False)[1]
    l2 = m2(idx, idx)[1]
    l1.backward()
    l2.backward()
    torch.cuda.synchronize()
    assert abs(float(l1.detach()) - float(l2.detach())) < 2e-2
    for n, p in m1.named_parameters():
        q = dict(m2.named_parameters())[n]
        assert _rel(p.grad, q.grad) < 6e-2, n


@pytest.mark.parametrize("layout", ["head_repeat", "right_padded"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("V,C,N", [(50257, 768, 8192), (1024, 256, 512), (7, 64, 1000), (33, 4096, 5), (49152, 576, 2048)])
def test_embedding_backward(dev, dt, V, C, N, layout):
    g = torch.Generator(device="cpu").manual_seed(V + N)
    idx = torch.randint(0, V, (N,), generator=g)
    if layout == "head_repeat":
        idx[: N // 4] = idx[0]  # one heavily repeated id
    else:  # 16 right-padded rows: each row's tail is the pad id 2 (runs across many waves' slots)
        r = idx.view(16, -1) if N % 16 == 0 else idx.view(1, -1)
        for i in range(r.shape[0]):
            r[i, int(torch.randint(1, r.shape[1] + 1, (1,), generator=g)):] = 2 % V
    w = torch.randn(V, C, generator=g).to(dev, dt).requires_grad_(True)
    dy = torch.randn(N, C, generator=g).to(dev, dt)
    ops.embedding(idx.to(dev), w).backward(dy)
    ref = torch.zeros(V, C, dtype=torch.float32).index_add_(0, idx, dy.float().cpu())
    tol = 2e-2 if dt == torch.bfloat16 else 1e-5
    assert w.grad.dtype == dt
    assert torch.allclose(w.grad.float().cpu(), ref, atol=tol * (1 + float(ref.abs().max()) * 0.1), rtol=tol)
