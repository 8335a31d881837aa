"""C++ autograd nodes of the Linear / MLP paths (csrc/kernels/autograd.hip) vs the Python
autograd.Functions running the same kernels (ops/gemm.py _Linear / _MLPGelu / _MLPSwiGLU), and
both vs a plain fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from nbdistributed_amd import ops  # noqa: E402
from nbdistributed_amd.ops import gemm as G  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu(require_gpu):
    ops.load_library()


def _both(fn, *args):
    """(native outputs + grads, python outputs + grads) of fn(*args) with a fixed upstream grad."""
    res = []
    for native in (True, False):
        G.NATIVE_AUTOGRAD = native
        try:
            ins = [a.detach().clone().requires_grad_(a.requires_grad) if a is not None else None for a in args]
            y = fn(*ins)
            gy = torch.randn(y.shape, device=y.device, generator=torch.Generator(device="cuda").manual_seed(5)).to(y.dtype)
            y.backward(gy)
            res.append((y.detach(), [a.grad if a is not None and a.requires_grad else None for a in ins]))
        finally:
            G.NATIVE_AUTOGRAD = True
    return res


def _rand(*shape, scale=1.0, grad=True):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16).requires_grad_(grad)


def _same(a, b):
    (ya, ga), (yb, gb) = a, b
    assert torch.equal(ya, yb)
    for x, y in zip(ga, gb):
        if (x is None) != (y is None):  # an unused output: no gradient natively, zeros from Python
            assert not (x if x is not None else y).any()
        elif x is not None:
            assert torch.equal(x, y), (x - y).abs().max()


@pytest.mark.parametrize("M,N,K", [(8192, 2304, 768), (2048, 576, 576), (256, 4096, 4096), (320, 192, 448)])
@pytest.mark.parametrize("bias", [True, False])
@pytest.mark.parametrize("x_grad", [True, False])
def test_linear_native_matches_python_and_reference(M, N, K, bias, x_grad):
    torch.manual_seed(M + N)
    x = _rand(2, M // 2, K, grad=x_grad)
    w = _rand(N, K, scale=K ** -0.5)
    b = _rand(N, scale=0.1) if bias else None
    nat, py = _both(G.gemm_linear, x, w, b)
    _same(nat, py)
    xr, wr = x.detach().float().requires_grad_(x_grad), w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_() if bias else None
    yr = F.linear(xr, wr, br)
    yr.backward(torch.randn(yr.shape, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
                .to(torch.bfloat16).float())
    rel = lambda a, r: ((a.float() - r).abs().max() / r.abs().max()).item()  # noqa: E731
    assert rel(nat[0], yr) < 2e-2
    assert rel(nat[1][1], wr.grad) < 2e-2
    if x_grad:
        assert rel(nat[1][0], xr.grad) < 2e-2
    if bias:
        assert rel(nat[1][2], br.grad) < 2e-2


@pytest.mark.parametrize("M,H,I", [(8192, 768, 3072), (512, 256, 1024)])
@pytest.mark.parametrize("bias", [True, False])
def test_mlp_gelu_native_matches_python(M, H, I, bias):
    torch.manual_seed(H)
    x = _rand(M, H)
    w1, w2 = _rand(I, H, scale=H ** -0.5), _rand(H, I, scale=I ** -0.5)
    b1, b2 = (_rand(I, scale=0.1), _rand(H, scale=0.1)) if bias else (None, None)
    _same(*_both(G.mlp_gelu, x, w1, b1, w2, b2))


@pytest.mark.parametrize("M,H,I", [(2048, 576, 1536), (512, 256, 640)])
def test_mlp_swiglu_native_matches_python_and_reference(M, H, I):
    torch.manual_seed(I)
    x = _rand(M, H)
    wgu, wd = _rand(2 * I, H, scale=H ** -0.5), _rand(H, I, scale=I ** -0.5)
    nat, py = _both(G.mlp_swiglu, x, wgu, wd)
    _same(nat, py)
    xr, gr, dr = (t.detach().float().requires_grad_() for t in (x, wgu, wd))
    g, u = F.linear(xr, gr).chunk(2, -1)
    yr = F.linear(F.silu(g) * u, dr)
    assert ((nat[0].float() - yr).abs().max() / yr.abs().max()).item() < 3e-2


def test_native_nodes_without_autograd_and_in_graphs():
    x, w, b = _rand(512, 256, grad=False), _rand(384, 256, scale=0.06, grad=False), _rand(384, grad=False)
    with torch.inference_mode():  # the CUDA-key registration: forward only
        y0 = G.gemm_linear(x, w, b)
    with torch.no_grad():
        y1 = G.gemm_linear(x, w, b)
    assert torch.equal(y0, y1)
    # forward + backward of the native node captured and replayed as a HIP graph
    xg, wg = _rand(512, 256), _rand(384, 256, scale=0.06)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            G.gemm_linear(xg, wg, None).sum().backward()
    torch.cuda.current_stream().wait_stream(s)
    xg.grad = wg.grad = None
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = G.gemm_linear(xg, wg, None)
        out.sum().backward()
    for _ in range(2):
        graph.replay()
    torch.cuda.synchronize()
    ref = G.gemm_linear(xg.detach(), wg.detach(), None)
    assert torch.equal(out, ref)
    want = torch.ones_like(ref).t().float() @ xg.detach().float()  # d(sum)/dW = 1ᵀ·x
    assert (wg.grad.float() - want).abs().max().item() < 0.5


@pytest.mark.parametrize("kind", ["rms", "add_rms", "ln", "add_ln"])
@pytest.mark.parametrize("use", ["both", "y_only", "s_only"])
def test_norm_nodes_native_match_python(kind, use):
    if use != "both" and not kind.startswith("add"):
        pytest.skip("one output")
    torch.manual_seed(len(kind))
    C = 576 if "rms" in kind else 768
    x, d = _rand(4, 256, C), _rand(4, 256, C)
    w = (torch.rand(C, device="cuda") + 0.5).to(torch.bfloat16).requires_grad_()
    b = _rand(C, scale=0.1)

    def fn(x, d, w, b):
        if kind == "rms":
            return ops.rms_norm(x, w, 1e-6)
        if kind == "ln":
            return ops.layer_norm(x, w, b, 1e-5)
        s, y = ops.add_rms_norm(x, d, w, 1e-6) if kind == "add_rms" else ops.add_layer_norm(x, d, w, b, 1e-5)
        return {"both": s * 0.5 + y, "y_only": y * 1.0, "s_only": s * 1.0}[use]

    _same(*_both(fn, x, d, w, b))


@pytest.mark.parametrize("H,Hkv,rope", [(12, 12, False), (9, 3, True)])
def test_attention_qkv_node_native_matches_python(H, Hkv, rope):
    torch.manual_seed(H)
    B, T, D = 2, 256, 64
    qkv = _rand(B, T, (H + 2 * Hkv) * D)
    tabs = ops.rope_tables(T, D, 10000.0, "cuda") if rope else None
    _same(*_both(lambda q: ops.attention_qkv(q, H, causal=True, n_kv_head=Hkv, rope=tabs), qkv))
