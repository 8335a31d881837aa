"""HIP MFMA GEMM (csrc/kernels/gemm.hip) vs an fp32 PyTorch reference of the same product."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from nbdistributed_amd.ops import gemm as G  # noqa: E402

LAYOUTS = [(False, False), (False, True), (True, True)]  # forward, dgrad, wgrad


@pytest.fixture(scope="module", autouse=True)
def _gpu(require_gpu):
    from nbdistributed_amd import ops

    ops.load_library()


def _operands(M, N, K, a_km, b_kn, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn(*((K, M) if a_km else (M, K)), device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(*((K, N) if b_kn else (N, K)), device="cuda", generator=g).to(torch.bfloat16)
    return a, b


def _ref(a, b, a_km, b_kn):
    A = a.float().t() if a_km else a.float()
    B = b.float() if b_kn else b.float().t()
    return A @ B


def _err(x, ref):
    return float((x.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6))


@pytest.mark.parametrize("layout", LAYOUTS, ids=["fwd", "dgrad", "wgrad"])
@pytest.mark.parametrize("tile", [128128, 128064, 64128, 64064, 3128128, 3128064, 3064128, 3064064, 82128128, 83128128,
                                  202064064, 203064064, 202128064, 203064128])
@pytest.mark.parametrize("shape", [(256, 256, 320), (384, 640, 192), (128, 128, 64), (128, 128, 128)])
def test_gemm_layouts_and_tiles(layout, tile, shape):
    M, N, K = shape
    if tile >= 100000000:  # intra-workgroup K-split: K in multiples of 2 x 64
        K = 2 * K if K % 128 else K
    a_km, b_kn = layout
    a, b = _operands(M, N, K, a_km, b_kn)
    c = G.matmul(a, b, a_km=a_km, b_kn=b_kn, tile=tile, splits=1)
    assert c.shape == (M, N) and c.dtype == torch.bfloat16
    assert _err(c, _ref(a, b, a_km, b_kn)) < 1e-2


@pytest.mark.parametrize("tile", [2128096, 3128096, 82128192, 83128192])
@pytest.mark.parametrize("shape", [(256, 576, 320), (384, 192, 192), (128, 384, 64), (512, 768, 1216)])  # N % 192 == 0
@pytest.mark.parametrize("epi", [0, 1])
def test_gemm_forward_128x96_tile(tile, shape, epi):
    """The 128x96 (4 waves) and 128x192 (8 waves) forward tiles (row images only), plain and with
    the bias + GELU epilogue."""
    M, N, K = shape
    a, b = _operands(M, N, K, False, False, seed=3)
    bias = torch.randn(N, device="cuda").to(torch.bfloat16)
    ref = _ref(a, b, False, False) + bias.float()
    if epi == G.EPI_GELU:
        act, pre = G.matmul(a, b, bias=bias, epi=epi, tile=tile, splits=1)
        assert _err(pre, ref) < 1e-2
        assert _err(act, torch.nn.functional.gelu(ref, approximate="tanh")) < 1e-2
    else:
        c = G.matmul(a, b, bias=bias, tile=tile, splits=1)
        assert c.shape == (M, N) and _err(c, ref) < 1e-2
    with pytest.raises(RuntimeError):  # transposed images: not built for 96-wide tiles
        G.matmul(*_operands(M, N, K, False, True), b_kn=True, tile=tile, splits=1)


@pytest.mark.parametrize("layout", LAYOUTS, ids=["fwd", "dgrad", "wgrad"])
@pytest.mark.parametrize("tile,K", [(3064064, 1216), (3128128, 704), (203064064, 1280), (203128064, 1408),
                                    (83128128, 1216)])
def test_gemm_deep_ring_wraps(layout, tile, K):
    # K-tile counts that wrap the S-stage ring several times and end mid-ring
    M, N = 256, 384
    a_km, b_kn = layout
    a, b = _operands(M, N, K, a_km, b_kn, seed=5)
    c = G.matmul(a, b, a_km=a_km, b_kn=b_kn, tile=tile, splits=1)
    assert _err(c, _ref(a, b, a_km, b_kn)) < 1e-2


def test_gemm_identity_with_asymmetric_b():
    # A = I catches a row/column swap in the C write (cdna_hip_programming.md §3)
    M = N = K = 128
    a = torch.eye(M, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(N, device="cuda").view(N, 1) * 3 + torch.arange(K, device="cuda").view(1, K)).to(torch.bfloat16)
    c = G.matmul(a, b, splits=1)  # C = I·Bᵀ
    assert torch.equal(c, b.t().contiguous())


@pytest.mark.parametrize("layout", LAYOUTS, ids=["fwd", "dgrad", "wgrad"])
@pytest.mark.parametrize("splits", [2, 4])
def test_gemm_split_k(layout, splits):
    M, N, K = 128, 192, 2048
    a_km, b_kn = layout
    a, b = _operands(M, N, K, a_km, b_kn, seed=1)
    c = G.matmul(a, b, a_km=a_km, b_kn=b_kn, splits=splits)
    assert _err(c, _ref(a, b, a_km, b_kn)) < 1e-2


def test_gemm_auto_split_for_weight_gradient_shape():
    # GPT-2 attention-projection weight gradient: 768x768 output, K = 8192 tokens
    a, b = _operands(768, 768, 8192, True, True, seed=2)
    c = G.matmul(a, b, a_km=True, b_kn=True)
    assert _err(c, _ref(a, b, True, True)) < 1e-2


def test_gemm_bias_epilogue():
    M, N, K = 256, 384, 256
    a, b = _operands(M, N, K, False, False, seed=3)
    bias = torch.randn(N, device="cuda").to(torch.bfloat16)
    c = G.matmul(a, b, bias=bias)
    assert _err(c, _ref(a, b, False, False) + bias.float()) < 1e-2


def test_gemm_gelu_epilogue():
    M, N, K = 256, 384, 256
    a, b = _operands(M, N, K, False, False, seed=4)
    bias = torch.randn(N, device="cuda").to(torch.bfloat16)
    g, pre = G.matmul(a, b, bias=bias, epi=G.EPI_GELU)
    ref_pre = _ref(a, b, False, False) + bias.float()
    assert _err(pre, ref_pre) < 1e-2
    assert _err(g, torch.nn.functional.gelu(ref_pre, approximate="tanh")) < 1e-2


def test_gemm_dgelu_epilogue():
    M, N, K = 256, 384, 256
    a, b = _operands(M, N, K, False, True, seed=5)
    pre = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    c = G.matmul(a, b, b_kn=True, epi=G.EPI_DGELU, aux=pre)
    x = pre.float().requires_grad_()
    torch.nn.functional.gelu(x, approximate="tanh").backward(_ref(a, b, False, True))
    assert _err(c, x.grad) < 1e-2


def test_gemm_linear_autograd_matches_fp32():
    torch.manual_seed(0)
    x = torch.randn(4, 64, 192, device="cuda").to(torch.bfloat16).requires_grad_()
    w = (torch.randn(320, 192, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_()
    bias = torch.randn(320, device="cuda").to(torch.bfloat16).requires_grad_()
    y = G.gemm_linear(x, w, bias)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, bias))
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(dy.float())
    assert _err(y, yr) < 1e-2
    assert _err(x.grad, xr.grad) < 1e-2
    assert _err(w.grad, wr.grad) < 1e-2
    assert _err(bias.grad, br.grad) < 1e-2


def test_mlp_gelu_autograd_matches_fp32():
    torch.manual_seed(1)
    C, H = 192, 768
    x = torch.randn(2, 128, C, device="cuda").to(torch.bfloat16).requires_grad_()
    w1 = (torch.randn(H, C, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_()
    b1 = (torch.randn(H, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_()
    w2 = (torch.randn(C, H, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_()
    b2 = (torch.randn(C, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_()
    y = G.mlp_gelu(x, w1, b1, w2, b2)
    dy = torch.randn_like(y)
    y.backward(dy)
    ref = [t.detach().float().requires_grad_() for t in (x, w1, b1, w2, b2)]
    F = torch.nn.functional
    yr = F.linear(F.gelu(F.linear(ref[0], ref[1], ref[2]), approximate="tanh"), ref[3], ref[4])
    yr.backward(dy.float())
    assert _err(y, yr) < 2e-2
    for t, r in zip((x, w1, b1, w2, b2), ref):
        assert _err(t.grad, r.grad) < 2e-2


@pytest.mark.parametrize("tile", [64064, 3064128, 128128, 82128128, 203064064, 202128064])
def test_swiglu_epilogue(tile):
    # [g|u] = x·[W_gate; W_up]ᵀ: the workgroup of column block tn takes gate AND up rows
    M, I, K = 256, 384, 256
    x, w = _operands(M, 2 * I, K, False, False, seed=21)
    act, pre = G.matmul(x, w, epi=G.EPI_SWIGLU, tile=tile, splits=1)
    ref = _ref(x, w, False, False)
    assert act.shape == (M, I) and pre.shape == (M, 2 * I)
    assert _err(pre, ref) < 1e-2
    g, u = ref[:, :I], ref[:, I:]
    assert _err(act, torch.nn.functional.silu(g) * u) < 1e-2


@pytest.mark.parametrize("tile", [64064, 2064064, 128128, 82128128, 202064064, 203064128])
def test_dswiglu_epilogue(tile):
    # d[g|u] from dact = dy·W_down, written straight into the [M, 2I] gradient of the projection
    M, H, I = 256, 256, 384
    dy, wd = _operands(M, I, H, False, True, seed=22)  # dy [M, H], W_down [H, I]
    pre = torch.randn(M, 2 * I, device="cuda").to(torch.bfloat16)
    dgu = G.matmul(dy, wd, b_kn=True, epi=G.EPI_DSWIGLU, aux=pre, tile=tile, splits=1)
    assert dgu.shape == (M, 2 * I)
    dact = _ref(dy, wd, False, True)
    g, u = pre.float()[:, :I], pre.float()[:, I:]
    s = torch.sigmoid(g)
    ref = torch.cat([dact * u * s * (1 + g * (1 - s)), dact * g * s], dim=1)
    assert _err(dgu, ref) < 1e-2


def test_mlp_swiglu_autograd_matches_fp32():
    torch.manual_seed(2)
    H, I = 576, 1536  # SmolLM2-135M
    x = torch.randn(2, 128, H, device="cuda").to(torch.bfloat16).requires_grad_()
    wgu = (torch.randn(2 * I, H, device="cuda") * 0.04).to(torch.bfloat16).requires_grad_()
    wd = (torch.randn(H, I, device="cuda") * 0.03).to(torch.bfloat16).requires_grad_()
    y = G.mlp_swiglu(x, wgu, wd)
    dy = torch.randn_like(y)
    y.backward(dy)
    ref = [t.detach().float().requires_grad_() for t in (x, wgu, wd)]
    F = torch.nn.functional
    g, u = F.linear(ref[0], ref[1]).chunk(2, dim=-1)
    yr = F.linear(F.silu(g) * u, ref[2])
    yr.backward(dy.float())
    assert _err(y, yr) < 2e-2
    for t, r in zip((x, wgu, wd), ref):
        assert _err(t.grad, r.grad) < 2e-2


def test_gemm_rejects_bad_shapes_loudly():
    a = torch.randn(100, 64, device="cuda").to(torch.bfloat16)
    b = torch.randn(64, 64, device="cuda").to(torch.bfloat16)
    with pytest.raises(RuntimeError):
        torch.ops.nbd.gemm(a, b, torch.empty(100, 64, device="cuda", dtype=torch.bfloat16), False, False, None, 0,
                           None, None, 1, 0)
    # the Python entry point routes uncovered shapes to PyTorch instead
    c = G.matmul(a, b)
    assert _err(c, a.float() @ b.float().t()) < 1e-2


def test_gemm_split_k_is_deterministic():
    a, b = _operands(768, 768, 8192, True, True, seed=7)
    outs = [G.matmul(a, b, a_km=True, b_kn=True, splits=8) for _ in range(3)]
    assert all(torch.equal(outs[0], o) for o in outs[1:])


@pytest.mark.parametrize("splits", [1, 2, 8])
@pytest.mark.parametrize("tile", [2128128, 3064128, 2064064, 3128064, 82128128, 83128128, 202064064, 203064128])
def test_gemm_rowsum_epilogue_is_the_bias_gradient(splits, tile):
    # weight-gradient layout: dW = dyᵀ·x and db = Σ_tokens dy from the same kernel
    M, N, K = 256, 384, 2048
    a, b = _operands(M, N, K, True, True, seed=8)
    c, rs = G.matmul(a, b, a_km=True, b_kn=True, epi=G.EPI_ROWSUM, splits=splits, tile=tile)
    assert _err(c, _ref(a, b, True, True)) < 1e-2
    assert rs.shape == (M,) and rs.dtype == torch.bfloat16
    assert _err(rs, a.float().sum(0)) < 1e-2


# ---------------------------------------------------------------- grouped backward (gemm_pair)
@pytest.mark.parametrize("dgelu", [False, True])
@pytest.mark.parametrize("bias_grad", [False, True])
@pytest.mark.parametrize("M,N,K", [(8192, 768, 3072), (8192, 3072, 768), (1024, 256, 384), (8192, 768, 768),
                                   (2048, 576, 960), (2048, 1536, 576)])  # 64-granular: SmolLM2 (64x64 tiles)
def test_gemm_pair_matches_separate_products(dgelu, bias_grad, M, N, K):
    """dx = dy·W (· gelu'(pre)), dW = dyᵀ·x, db = Σ dy from one grouped launch = the fp32 reference."""
    from nbdistributed_amd.ops import gemm as G

    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    dy = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    pre = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16) if dgelu else None
    r = G.backward_pair(dy, w, x, G.EPI_DGELU if dgelu else G.EPI_NONE, pre, bias_grad=bias_grad)
    assert r is not None
    dx, dw, db = r
    ref_dx = dy.float() @ w.float()
    if dgelu:
        ref_dx = G._dgelu_ref(ref_dx, pre).float()
    rel = lambda a, b: float((a.float() - b).abs().max() / b.abs().max())  # noqa: E731
    assert rel(dx, ref_dx) < 1e-2
    assert rel(dw, dy.float().t() @ x.float()) < 1e-2
    if bias_grad:
        assert rel(db, dy.float().sum(0)) < 1e-2
    else:
        assert db is None


@pytest.mark.parametrize("sched", [1 | 16, 2, 2 | 16, 4 | 16, 8, 8 | 16])
@pytest.mark.parametrize("M,N,K", [(2048, 384, 640), (1024, 320, 192)])  # 128- and 64-tile kernels
def test_gemm_pair_schedules(sched, M, N, K):
    """Every split count / dispatch order of the grouped launch (S | wfirst << 4, including unit
    counts that are not multiples of 8: 3x5x2 weight-gradient tiles) = the fp32 reference."""
    from nbdistributed_amd.ops import gemm as G

    g = torch.Generator(device="cuda").manual_seed(sched + M)
    dy = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    pre = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    dx = torch.full((M, K), float("nan"), device="cuda", dtype=torch.bfloat16)
    dw = torch.full((N, K), float("nan"), device="cuda", dtype=torch.bfloat16)
    db = torch.full((N,), float("nan"), device="cuda", dtype=torch.bfloat16)
    torch.ops.nbd.gemm_pair(dy, w, dx, G.EPI_DGELU, pre, dy, x, dw, G.EPI_ROWSUM, db, sched)
    rel = lambda a, b: float((a.float() - b).abs().max() / b.abs().max())  # noqa: E731
    assert rel(dx, G._dgelu_ref(dy.float() @ w.float(), pre).float()) < 1e-2
    assert rel(dw, dy.float().t() @ x.float()) < 1e-2
    assert rel(db, dy.float().sum(0)) < 1e-2


@pytest.mark.parametrize("M,N,I", [(2048, 576, 1536), (1024, 512, 1024)])
def test_gemm_pair_swiglu_backward(M, N, I):
    """Llama MLP backward through the grouped launch: d[g|u] (SwiGLU′ epilogue) + dW_down."""
    from nbdistributed_amd.ops import gemm as G

    g = torch.Generator(device="cuda").manual_seed(M + I)
    dy = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    w_down = (torch.randn(N, I, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    act = torch.randn(M, I, device="cuda", generator=g).to(torch.bfloat16)
    pre = torch.randn(M, 2 * I, device="cuda", generator=g).to(torch.bfloat16)
    r = G.backward_pair(dy, w_down, act, G.EPI_DSWIGLU, pre)
    assert r is not None
    dgu, dw, db = r
    ref = G._dswiglu_ref((dy.float() @ w_down.float()).to(torch.bfloat16), pre).float()
    rel = lambda a, b: float((a.float() - b).abs().max() / b.abs().max())  # noqa: E731
    assert dgu.shape == (M, 2 * I) and rel(dgu, ref) < 2e-2
    assert rel(dw, dy.float().t() @ act.float()) < 1e-2 and db is None


@pytest.mark.parametrize("layout", ["fwd", "dgrad", "wgrad"])
@pytest.mark.parametrize("K", [64, 128, 192, 768])
def test_gemm_ping_pong_schedule(layout, K):
    """Tile code 89128128: 128x128, 8 waves, 3-buffer ring, staggered wave groups (one barrier
    apart) — every ring phase (K = 1, 2, 3 and 12 K-tiles) against the fp32 reference."""
    a_km, b_kn = {"fwd": (False, False), "dgrad": (False, True), "wgrad": (True, True)}[layout]
    g = torch.Generator(device="cuda").manual_seed(K)
    M, N = 256, 384
    A = (torch.randn(*((K, M) if a_km else (M, K)), device="cuda", generator=g)).to(torch.bfloat16)
    B = (torch.randn(*((K, N) if b_kn else (N, K)), device="cuda", generator=g)).to(torch.bfloat16)
    ref = (A.float().t() if a_km else A.float()) @ (B.float() if b_kn else B.float().t())
    out = G.matmul(A, B, a_km=a_km, b_kn=b_kn, tile=89128128, splits=1)
    assert (out.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    if layout == "fwd":
        bias = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
        y, pre = G.matmul(A, B, bias=bias, epi=G.EPI_GELU, tile=89128128, splits=1)
        rp = ref + bias.float()
        assert (pre.float() - rp).abs().max().item() < 2e-2 * rp.abs().max().item()
        ry = torch.nn.functional.gelu(rp, approximate="tanh")
        assert (y.float() - ry).abs().max().item() < 2e-2 * ry.abs().max().item()
    if layout == "wgrad":
        c, rs = G.matmul(A, B, a_km=True, b_kn=True, epi=G.EPI_ROWSUM, tile=89128128, splits=1)
        assert (rs.float() - A.float().sum(0)).abs().max().item() < 2e-2 * A.float().sum(0).abs().max().item()


@pytest.mark.parametrize("dgelu", [False, True])
def test_gemm_pair_ping_pong(dgelu, monkeypatch):
    monkeypatch.setenv("NBD_GEMM_PAIR_PP", "1")
    g = torch.Generator(device="cuda").manual_seed(3)
    M, N, K = 1024, 384, 256
    dy = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    aux = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16) if dgelu else None
    dx, dw, db = G.backward_pair(dy, w, x, G.EPI_DGELU if dgelu else G.EPI_NONE, aux, True)
    rdx = dy.float() @ w.float()
    if dgelu:
        rdx = G._dgelu_ref(rdx, aux)
    rdw = dy.float().t() @ x.float()
    assert (dx.float() - rdx.float()).abs().max().item() < 2e-2 * rdx.float().abs().max().item()
    assert (dw.float() - rdw).abs().max().item() < 2e-2 * rdw.abs().max().item()
    assert (db.float() - dy.float().sum(0)).abs().max().item() < 2e-2 * dy.float().sum(0).abs().max().item()


def test_gemm_next_weight_warm_up(monkeypatch):
    """The warm-up blocks (gemm.hip namespace warm) only read: results are bit-identical with and
    without them, for learned forward / backward chains, weights that are views at odd offsets of
    a larger storage, and after the next weight's storage was freed."""
    g = torch.Generator(device="cuda").manual_seed(7)
    M, K = 512, 384
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    flat = torch.randn(3 * 384 * K + 40, device="cuda", generator=g).to(torch.bfloat16)
    w1 = flat[8:8 + 384 * K].view(384, K)  # 16-B aligned, not 128-B aligned
    w2 = flat[8 + 384 * K:8 + 2 * 384 * K].view(384, K)
    w3 = torch.randn(256, K, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(M, 384, device="cuda", generator=g).to(torch.bfloat16)

    def seq():
        out = [G.matmul(x, w, splits=1) for w in (w1, w2, w3)]
        out += [G.matmul(dy, w, b_kn=True, splits=1) for w in (w2, w1)]
        out += list(G.backward_pair(dy, w1, x, 0, None, True))
        return out

    monkeypatch.setenv("NBD_GEMM_WARM", "0")
    ref = seq()
    monkeypatch.setenv("NBD_GEMM_WARM", "1")
    for _ in range(3):  # learn, then run with the warm-up blocks in place
        got = seq()
        torch.cuda.synchronize()
        for r, o in zip(ref, got):
            assert torch.equal(r, o)
    del w3  # the entry pointing at w3's storage must be dropped, not read
    torch.cuda.empty_cache()
    assert torch.equal(G.matmul(x, w2, splits=1), ref[1])
    torch.cuda.synchronize()



# column split (gemm.hip kColSplit): the columns that make whole rounds of 256x256 tiles on the
# 8-phase kernel, the rest on the tail tile, both writing one C; M = 8192 -> 2048 columns a round
@pytest.mark.parametrize("N,tail", [(2304, 82128128), (3072, 82128128), (3072, 2128128), (2048, 82128128),
                                    (768, 82128128)])
@pytest.mark.parametrize("epi", [G.EPI_NONE, G.EPI_GELU])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm_column_split(N, tail, epi, bias):
    M, K = 8192, 256
    a, b = _operands(M, N, K, False, False, seed=N + epi)
    bb = (torch.randn(N, device="cuda") * 0.5).to(torch.bfloat16) if bias else None
    ref = _ref(a, b, False, False) + (bb.float() if bias else 0.0)
    out = G.matmul(a, b, bias=bb, epi=epi, tile=G.COLSPLIT + tail, splits=1)
    if epi == G.EPI_GELU:
        g, pre = out
        assert _err(pre, ref) < 1e-2
        assert _err(g, torch.nn.functional.gelu(ref, approximate="tanh")) < 1e-2
    else:
        assert _err(out, ref) < 1e-2


@pytest.mark.parametrize("N", [2304, 3072])
def test_gemm_column_split_dgrad_layout(N):
    """The split on the input-gradient layout (B as [K][N]: column blocks), with GELU'."""
    M, K = 8192, 256
    a, b = _operands(M, N, K, False, True, seed=N)
    ref = _ref(a, b, False, True)
    assert _err(G.matmul(a, b, b_kn=True, tile=G.COLSPLIT + 82128128, splits=1), ref) < 1e-2
    pre = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    want = G._dgelu_ref(ref.to(torch.bfloat16), pre).float()
    got = G.matmul(a, b, b_kn=True, epi=G.EPI_DGELU, aux=pre, tile=G.COLSPLIT + 82128128, splits=1)
    assert _err(got, want) < 2e-2


@pytest.mark.parametrize("M", [1, 63, 1000, 8001])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm_linear_odd_rows_padded(M, bias):
    """A row count off the 64-grid runs on the HIP kernels with zero rows appended (no library
    GEMM): output, input / weight / bias gradients against fp32."""
    import torch.nn.functional as F

    from nbdistributed_amd.ops import gemm as G

    torch.manual_seed(M)
    x = torch.randn(M, 256, device="cuda").to(torch.bfloat16).requires_grad_()
    w = (torch.randn(192, 256, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_()
    b = (torch.randn(192, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_() if bias else None
    assert G._pad_rows(x, w) is not None
    y = G.gemm_linear(x, w, b)
    assert y.shape == (M, 192)
    dy = torch.randn(M, 192, device="cuda").to(torch.bfloat16)
    y.backward(dy)
    xf, wf = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    bf = b.detach().float().requires_grad_() if bias else None
    yf = F.linear(xf, wf, bf)
    yf.backward(dy.float())

    def rel(a, r):
        return float((a.float() - r).abs().max() / r.abs().max().clamp_min(1e-6))

    assert rel(y, yf) < 1e-2 and rel(x.grad, xf.grad) < 1e-2 and rel(w.grad, wf.grad) < 2e-2
    if bias:
        assert rel(b.grad, bf.grad) < 2e-2


@pytest.mark.parametrize("M,N,K", [(1000, 1000, 1000), (256, 100, 320), (64, 192, 70)])
def test_gemm_linear_odd_dims_padded(M, N, K, monkeypatch):
    """Weight dims off the 64-grid zero-padded onto the HIP kernels (NBD_GEMM_PAD_DIMS) — output and
    all gradients against fp32."""
    import torch.nn.functional as F

    monkeypatch.setattr(G, "PAD_DIMS", True)
    torch.manual_seed(N + K)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_()
    b = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_()
    assert G._pad_dims(x, w, b) is not None
    y = G.gemm_linear(x, w, b)
    assert y.shape == (M, N)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    y.backward(dy)
    xf, wf, bf = (t.detach().float().requires_grad_() for t in (x, w, b))
    F.linear(xf, wf, bf).backward(dy.float())

    def rel(a, r):
        return float((a.float() - r).abs().max() / r.abs().max().clamp_min(1e-6))

    assert rel(y, F.linear(xf, wf, bf)) < 1e-2
    assert rel(x.grad, xf.grad) < 1e-2 and rel(w.grad, wf.grad) < 2e-2 and rel(b.grad, bf.grad) < 2e-2
