"""256x256 phase-interleaved HIP GEMM (csrc/kernels/gemm256.hip) vs an fp32 PyTorch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from nbdistributed_amd.ops import gemm as G  # noqa: E402

LAYOUTS = [(False, False), (False, True), (True, True)]  # forward, dgrad, wgrad
T256 = 80256256  # 8 waves, 256 x 256


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


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("layout", LAYOUTS, ids=["fwd", "dgrad", "wgrad"])
@pytest.mark.parametrize("shape", [(256, 256, 64), (256, 256, 128), (256, 512, 192), (512, 256, 320),
                                   (768, 1024, 768), (256, 256, 1088)])
def test_gemm256_layouts(layout, shape, variant):
    # K-tile counts 1, 2, 3 (odd: the loop ends on buffer 0), 5, 12 and 17; every schedule variant
    M, N, K = shape
    a_km, b_kn = layout
    a, b = _operands(M, N, K, a_km, b_kn)
    c = G.matmul(a, b, a_km=a_km, b_kn=b_kn, tile=T256 + (variant + 2) * 1000000, splits=1)
    assert c.shape == (M, N)
    assert _err(c, _ref(a, b, a_km, b_kn)) < 1e-2


def test_gemm256_identity_with_asymmetric_b():
    # A = I: a row/column swap or a wrong half-image row map in the C write shows up exactly
    M = N = K = 256
    a = torch.eye(M, device="cuda", dtype=torch.bfloat16)
    b = ((torch.arange(N, device="cuda").view(N, 1) * 3 + torch.arange(K, device="cuda").view(1, K)) % 251).to(torch.bfloat16)
    c = G.matmul(a, b, tile=T256, splits=1)
    assert torch.equal(c, b.t().contiguous())


@pytest.mark.parametrize("layout", LAYOUTS, ids=["fwd", "dgrad", "wgrad"])
@pytest.mark.parametrize("splits", [2, 4])
@pytest.mark.parametrize("variant", [0, 6])  # 6: non-temporal C stores (slabs keep plain stores)
def test_gemm256_split_k(layout, splits, variant):
    M, N, K = 256, 512, 2048
    a_km, b_kn = layout
    a, b = _operands(M, N, K, a_km, b_kn, seed=1)
    c = G.matmul(a, b, a_km=a_km, b_kn=b_kn, tile=T256 + (variant + 2) * 1000000, splits=splits)
    assert _err(c, _ref(a, b, a_km, b_kn)) < 1e-2


def test_gemm256_bias_and_gelu_epilogues():
    M, N, K = 512, 768, 320
    a, b = _operands(M, N, K, False, False, seed=3)
    bias = (torch.randn(N, device="cuda") * 0.5).to(torch.bfloat16)
    ref = _ref(a, b, False, False) + bias.float()
    c = G.matmul(a, b, bias=bias, tile=T256, splits=1)
    assert _err(c, ref) < 1e-2
    g, pre = G.matmul(a, b, bias=bias, epi=G.EPI_GELU, tile=T256, splits=1)
    assert _err(pre, ref) < 1e-2
    assert _err(g, torch.nn.functional.gelu(pre.float(), approximate="tanh")) < 1e-2


def test_gemm256_dgelu_epilogue():
    M, N, K = 512, 256, 768  # dgrad layout: A = dy [M][K'], B = W as [K'][N]
    dy, w = _operands(M, N, K, False, True, seed=4)
    pre = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    c = G.matmul(dy, w, b_kn=True, epi=G.EPI_DGELU, aux=pre, tile=T256, splits=1)
    assert _err(c, G._dgelu_ref(_ref(dy, w, False, True), pre).float()) < 2e-2


def test_gemm256_matches_128_tile_kernel():
    # same product through both kernel families: equal up to fp32 summation order
    M, N, K = 1024, 1024, 1536
    a, b = _operands(M, N, K, False, False, seed=6)
    c256 = G.matmul(a, b, tile=T256, splits=1).float()
    c128 = G.matmul(a, b, tile=2128128, splits=1).float()
    assert _err(c256, c128) < 8e-3


def test_large_plain_product_routes_to_library_and_gelu_stays_fused():
    # 2*M*N*K >= 2^36 without an epilogue -> hipBLASLt; with GELU -> the 256x256 kernel
    M, N, K = 4096, 4096, 2048
    a, b = _operands(M, N, K, False, False, seed=8)
    assert G.prefer_library(False, False, M, N, K, G.EPI_NONE)
    bias = torch.randn(N, device="cuda").to(torch.bfloat16)
    ref = _ref(a, b, False, False) + bias.float()
    assert _err(G.matmul(a, b, bias=bias), ref) < 1e-2
    g, pre = G.matmul(a, b, bias=bias, epi=G.EPI_GELU)
    assert G.config(False, False, M, N, K, can_split=False, epi=G.EPI_GELU) == (G.G256, 1)
    assert _err(pre, ref) < 1e-2
