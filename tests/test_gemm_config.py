"""Kernel selection of ops.gemm.config (CPU: pure Python)."""
from nbdistributed_amd.ops import gemm as G


def test_large_forward_products_take_the_256_kernel():
    assert G.config(False, False, 4096, 4096, 4096) == (G.G256, 1)
    assert G.config(False, False, 8192, 8192, 8192, epi=G.EPI_GELU) == (G.G256, 1)
    assert G.config(False, False, 8192, 3072, 2048)[0] != G.G256  # 384 tiles: 1.5 rounds


def test_large_plain_products_prefer_hipblaslt():
    assert G.prefer_library(False, False, 8192, 2048, 8192, G.EPI_NONE)
    assert not G.prefer_library(False, False, 8192, 2048, 8192, G.EPI_GELU)  # fused epilogue: ours
    assert not G.prefer_library(False, False, 8192, 3072, 768, G.EPI_NONE)  # GPT-2 c_fc: tuned, ours
    assert not G.prefer_library(False, False, 2048, 960, 576, G.EPI_NONE)  # small: ours


def test_256_kernel_only_where_it_applies():
    # transposed layouts, epilogues it lacks, short K, too few tiles, ragged shapes
    assert G.config(False, True, 4096, 4096, 4096)[0] != G.G256
    assert G.config(True, True, 4096, 4096, 4096)[0] != G.G256
    assert G.config(False, False, 4096, 4096, 4096, epi=G.EPI_SWIGLU)[0] != G.G256
    assert G.config(False, False, 4096, 4096, 512)[0] != G.G256
    assert G.config(False, False, 2048, 2048, 4096)[0] != G.G256  # 64 tiles
    assert G.config(False, False, 4096, 4160, 4096)[0] != G.G256


def test_tuned_workload_shapes_keep_their_kernels():
    assert G.config(False, False, 8192, 3072, 768) == (82128128, 1)  # gpt2 c_fc forward
    assert G.config(True, True, 3072, 768, 8192) == (3064128, 4)  # gpt2 c_fc weight gradient


def test_pair_schedule_model_and_table():
    """Grouped-backward schedules: measured entries for the workload shapes, the dispatch model
    for the rest — always a legal (S, order) for the kernel (M divisible into S 64-deep splits)."""
    from nbdistributed_amd.ops import gemm as G

    assert G.pair_schedule(8192, 768, 3072, 128, G.EPI_DGELU) == 2 | 16
    assert G.pair_schedule(8192, 3072, 768, 128) == 4 | 16
    for M, N, K in [(8192, 1024, 4096), (4096, 512, 512), (2048, 640, 384), (1024, 4096, 1024), (512, 128, 128)]:
        tile = 128 if M % 128 == 0 and N % 128 == 0 and K % 128 == 0 else 64
        v = G.pair_schedule(M, N, K, tile)
        s, o = v & 15, v >> 4
        assert s in (1, 2, 4, 8) and o in (0, 1) and M % (64 * s) == 0
    # the model: a long-unit half dispatched first finishes no later than the other order
    assert G._greedy_end([10.0] * 3 + [1.0] * 6, 3) <= G._greedy_end([1.0] * 6 + [10.0] * 3, 3)
