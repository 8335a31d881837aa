"""bf16 GEMM on the MI355X matrix cores with fused epilogues (K12, ``csrc/kernels/gemm.hip``).

``matmul`` is the raw product with the three operand layouts of a Linear layer (forward
``x·Wᵀ``, input gradient ``dy·W``, weight gradient ``dyᵀ·x`` — no transposed copies);
``gemm_linear`` and ``mlp_gelu`` are autograd functions built on it.  ``mlp_gelu`` is GPT-2's
MLP (``c_proj(gelu_tanh(c_fc(x)))``) with the activation fused into the GEMM epilogues: the
forward GEMM writes both the pre-activation and GELU(pre), the backward dgrad of ``c_proj``
multiplies by GELU'(pre) as it stores — no separate elementwise kernels either way.

Shapes the kernel does not cover (a dimension not a multiple of 64, non-bf16, CPU) fall back
to PyTorch (hipBLASLt on ROCm) with identical semantics.
"""
from __future__ import annotations

import os

from ._lib import _require

# NBD_HIP_GEMM=0 routes gemm_linear / mlp_gelu to PyTorch (hipBLASLt) — for A/B measurements
ENABLED = os.environ.get("NBD_HIP_GEMM", "1") != "0"
KSPLIT = os.environ.get("NBD_GEMM_KSPLIT", "1") != "0"
# NBD_GEMM_COLSPLIT=0: the column-split tuned entries run their tail tile over all columns (A/B)
COLSPLIT_ON = os.environ.get("NBD_GEMM_COLSPLIT", "1") != "0"
FUSED_SWIGLU = os.environ.get("NBD_FUSED_SWIGLU", "1") != "0"  # 0: separate swiglu kernels (A/B)
# backward: a Linear's input- and weight-gradient GEMMs as one grouped launch (nbd::gemm_pair,
# 128x128 tiles): the weight-gradient tiles fill the CUs the input-gradient grid leaves idle
PAIR_BWD = os.environ.get("NBD_GEMM_PAIR", "1") != "0"
PAIR_UNITS = int(os.environ.get("NBD_GEMM_PAIR_UNITS", "256"))  # weight-gradient units to split up to
# the Linear / MLP autograd nodes in C++ (csrc/kernels/autograd.hip) instead of the Python
# autograd.Functions below: same kernels, no Python between the dispatcher and the launches
NATIVE_AUTOGRAD = os.environ.get("NBD_NATIVE_AUTOGRAD", "1") != "0"

EPI_NONE, EPI_GELU, EPI_DGELU, EPI_ROWSUM, EPI_SWIGLU, EPI_DSWIGLU = 0, 1, 2, 3, 4, 5


def pair_splits(M2: int, N2: int, K2: int, tile: int = 128) -> int:
    """K splits of the weight-gradient half of a grouped backward launch: enough units to cover
    the CUs (≥ 256 with the input-gradient tiles running alongside), each split ≥ 1024 deep.
    (The round-2 rule; ``pair_schedule`` below supersedes it for the launches.)"""
    t2 = (M2 // tile) * (N2 // tile)
    s = 1
    while t2 * s < PAIR_UNITS and s < 8 and K2 % (64 * 2 * s) == 0 and K2 // (2 * s) >= 1024:
        s *= 2
    return s


# Grouped-backward dispatch model (pair_schedule): workgroup slots resident at once (2 per CU at
# 128x128 / 8 waves — 68 KiB of LDS each; 3 at 64x64), per-unit cost in 64-deep K-steps plus a
# fixed prologue/epilogue, a split-K unit's fp32 slab store, and the reduce kernel's HBM pass.
_PAIR_SLOTS = {128: 512, 64: 768}
_UNIT_OVERHEAD = 3.0   # K-steps: pipeline fill + epilogue of one tile
_SLAB_OVERHEAD = 1.0   # K-steps: fp32 slab instead of a bf16 tile
_STEP_US = 1.0         # ≈ µs per 128x128x64 K-step with two workgroups per CU (c_fc dgrad: 50.9 µs / 48)
_HBM_BPUS = 5.0e6      # bytes per µs (reduce kernel)
# NBD_GEMM_PAIR_SCHED="S:order" forces the split count and the order (0 = input gradient first,
# 1 = weight gradient first) of every grouped launch; "legacy" = the round-2 rule (pair_splits,
# input gradient first) — A/B measurements
_SCHED_ENV = os.environ.get("NBD_GEMM_PAIR_SCHED", "")


def _greedy_end(units, slots: int) -> float:
    """Finish time of `units` (durations, in dispatch order) handed to the earliest-free slot."""
    import heapq

    h = [0.0] * slots
    end = 0.0
    for d in units:
        t = heapq.heappop(h) + d
        end = max(end, t)
        heapq.heappush(h, t)
    return end


# Measured best schedules (S | wfirst << 4) of the workload's grouped launches, keyed by
# (M, N, K, epi1) for dy [M, N], W [N, K] (benchmarks/pair_sched.py, profiles/pair_sched_r3.txt);
# the model below covers other shapes (it picks these or schedules within 1-7 % of them)
_PAIR_TUNED = {
    (8192, 2304, 768, EPI_NONE): 2 | 16,   # gpt2.c_attn   74.0 us (round-2 rule S=4, input first: 79.0)
    (8192, 768, 768, EPI_NONE): 8 | 16,    # gpt2.attn.c_proj 35.6 us (38.5)
    (8192, 3072, 768, EPI_NONE): 4 | 16,   # gpt2.c_fc     92.5 us (S=2, input first: 102.8)
    (8192, 768, 3072, EPI_DGELU): 2 | 16,  # gpt2.mlp.c_proj 98.9 us (110.7)
    (2048, 960, 576, EPI_NONE): 2 | 16,    # smollm2.qkv   15.5 us (16.1)
    (2048, 576, 576, EPI_NONE): 2 | 16,    # smollm2.o_proj 12.9 us (13.4)
    (2048, 3072, 576, EPI_NONE): 1,        # smollm2.gate_up 25.0 us
    (2048, 576, 1536, EPI_DSWIGLU): 1 | 16,  # smollm2.down (+SwiGLU') 18.4-18.7 us (model: S=2 input first 23.4-25.5;
                                             # profiles/pair_sched_smollm2_r3.txt)
}


# NBD_GEMM_PAIR_TUNE (in-step A/B runs): entries "M:N:K:epi1=S:wfirst" joined by "+"
for _ent in filter(None, (e.strip() for e in os.environ.get("NBD_GEMM_PAIR_TUNE", "").split("+"))):
    _k, _v = _ent.split("=")
    _m, _n, _kk, _e = (int(v) for v in _k.split(":"))
    _s, _o = (int(v) for v in _v.split(":"))
    _PAIR_TUNED[(_m, _n, _kk, _e)] = _s | (_o << 4)


def pair_schedule(M: int, N: int, K: int, tile: int = 128, epi1: int = EPI_NONE) -> int:
    """Split count and dispatch order of the grouped backward launch for dy [M, N], W [N, K]
    (dx = dy·W: (M/t)(K/t) units of N/64 K-steps; dW = dyᵀ·x: (N/t)(K/t)·S units of M/(64 S)),
    encoded as S | wfirst << 4 (gemm.hip gemm_pair_hip).  The workgroup dispatcher hands out
    blocks in id order as slots free up, so the finish time is the greedy list schedule of the
    two halves: chosen by that model over S ∈ {1, 2, 4, 8} and both orders, plus the reduce
    pass S > 1 costs; measured entries (``_PAIR_TUNED``) first.  GPT-2 small (8192 tokens): the
    MLP pairs went from S = 2, input gradient first (a 48- or 12-step half, then 64-step
    weight-gradient units as a serial tail) to weight gradient first (docs/FINDINGS.md §24)."""
    if _SCHED_ENV == "legacy":
        return pair_splits(N, K, M, tile)
    if _SCHED_ENV:
        s, o = (int(v) for v in _SCHED_ENV.split(":"))
        return s | (o << 4)
    hit = _PAIR_TUNED.get((M, N, K, epi1))
    if hit is not None:
        return hit
    slots = _PAIR_SLOTS.get(tile, 512)
    t1 = (M // tile) * (K // tile)
    t2 = (N // tile) * (K // tile)
    best = None
    for s in (1, 2, 4, 8):
        if M % (64 * s) or (s > 1 and M // s < 512):
            continue
        d1 = [N / 64 + _UNIT_OVERHEAD + (1.0 if epi1 != EPI_NONE else 0.0)] * t1
        d2 = [M / 64 / s + _UNIT_OVERHEAD + (_SLAB_OVERHEAD if s > 1 else 0.0)] * (t2 * s)
        red = (s * N * K * 4 + N * K * 2) / _HBM_BPUS / _STEP_US if s > 1 else 0.0
        for order, units in ((0, d1 + d2), (1, d2 + d1)):
            t = _greedy_end(units, slots) + red
            if best is None or t < best[0] - 1e-9:
                best = (t, s | (order << 4))
    return best[1] if best else 1


def backward_pair(dy2, w, x2, epi1: int = EPI_NONE, aux1=None, bias_grad: bool = False):
    """(dy2·w [· act′(aux1)], dy2ᵀ·x2, Σ_rows dy2 or None) — a Linear's input gradient, weight
    gradient and bias gradient from one grouped HIP launch (``epi1`` = EPI_DGELU with the GELU
    pre-activation, or EPI_DSWIGLU with the [g|u] pre-activations: the input gradient is then
    d[g|u] [M, 2K]); None when the shapes / dtypes do not fit it (the caller then runs the
    products one by one)."""
    import torch

    if not (PAIR_BWD and ENABLED and dy2.is_cuda and dy2.dtype == w.dtype == x2.dtype == torch.bfloat16
            and not torch.is_autocast_enabled()):
        return None
    M, N = dy2.shape
    K = w.shape[1]
    cols = 2 * K if epi1 == EPI_DSWIGLU else K
    if (M % 64 or N % 64 or K % 64 or w.shape[0] != N or x2.shape != (M, K) or not dy2.is_contiguous()
            or not w.is_contiguous() or not x2.is_contiguous()
            or (aux1 is not None and (not aux1.is_contiguous() or aux1.shape != (M, cols)))):
        return None
    _require()
    tile = 128 if M % 128 == 0 and N % 128 == 0 and K % 128 == 0 else 64
    dx = torch.empty(M, cols, dtype=dy2.dtype, device=dy2.device)
    dw = torch.empty(N, K, dtype=dy2.dtype, device=dy2.device)
    db = torch.empty(N, dtype=dy2.dtype, device=dy2.device) if bias_grad else None
    torch.ops.nbd.gemm_pair(dy2, w, dx, epi1, aux1, dy2, x2, dw, EPI_ROWSUM if bias_grad else EPI_NONE, db,
                            pair_schedule(M, N, K, tile, epi1))
    return dx, dw, db


def gemm_ok(M: int, N: int, K: int) -> bool:
    return M > 0 and N > 0 and K > 0 and M % 64 == 0 and N % 64 == 0 and K % 64 == 0


# Measured best (kernel, split-K) per (a_km, b_kn, M, N, K) on MI355X for the bench workloads'
# Linear products — kernel = ks*10^8 (2 K-groups in the workgroup; 1 if absent) + waves*10^7
# (8 waves; 4 if absent) + stages*10^6 + BM*1000 + BN; from
# benchmarks/gemm_bench.py --sweep
# (profiles/gemm_bench_r1.txt; split-K only where it beats the best unsplit kernel by > 5 %).
_TUNED = {
    # gpt2.c_attn fwd 44.5 us.  (A column split — columns 0..2047 on the 256x256 kernel, one round,
    # the rest on 128x128: 41.1 us isolated — made the graphed step 0.12 ms slower: COLSPLIT below)
    (False, False, 8192, 2304, 768): (82128128, 1),
    (False, True, 8192, 768, 2304): (82128128, 1),  # gpt2.c_attn dgrad 42.3 us
    (True, True, 2304, 768, 8192): (203128064, 1),  # gpt2.c_attn wgrad 49.7 us (K-split groups)
    (False, False, 8192, 768, 768): (2128096, 1),  # gpt2.attn.c_proj fwd 14.8 us (128x128/8 waves 16.5: 512 tiles = one round)
    (False, True, 8192, 768, 768): (2128064, 1),  # gpt2.attn.c_proj dgrad 21.8 us
    (True, True, 768, 768, 8192): (203064064, 1),  # gpt2.attn.c_proj wgrad 32.7 us (no reduce kernel)
    (False, False, 8192, 3072, 768): (82128128, 1),  # gpt2.c_fc fwd 49.7 us
    (False, True, 8192, 768, 3072): (2128128, 1),  # gpt2.c_fc dgrad 50.9 us
    (True, True, 3072, 768, 8192): (3064128, 4),  # gpt2.c_fc wgrad 72.6 us
    # gpt2.mlp.c_proj fwd (128x192 / 8 waves / 3 stages, 256 tiles = one round: 44.6 us plain, 47.5
    # with bias vs 45.8 / 49.1 isolated, the GPT-2 step unchanged at 11.00 ms; profiles/gemm_tile192_r5.txt)
    (False, False, 8192, 768, 3072): (2128096, 1),  # 48.2 us (128x128 50.0; profiles/gemm96_r2.txt)
    (False, True, 8192, 3072, 768): (82128128, 1),  # gpt2.mlp.c_proj dgrad 50.9 us
    (True, True, 768, 3072, 8192): (82128128, 2),  # gpt2.mlp.c_proj wgrad 68.9 us
    (False, False, 2048, 960, 576): (3064064, 1),  # smollm2.qkv fwd 13.5 us
    (False, True, 2048, 576, 960): (3064064, 1),  # smollm2.qkv dgrad 14.9 us
    (True, True, 960, 576, 2048): (203064064, 1),  # smollm2.qkv wgrad 13.2 us (15.3 one K-group)
    (False, False, 2048, 576, 576): (3064064, 1),  # smollm2.o_proj fwd 7.3 us vs 7.9 (2-stage;
                                                   # profiles/gemm_fwd_smollm2_r3.txt)
    (False, True, 2048, 576, 576): (2064064, 1),  # smollm2.o_proj dgrad 13.0 us
    (True, True, 576, 576, 2048): (203064064, 1),  # smollm2.o_proj wgrad 13.2 us (15.0)
    (False, False, 2048, 3072, 576): (2064128, 1),  # smollm2.gate_up fwd 19.4 us
    (False, True, 2048, 576, 3072): (202064064, 1),  # smollm2.gate_up dgrad 22.3 us
    (True, True, 3072, 576, 2048): (3064064, 1),  # smollm2.gate_up wgrad 22.0 us
    (False, False, 2048, 576, 1536): (202064064, 1),  # smollm2.down fwd 13.6 us (14.5)
    (False, True, 2048, 1536, 576): (2064064, 1),  # smollm2.down dgrad 15.3 us
    (True, True, 576, 1536, 2048): (203064064, 1),  # smollm2.down wgrad 13.7 us (15.6)
}

# epilogue-specific entries, checked first: (a_km, b_kn, M, N, K, epi).  (The column split of c_fc +
# GELU — 53.4 vs 57.2 us isolated, profiles/gemm_colsplit_r6.txt — lost in the step with q|k|v's:
# graphed GPT-2 10.53-10.58 vs 10.41-10.44 ms, eager 10.73-10.75 vs 10.60-10.66,
# profiles/colsplit_step_ab_r6.txt: the 256x256 head launch has no next-weight warm-up and the
# two launches each pay a ramp; in the step each product measured 43.1 / 56.4 us split vs 43.1 /
# 57.4 whole, profiles/gpt2_graph_prof_r6a.md)
_TUNED_EPI: dict = {}


def _env_tuned(spec: str) -> dict:
    """NBD_GEMM_TUNE (in-step A/B runs): entries "a_km:b_kn:M:N:K=tile:splits" joined by "+",
    e.g. "0:0:2048:576:576=203064064:1", overriding the measured table."""
    out = {}
    for ent in filter(None, (e.strip() for e in spec.split("+"))):
        key, val = ent.split("=")
        a, b, m, n, k = (int(v) for v in key.split(":"))
        t, sp = (int(v) for v in val.split(":"))
        out[(bool(a), bool(b), m, n, k)] = (t, sp)
    return out


_TUNED.update(_env_tuned(os.environ.get("NBD_GEMM_TUNE", "")))

_TILES = (128128, 128064, 64128, 64064)  # (+ 128096: forward only, tuned entries)


def _ntiles(tile: int, M: int, N: int) -> int:
    bm, bn = tile // 1000 % 1000, tile % 1000
    return (M // bm) * (N // bn) if M % bm == 0 and N % bn == 0 else 0


# the 256x256 phase-interleaved kernel (gemm256.hip) with staggered wave groups: forward products
# with whole rounds of 256 such tiles (256, 512, ... or >= 1024) and K >= 1024 (1.22-1.34 PF vs
# 0.98-1.16 for the 128x128 kernel at 4096^3, 8192^3 and Llama-1B's o_proj / down; 1.5 rounds
# (Llama-1B q|k|v, 384 tiles) lose: docs/FINDINGS.md §10); its epilogues: none / bias / GELU
G256 = 86256256
G256_EPIS = (EPI_NONE, EPI_GELU)
# column split (gemm.hip kColSplit): COLSPLIT + tail tile runs the columns that make whole rounds
# of 256x256 tiles on the 8-phase kernel and the rest on the tail tile (two launches, one C) —
# available as a tile hint, in no tuned entry (slower in the GPT-2 step, _TUNED_EPI note)
COLSPLIT = 1000000000
# Plain products at least this large (FLOPs) with no tuned entry go to hipBLASLt: it measured
# 1.16-1.61 PF on them, 15-30 % ahead of both hand-written families (profiles/gemm256_bench_r2.txt);
# the hand-written kernels keep the fused epilogues and the workload shapes they win on.
LIBRARY_MIN_FLOPS = 2 ** 36


def prefer_library(a_km: bool, b_kn: bool, M: int, N: int, K: int, epi: int) -> bool:
    return (epi == EPI_NONE and (a_km, b_kn, M, N, K) not in _TUNED and 2.0 * M * N * K >= LIBRARY_MIN_FLOPS)


def config(a_km: bool, b_kn: bool, M: int, N: int, K: int, can_split: bool = True, epi: int = EPI_NONE):
    """(kernel, splits) for a product: the tuned entry when there is one, else a heuristic —
    large forward products on the 256x256 kernel; else the largest tile with >= 1024 workgroups
    (128x128), else >= 256 (128x64 / 64x128), else 64x64; the 3-stage pipeline when there are
    < 512 workgroups (one per CU cannot hide a drained pipeline); long-K products with < 400
    workgroups split K (the largest tile needing <= 8 splits, each >= 512 deep) — split-K (a
    second, reducing kernel) only without an epilogue."""
    hit = _TUNED_EPI.get((a_km, b_kn, M, N, K, epi)) or _TUNED.get((a_km, b_kn, M, N, K))
    if hit is not None and hit[0] >= COLSPLIT and not COLSPLIT_ON:
        hit = (hit[0] - COLSPLIT, hit[1])
    if hit is not None and (can_split or hit[1] == 1):
        return hit if KSPLIT else (hit[0] % 100000000, hit[1])
    t256 = (M // 256) * (N // 256)
    if (not a_km and not b_kn and epi in G256_EPIS and M % 256 == 0 and N % 256 == 0
            and (t256 % 256 == 0 or t256 >= 1024) and t256 > 0 and K >= 1024):
        return G256, 1
    fits = [t for t in _TILES if _ntiles(t, M, N)]
    if not fits:
        return 0, 1
    tile = fits[-1]
    for t in fits:
        n = _ntiles(t, M, N)
        if n >= (1024 if t == 128128 else 256):
            tile = t
            break
    if can_split and _ntiles(tile, M, N) < 400 and K >= 2048:
        for t in fits:
            s = 1
            while _ntiles(t, M, N) * s < 400 and s < 8 and K % (64 * 2 * s) == 0 and K // (2 * s) >= 512:
                s *= 2
            if _ntiles(t, M, N) * s >= 400:
                return (3 if _ntiles(t, M, N) * s < 512 else 2) * 1000000 + t, s
    return (3 if _ntiles(tile, M, N) < 512 else 2) * 1000000 + tile, 1


def matmul(a, b, a_km: bool = False, b_kn: bool = False, bias=None, epi: int = EPI_NONE, aux=None, out=None,
           splits: int = 0, tile: int = 0):
    """C[M,N] = A·B.  ``a`` is [M,K] (or [K,M] with ``a_km``), ``b`` is [N,K] (or [K,N] with
    ``b_kn``).  ``epi``: EPI_NONE (+bias), EPI_GELU (+bias, returns (gelu(pre), pre)),
    EPI_DGELU (C · gelu'(aux)), EPI_ROWSUM (weight-gradient layout; returns (C, Σ_k A[m,k]) —
    the bias gradient of the Linear whose weight gradient C is), EPI_SWIGLU (``b`` = [gate; up]
    weights [2I, K]; returns (silu(g)·u [M, I], [g|u] [M, 2I])), EPI_DSWIGLU (dgrad layout,
    ``aux`` = [g|u] [M, 2N]; returns d[g|u] [M, 2N] from dact = A·B).  ``splits=0`` picks split-K
    automatically (no-epilogue only);
    ``tile`` = ks*10^8 + waves*10^7 + stages*10^6 + BM*1000 + BN forces a kernel (waves 4 or 8,
    8 only at 128x128; stages 2 or 3; ks = 2 runs two K-groups of 4 waves inside the workgroup,
    tiles other than 128x128, K a multiple of 128; benchmarks)."""
    import torch

    M = a.shape[1] if a_km else a.shape[0]
    K = a.shape[0] if a_km else a.shape[1]
    N = b.shape[1] if b_kn else b.shape[0]
    library = tile == 0 and splits == 0 and prefer_library(a_km, b_kn, M, N, K, epi)
    if (not library and a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and gemm_ok(M, N, K)
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0 and (out is None or out.data_ptr() % 16 == 0)
            and (bias is None or (bias.data_ptr() % 8 == 0 and bias.dtype == torch.bfloat16))):
        _require()
        a = a if a.is_contiguous() else a.contiguous()
        b = b if b.is_contiguous() else b.contiguous()
        cN = N // 2 if epi == EPI_SWIGLU else 2 * N if epi == EPI_DSWIGLU else N
        c = out if out is not None else torch.empty(M, cN, device=a.device, dtype=a.dtype)
        pre = torch.empty_like(c) if epi == EPI_GELU else None
        if epi == EPI_ROWSUM:
            pre = torch.empty(M, device=a.device, dtype=a.dtype)
        if epi == EPI_SWIGLU:
            pre = torch.empty(M, N, device=a.device, dtype=a.dtype)
        if epi == EPI_DSWIGLU and not aux.is_contiguous():
            aux = aux.contiguous()
        if splits == 0 or tile == 0:
            t, s = config(a_km, b_kn, M, N, K, can_split=(epi in (EPI_NONE, EPI_ROWSUM) and bias is None), epi=epi)
            tile = tile or t
            splits = splits or s
        torch.ops.nbd.gemm(a, b, c, a_km, b_kn, bias, epi, aux, pre, splits, tile)
        return (c, pre) if epi in (EPI_GELU, EPI_ROWSUM, EPI_SWIGLU) else c
    # reference path (CPU / uncovered shapes) and large plain products: same math through PyTorch
    # (hipBLASLt on ROCm)
    A = a.t() if a_km else a
    B = b if b_kn else b.t()
    if bias is not None and epi in (EPI_NONE, EPI_GELU):
        c = torch.addmm(bias, A, B)  # the bias rides in the library GEMM's epilogue
    else:
        c = A @ B
        if bias is not None:
            c = c + bias
    if epi == EPI_GELU:
        pre = c
        c = torch.nn.functional.gelu(pre, approximate="tanh")
        return c, pre
    if epi == EPI_DGELU:
        c = _dgelu_ref(c, aux)
    if epi == EPI_SWIGLU:
        g, u = c.float().chunk(2, dim=1)
        return (torch.nn.functional.silu(g) * u).to(c.dtype), c
    if epi == EPI_DSWIGLU:
        c = _dswiglu_ref(c, aux)
    if epi == EPI_ROWSUM:
        return c, A.float().sum(1).to(a.dtype)
    if out is not None:
        out.copy_(c)
        return out
    return c


def _dgelu_ref(g, pre):
    import torch

    x = pre.float()
    k = 0.7978845608028654
    t = torch.tanh(k * (x + 0.044715 * x * x * x))
    d = 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k * (1 + 3 * 0.044715 * x * x)
    return (g.float() * d).to(g.dtype)


def _dswiglu_ref(dact, pre):
    import torch

    g, u = pre.float().chunk(2, dim=-1)
    d = dact.float()
    sg = torch.sigmoid(g)
    return torch.cat([d * u * sg * (1 + g * (1 - sg)), d * g * sg], dim=-1).to(dact.dtype)


_Fns = None


def _fns():
    global _Fns
    if _Fns is not None:
        return _Fns
    import torch

    def _c(t):
        return t if t.is_contiguous() else t.contiguous()

    def _colsum(x2, dtype):
        return torch.ops.nbd.colsum(x2, dtype) if x2.is_cuda else x2.float().sum(0).to(dtype)

    class _Linear(torch.autograd.Function):
        """y = x·Wᵀ + b on the HIP GEMM; backward = dgrad + wgrad GEMMs + column-sum bias grad."""

        @staticmethod
        def forward(ctx, x, w, b):
            x2 = _c(x).view(-1, x.shape[-1])
            ctx.save_for_backward(x2, w)
            ctx.xshape = x.shape
            ctx.has_bias = b is not None
            y = matmul(x2, w, bias=b)
            return y.view(*x.shape[:-1], w.shape[0])

        @staticmethod
        def backward(ctx, dy):
            x2, w = ctx.saved_tensors
            dy2 = _c(dy).view(-1, dy.shape[-1])
            dx = dw = db = None
            want_db = ctx.has_bias and ctx.needs_input_grad[2]

            def wgrad():
                if ctx.needs_input_grad[1] and want_db:  # bias grad rides in the weight-grad GEMM
                    return matmul(dy2, x2, a_km=True, b_kn=True, epi=EPI_ROWSUM)
                if ctx.needs_input_grad[1]:
                    return matmul(dy2, x2, a_km=True, b_kn=True), None
                return None, (_colsum(dy2, w.dtype) if want_db else None)

            if ctx.needs_input_grad[0] and ctx.needs_input_grad[1]:
                r = backward_pair(dy2, w, x2, bias_grad=want_db)
                if r is not None:
                    return r[0].view(ctx.xshape), r[1], r[2]
            if ctx.needs_input_grad[0]:
                dx = matmul(dy2, w, b_kn=True).view(ctx.xshape)
            dw, db = wgrad()
            return dx, dw, db

    class _MLPGelu(torch.autograd.Function):
        """y = c_proj(gelu_tanh(c_fc(x))) with GELU / GELU' in the GEMM epilogues."""

        @staticmethod
        def forward(ctx, x, w1, b1, w2, b2):
            x2 = _c(x).view(-1, x.shape[-1])
            g, pre = matmul(x2, w1, bias=b1, epi=EPI_GELU)
            y = matmul(g, w2, bias=b2)
            ctx.save_for_backward(x2, w1, w2, pre, g)
            ctx.xshape = x.shape
            ctx.bias = (b1 is not None, b2 is not None)
            return y.view(*x.shape[:-1], w2.shape[0])

        @staticmethod
        def backward(ctx, dy):
            x2, w1, w2, pre, g = ctx.saved_tensors
            dy2 = _c(dy).view(-1, dy.shape[-1])
            r2 = backward_pair(dy2, w2, g, EPI_DGELU, pre, bias_grad=ctx.bias[1])
            if r2 is not None:
                dpre, dw2, db2 = r2
                r1 = backward_pair(dpre, w1, x2, bias_grad=ctx.bias[0]) if ctx.needs_input_grad[0] else None
                if r1 is not None:
                    return r1[0].view(ctx.xshape), r1[1], r1[2], dw2, db2
                if ctx.bias[0]:
                    dw1, db1 = matmul(dpre, x2, a_km=True, b_kn=True, epi=EPI_ROWSUM)
                else:
                    dw1, db1 = matmul(dpre, x2, a_km=True, b_kn=True), None
                dx = matmul(dpre, w1, b_kn=True).view(ctx.xshape) if ctx.needs_input_grad[0] else None
                return dx, dw1, db1, dw2, db2

            def wgrad2():
                if ctx.bias[1]:
                    return matmul(dy2, g, a_km=True, b_kn=True, epi=EPI_ROWSUM)
                return matmul(dy2, g, a_km=True, b_kn=True), None

            dpre = matmul(dy2, w2, b_kn=True, epi=EPI_DGELU, aux=pre)
            dw2, db2 = wgrad2()

            def wgrad1():
                if ctx.bias[0]:
                    return matmul(dpre, x2, a_km=True, b_kn=True, epi=EPI_ROWSUM)
                return matmul(dpre, x2, a_km=True, b_kn=True), None

            dx = matmul(dpre, w1, b_kn=True).view(ctx.xshape) if ctx.needs_input_grad[0] else None
            dw1, db1 = wgrad1()
            return dx, dw1, db1, dw2, db2

    class _MLPSwiGLU(torch.autograd.Function):
        """y = down(silu(g)·u), [g|u] = x·W_guᵀ (Llama MLP) with SwiGLU / its backward in the GEMM
        epilogues: two GEMMs forward, four backward, no elementwise kernels."""

        @staticmethod
        def forward(ctx, x, w_gu, w_down):
            x2 = _c(x).view(-1, x.shape[-1])
            act, pre = matmul(x2, w_gu, epi=EPI_SWIGLU)
            y = matmul(act, w_down)
            ctx.save_for_backward(x2, w_gu, w_down, pre, act)
            ctx.xshape = x.shape
            return y.view(*x.shape[:-1], w_down.shape[0])

        @staticmethod
        def backward(ctx, dy):
            x2, w_gu, w_down, pre, act = ctx.saved_tensors
            dy2 = _c(dy).view(-1, dy.shape[-1])
            r2 = backward_pair(dy2, w_down, act, EPI_DSWIGLU, pre)
            if r2 is not None:
                dgu, dw_down, _ = r2
                r1 = backward_pair(dgu, w_gu, x2) if ctx.needs_input_grad[0] else None
                if r1 is not None:
                    return r1[0].view(ctx.xshape), r1[1], dw_down
                dx = matmul(dgu, w_gu, b_kn=True).view(ctx.xshape) if ctx.needs_input_grad[0] else None
                return dx, matmul(dgu, x2, a_km=True, b_kn=True), dw_down
            dgu = matmul(dy2, w_down, b_kn=True, epi=EPI_DSWIGLU, aux=pre)
            dw_down = matmul(dy2, act, a_km=True, b_kn=True)
            dx = matmul(dgu, w_gu, b_kn=True).view(ctx.xshape) if ctx.needs_input_grad[0] else None
            return dx, matmul(dgu, x2, a_km=True, b_kn=True), dw_down

    _Fns = (_Linear, _MLPGelu, _MLPSwiGLU)
    return _Fns


# ---------------------------------------------------------------- plans for the C++ autograd nodes
_PLANS: dict = {}


def _prod(a_km: bool, b_kn: bool, M: int, N: int, K: int, epi: int = EPI_NONE, can_split: bool = True) -> list:
    """[library?, tile, splits] — exactly what ``matmul`` picks for this product."""
    t, s = config(a_km, b_kn, M, N, K, can_split=can_split, epi=epi)
    return [1 if prefer_library(a_km, b_kn, M, N, K, epi) else 0, t, s]


def _pair_plan(M: int, N: int, K: int, epi1: int = EPI_NONE) -> int:
    """Schedule (S | wfirst << 4) of the grouped backward launch for dy [M, N], W [N, K]
    (``backward_pair``), or -1 when the grouped launch is off."""
    if not PAIR_BWD:
        return -1
    tile = 128 if M % 128 == 0 and N % 128 == 0 and K % 128 == 0 else 64
    return pair_schedule(M, N, K, tile, epi1)


def native_plan(kind: str, M: int, H: int, I: int, bias1: bool = False, bias2: bool = False) -> list:
    """The int plan of ``torch.ops.nbd.{linear,mlp_gelu,mlp_swiglu}_ag`` (layout: autograd.hip),
    cached per shape.  ``linear``: x [M, I] -> [M, H] (W [H, I]); MLPs: x [M, H], hidden I."""
    key = (kind, M, H, I, bias1, bias2)
    p = _PLANS.get(key)
    if p is not None:
        return p
    R = EPI_ROWSUM
    if kind == "linear":
        N, K = H, I
        p = (_prod(False, False, M, N, K, can_split=not bias1) + _prod(False, True, M, K, N)
             + _prod(True, True, N, K, M, R if bias1 else EPI_NONE) + [_pair_plan(M, N, K)])
    elif kind == "mlp_gelu":
        p = (_prod(False, False, M, I, H, EPI_GELU, can_split=False) + _prod(False, False, M, H, I, can_split=not bias2)
             + _prod(False, True, M, I, H, EPI_DGELU, can_split=False) + _prod(True, True, H, I, M, R if bias2 else EPI_NONE)
             + _prod(False, True, M, H, I) + _prod(True, True, I, H, M, R if bias1 else EPI_NONE)
             + [_pair_plan(M, H, I, EPI_DGELU), _pair_plan(M, I, H)])
    elif kind == "mlp_swiglu":
        p = (_prod(False, False, M, 2 * I, H, EPI_SWIGLU, can_split=False) + _prod(False, False, M, H, I)
             + _prod(False, True, M, I, H, EPI_DSWIGLU, can_split=False) + _prod(True, True, H, I, M)
             + _prod(False, True, M, H, 2 * I) + _prod(True, True, 2 * I, H, M)
             + [_pair_plan(M, H, I, EPI_DSWIGLU), _pair_plan(M, 2 * I, H)])
    else:
        raise ValueError(kind)
    _PLANS[key] = p
    return p


_native_ready = None


def _native(*biases) -> bool:
    global _native_ready
    if not NATIVE_AUTOGRAD:
        return False
    if _native_ready is None:
        _require()  # a GPU path without its extension fails loudly
        _native_ready = True
    import torch

    return all(b is None or b.dtype == torch.bfloat16 for b in biases)


def _fast(x, *ws) -> bool:
    import torch

    if not (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and not torch.is_autocast_enabled()):
        return False
    if (x.numel() // x.shape[-1]) % 64:
        return False
    return all(w.dtype == torch.bfloat16 and w.shape[-1] % 64 == 0 and w.shape[0] % 64 == 0 for w in ws)


# rows (tokens) not a multiple of 64: pad them with zero rows for the HIP kernels instead of
# falling back to the library (NBD_GEMM_PAD_ROWS=0: the library for such shapes)
PAD_ROWS = os.environ.get("NBD_GEMM_PAD_ROWS", "1") != "0"


def _pad_rows(x, *ws):
    """(x as [M64, K] with zero rows appended, M) when only the row count keeps ``x`` off the HIP
    kernels (the weights' dims are multiples of 64), else None.  Autograd sees a pad and a slice:
    the padded rows' gradients are dropped, and zero rows add nothing to a weight gradient."""
    import torch

    if not (PAD_ROWS and ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and not torch.is_autocast_enabled()
            and x.dim() >= 1 and x.shape[-1] % 64 == 0):
        return None
    M = x.numel() // max(1, x.shape[-1])
    if M == 0 or M % 64 == 0:
        return None
    if not all(w.dtype == torch.bfloat16 and w.shape[-1] % 64 == 0 and w.shape[0] % 64 == 0 for w in ws):
        return None
    import torch.nn.functional as F

    # to a multiple of 256, not 64: the measured table and the 128-row tiles are for such counts
    # (M = 8100 padded to 8128 ran 10-40 % slower than to 8192: profiles/odd_rows_r6.txt)
    return F.pad(x.reshape(M, x.shape[-1]), (0, 0, 0, (-M) % 256)), M


# weight dims (N outputs, K inputs) off the 64-grid: zero-pad the weight (N to 128, K to 64) and
# the input's columns onto the HIP kernels (NBD_GEMM_PAD_DIMS=0: the library; faster than
# hipBLASLt on the measured odd shapes despite the weight copy per call — FINDINGS §36)
PAD_DIMS = os.environ.get("NBD_GEMM_PAD_DIMS", "1") != "0"


def _pad_dims(x, weight, bias):
    """(x, weight, bias) zero-padded so that N and K are multiples of 64, or None."""
    import torch

    if not (PAD_DIMS and ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and weight.dim() == 2 and not torch.is_autocast_enabled()
            and (bias is None or bias.dtype == torch.bfloat16)):
        return None
    N, K = weight.shape
    if N <= 64 or (N % 64 == 0 and K % 64 == 0):  # (heads: tiny-linear kernels; aligned: as is)
        return None
    # N to a multiple of 128 (128-wide tiles; 64 left N = 3000 on 64-wide tiles, slower than the library)
    pn, pk = (-N) % 128, (-K) % 64
    if pn == 0 and pk == 0:
        return None
    import torch.nn.functional as F

    return (F.pad(x, (0, pk)) if pk else x, F.pad(weight, (0, pk, 0, pn)),
            F.pad(bias, (0, pn)) if (bias is not None and pn) else bias)


def gemm_linear(x, weight, bias=None):
    """``F.linear`` on the HIP MFMA GEMM (bf16; weight dims multiples of 64 — or padded with
    NBD_GEMM_PAD_DIMS=1 —, a row count that is not is padded); PyTorch otherwise."""
    pd = _pad_dims(x, weight, bias)
    if pd is not None:
        y = gemm_linear(*pd)
        return y[..., :weight.shape[0]] if y.shape[-1] != weight.shape[0] else y
    pr = _pad_rows(x, weight)
    if pr is not None:
        return gemm_linear(pr[0], weight, bias)[:pr[1]].reshape(*x.shape[:-1], weight.shape[0])
    if _fast(x, weight):
        if _native(bias):
            import torch

            plan = native_plan("linear", x.numel() // x.shape[-1], weight.shape[0], weight.shape[1], bias is not None)
            return torch.ops.nbd.linear_ag(x, weight, bias, plan)
        return _fns()[0].apply(x, weight, bias)
    import torch.nn.functional as F

    return F.linear(x, weight, bias)


def mlp_gelu(x, w1, b1, w2, b2):
    """``F.linear(gelu_tanh(F.linear(x, w1, b1)), w2, b2)`` with the activation fused into the GEMMs."""
    pr = _pad_rows(x, w1, w2)
    if pr is not None:
        return mlp_gelu(pr[0], w1, b1, w2, b2)[:pr[1]].reshape(*x.shape[:-1], w2.shape[0])
    if _fast(x, w1, w2):
        if _native(b1, b2):
            import torch

            plan = native_plan("mlp_gelu", x.numel() // x.shape[-1], w1.shape[1], w1.shape[0], b1 is not None, b2 is not None)
            return torch.ops.nbd.mlp_gelu_ag(x, w1, b1, w2, b2, plan)
        return _fns()[1].apply(x, w1, b1, w2, b2)
    import torch.nn.functional as F

    return F.linear(F.gelu(F.linear(x, w1, b1), approximate="tanh"), w2, b2)


def mlp_swiglu(x, w_gu, w_down):
    """Llama MLP ``down(silu(g)·u)`` with ``[g|u] = F.linear(x, w_gu)`` (``w_gu`` = [gate; up],
    [2I, H]) — SwiGLU and its backward fused into the GEMM epilogues on the GPU path."""
    pr = _pad_rows(x, w_gu, w_down) if FUSED_SWIGLU else None
    if pr is not None:
        return mlp_swiglu(pr[0], w_gu, w_down)[:pr[1]].reshape(*x.shape[:-1], w_down.shape[0])
    if FUSED_SWIGLU and _fast(x, w_gu, w_down):
        if _native():
            import torch

            plan = native_plan("mlp_swiglu", x.numel() // x.shape[-1], w_gu.shape[1], w_down.shape[1])
            return torch.ops.nbd.mlp_swiglu_ag(x, w_gu, w_down, plan)
        return _fns()[2].apply(x, w_gu, w_down)
    if not FUSED_SWIGLU:
        return gemm_linear(_swiglu(gemm_linear(x, w_gu)), w_down)
    import torch.nn.functional as F

    return F.linear(_swiglu(F.linear(x, w_gu)), w_down)


def _swiglu(gu):
    from .llama import swiglu

    return swiglu(gu)


# plan for the C++ Linear node's library path (fp32 / fp16 weights): every product on hipBLASLt,
# no grouped backward launch (the node ignores tiles and splits there)
_LIB_PLAN = [1, 0, 1, 1, 0, 1, 1, 0, 1, -1]


def native_available_or_raise() -> None:
    """The C++ autograd nodes need the extension: fail loudly on a GPU box without it."""
    _require()


def linear_any(x, weight, bias=None):
    """``F.linear`` through the C++ Linear autograd node for any GPU dtype: bf16 with 64-granular
    dims runs the HIP MFMA GEMMs (``gemm_linear``), everything else the library GEMMs.  Either way
    the weight / bias gradients go to their registered DDP bucket slices (``ops.graddst``) — this
    is the forward ``parallel.DistributedDataParallel(fused_linear=True)`` gives ``nn.Linear``."""
    import torch

    if ((_fast(x, weight) or _pad_rows(x, weight) is not None or _pad_dims(x, weight, bias) is not None)
            and _native(bias)):
        return gemm_linear(x, weight, bias)  # (row counts / weight dims off the 64-grid are padded there)
    # bf16 heads with a tiny output dimension (classifiers: N <= 64): the tiny-linear kernels
    from .tiny import linear_tiny, supported as _tiny_ok

    if _tiny_ok(x, weight, bias):
        return linear_tiny(x, weight, bias)
    # (other bf16 shapes the HIP GEMMs cannot tile stay on F.linear: the node's bias-gradient row
    # sums need the HIP kernel)
    if (x.is_cuda and x.dtype == weight.dtype and x.dtype in (torch.float32, torch.float16)
            and (bias is None or bias.dtype == weight.dtype) and NATIVE_AUTOGRAD):
        _require()
        return torch.ops.nbd.linear_ag(x, weight, bias, _LIB_PLAN)
    import torch.nn.functional as F

    return F.linear(x, weight, bias)


# fused Llama decoder block (csrc/kernels/autograd.hip LlamaBlockFn): NBD_FUSED_BLOCK=0 runs the
# per-op nodes instead (same kernels, same results)
FUSED_BLOCK = os.environ.get("NBD_FUSED_BLOCK", "1") != "0"
_BLOCK_PLANS: dict = {}


def llama_block(x, h, w_qkv, b_qkv, w_o, b_o, w_post, w_gu, w_down, w_next, n_head: int, n_kv: int, eps: float,
                cos, sin, graphs: int = -1, owner: int = 0):
    """One pre-norm Llama decoder block as ONE autograd node: ``x1 = x + o_proj(attn(qkv(h)))``,
    ``h1 = rms(x1)·γ_post``, ``x2 = x1 + down(swiglu(gate_up(h1)))``, returns ``(x2, rms(x2)·γ_next)``
    — the per-op path's kernels in the same order, one Python call and one node instead of six and
    five (the eager SmolLM2 step is host-bound).  None when the block does not fit the fused path
    (the caller then runs the ops one by one).  ``graphs``: per-block HIP graph mode for this call
    (0 / 1 / 2, see ``block_graphs``; -1 = the process setting); ``owner``: the calling model's id,
    kept with its block graphs so that ``block_graphs_reset(owner)`` drops that model's only."""
    import torch

    if not (FUSED_BLOCK and FUSED_SWIGLU and NATIVE_AUTOGRAD and _fast(h, w_qkv, w_o, w_gu, w_down)
            and x.dtype == h.dtype and x.shape == h.shape and _native(b_qkv, b_o)):
        return None
    B, T, C = h.shape
    D = w_qkv.shape[0] // (n_head + 2 * n_kv)
    if not (D == 64 and T % 128 == 0 and n_head % n_kv == 0 and w_post.dtype == w_next.dtype == h.dtype
            and C % 8 == 0 and C <= 2048 and h.is_contiguous() and x.is_contiguous()):
        return None
    M = B * T
    key = (M, C, w_qkv.shape[0], w_o.shape[1], w_down.shape[1], b_qkv is not None, b_o is not None)
    plans = _BLOCK_PLANS.get(key)
    if plans is None:
        plans = (native_plan("linear", M, w_qkv.shape[0], C, b_qkv is not None),
                 native_plan("linear", M, C, w_o.shape[1], b_o is not None),
                 native_plan("mlp_swiglu", M, C, w_down.shape[1]))
        _BLOCK_PLANS[key] = plans
    return torch.ops.nbd.llama_block_ag(x, h, w_qkv, b_qkv, w_o, b_o, w_post, w_gu, w_down, w_next, plans[0],
                                        plans[1], plans[2], int(n_head), int(n_kv), D ** -0.5, float(eps), cos, sin,
                                        int(graphs), int(owner))


def block_graphs(enable=None) -> int:
    """Per-block HIP graphs for the EAGER Llama step (``csrc/kernels/autograd.hip`` namespace
    ``bg``; off by default, ``NBD_BLOCK_GRAPHS=1`` turns it on at start).  Each fused decoder
    block's forward is captured once per (block, shape) after two eager calls and replayed from
    then on — one graph launch for its seven kernels.  The block's outputs then live in static
    memory: they keep this pass's values until that block's next forward, so a caller keeping
    block outputs across steps must clone them.  ``enable=2`` (``NBD_BLOCK_GRAPHS=2``) graphs the
    backward too where every weight gradient goes to a DDP bucket slice.  In mode 1 a run of
    blocks that replays steadily is chained into one stack graph (one launch per forward;
    ``NBD_BLOCK_STACKS=0``: per-block graphs only).  Bit-identical to the eager block.  ``enable=None`` queries; True = 1; returns the previous mode (0, 1, 2)."""
    import torch

    _require()
    return int(torch.ops.nbd.llama_block_graphs(-1 if enable is None else int(enable)))


def block_graphs_reset(owner=None) -> None:
    """Drop captured block graphs: every one, or (``owner``) those made by one model — what a
    LlamaModel being garbage-collected does, so a throwaway model never costs a live one its
    graphs."""
    from . import _lib

    if _lib._loaded:
        import torch

        if owner is None:
            torch.ops.nbd.llama_block_graphs_reset()
        else:
            torch.ops.nbd.llama_block_graphs_reset_owner(int(owner))


def block_graphs_memory(device=None) -> dict:
    """Device memory the block graphs hold: the caching allocator's segments in their private
    pools (static activations, inputs and outputs kept between steps).  {"graphs": n,
    "reserved_bytes": ..., "allocated_bytes": ...}; zeros when none are live."""
    from . import _lib

    out = {"graphs": 0, "reserved_bytes": 0, "allocated_bytes": 0}
    if not _lib._loaded:
        return out
    import torch

    ids = list(torch.ops.nbd.llama_block_graphs_pools())
    pools = {(ids[i], ids[i + 1]) for i in range(0, len(ids), 2)}
    out["graphs"] = len(ids) // 2
    if not pools:
        return out
    dev = torch.cuda.current_device() if device is None else torch.device(device).index
    for seg in torch.cuda.memory_snapshot():
        if seg.get("device") != dev or tuple(seg.get("segment_pool_id", (0, 0))) not in pools:
            continue
        out["reserved_bytes"] += int(seg.get("total_size", 0))
        out["allocated_bytes"] += int(seg.get("allocated_size", 0))
    return out


def cast_buffers_memory() -> dict:
    """The kept compute-dtype casts of ``models.native()``'s fp32 master weights and their gradient
    buffers (autograd.hip ``castbuf``): memory the framework holds between steps."""
    import torch

    _require()
    n, cb, gb = torch.ops.nbd.cast_buffers_memory()
    return {"groups": n, "cast_bytes": cb, "grad_bytes": gb}


def block_graphs_stats() -> dict:
    """Counters of the per-block graphs: forward captures, replays, eager calls in graph mode, live
    graphs; backward captures, replays (captures included) and eager backwards of graphed forwards."""
    import torch

    _require()
    c, r, e, n, bc, br, be, sc, sr, ss, sd = torch.ops.nbd.llama_block_graphs_stats()
    return {"captures": c, "replays": r, "eager": e, "live": n, "bwd_captures": bc, "bwd_replays": br,
            "bwd_eager": be, "stack_captures": sc, "stack_replays": sr, "stack_served": ss, "stacks_dropped": sd}
