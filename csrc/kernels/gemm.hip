// gemm.hip — bf16 GEMM on the gfx950 matrix cores with fused epilogues, for the Linear layers of
// the GPT-2 / Llama workloads (forward, input-gradient and weight-gradient products).
//
//   C[M,N] = Σ_k A[m,k]·B[k,n]   (fp32 accumulation, v_mfma_f32_16x16x32_bf16)
//
// Operand storage (row-major, unit stride innermost; `ld*` = row stride in elements):
//   A: [M][K] ("row image": K-contiguous)    or  [K][M] (a_km: "transposed image")
//   B: [N][K] ("row image")                  or  [K][N] (b_kn: "transposed image")
// so the three products of a Linear y = x·Wᵀ are all direct, with no transposed copies:
//   forward  y  = x·Wᵀ   A = x  [M][K],  B = W  [N][K]            (row, row)
//   dgrad    dx = dy·W   A = dy [M][N],  B = W  [N][K] as [K][N]  (row, tr)
//   wgrad    dW = dyᵀ·x  A = dy as [K][M], B = x as [K][N]        (tr, tr)
//
// Structure (cdna_hip_programming.md §5 "minimum 2-phase" + T1 + T2 + T10):
//   * workgroup = 4 waves (2×2), tile BM×BN×64, each wave a (BM/2)×(BN/2) sub-tile of 16×16 MFMA
//     fragments; two LDS buffers: the next K-tile streams global→LDS with 16-byte
//     `global_load_lds_dwordx4` (no VGPR round trip) while the current one feeds the MFMAs.
//   * LDS images are lane-linear (the DMA writes base + 16·lane), so the bank-conflict swizzles
//     are applied to the per-lane *global source* address and undone on the LDS read:
//       row image  [R][64] (128-B rows): 16-B chunk c of row r lives at chunk c ^ ((r>>1)&7) —
//                  every 16-lane ds_read_b128 group of a 16x16x32 fragment hits 16 distinct slots;
//       tr image   [64][R]: 8-B slot s of k-row k lives at s ^ h(k), h chosen so the 32 lanes of
//                  each ds_read_b64_tr_b16 half (k rows {q, 8+q}, 4 column blocks) are distinct.
//     The transposed image is read with ds_read_b64_tr_b16 (hardware transpose, T10): that is
//     what lets dgrad / wgrad consume W, dy and x in their natural storage.
//   * The MFMA is fed (B-fragment, A-fragment), i.e. it computes Cᵀ: each lane then holds 4
//     consecutive output columns of one row → 8-byte stores, and bias / GELU operands are
//     loaded 4-wide in the epilogue.
//   * blockIdx → tile: bijective XCD remap (T1) then 8-row groups sweeping the column tiles, so
//     the blocks sharing an A row panel run on the same XCD's L2.
//   * split-K (grid.y) for long-K products (weight gradients, K = tokens): fp32 slabs, summed by
//     reduce_kernel in a fixed order.
//   * epilogue staged through LDS: each thread stores 8 consecutive bf16 of a row (16 B).
// Epilogues: + bias[n]; GELU-tanh (stores the pre-activation for the backward too);
// dGELU (multiplies by gelu'(pre-activation) — the MLP's activation backward fused into the
// dgrad of its output projection); SwiGLU (Llama: the gate|up projection's workgroup takes
// matching gate and up columns, writes silu(g)·u and the pre-activations) and its backward
// (the down projection's dgrad writes d[g|u] from dact and the saved pre-activations).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "gemm_common.h"
#include "graddst.h"

namespace nbd {
namespace gemm {

constexpr int NT = 256;

// STAGES >= 100: the ping-pong schedule (gemm_body, below) with a ring of STAGES - 100 buffers
constexpr int ring_of(int stages) { return stages >= 100 ? stages - 100 : stages; }

template <int BM, int BN, int STAGES, int KS = 1>
struct Smem {
  static constexpr int BUF = (BM + BN) * BK * 2;      // one A + B K-tile pair
  static constexpr int LDC = BN + 4;                  // fp32 C-tile row stride (+16 B: rows hit distinct banks)
  static constexpr int CT = BM * LDC * 4 + BM * 4;    // fp32 C tile (+ row-sum scratch), reuses the operand buffers
  static constexpr int PIPE = KS * ring_of(STAGES) * BUF;  // one pipeline per K-split group
  static constexpr int BYTES = PIPE > CT ? PIPE : CT;
};

// Wait until at most N of this wave's vector-memory ops (here: glds) are outstanding, retire
// its LDS reads, then a raw workgroup barrier — no vmcnt(0) drain, so a prefetched K-tile stays
// in flight across it (cdna_hip_programming.md §5 "Pipelining across barriers").
template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// STAGES = 2: load tile t+1 while computing t, drain + barrier per tile (fits 2 workgroups/CU at
// 128x128).  STAGES = 3: tile t+2 is issued while t is computed and stays in flight across the
// barrier (counted vmcnt) — the latency-bound regime of few, long-K tiles (weight gradients,
// small token counts) where one workgroup per CU cannot hide a drained pipeline.
// W = waves per K-group: 4 (2x2, each wave (BM/2)x(BN/2)) or 8 (2x4, each (BM/2)x(BN/4): twice
// the waves per SIMD to hide the barrier / DMA latency, at more LDS reads per MFMA).
// KS = K-split groups inside the workgroup: group g runs its own pipeline over K-tiles g, g+KS, …
// and the groups' fp32 tiles are summed in LDS before the epilogue — twice the independent work
// per CU for small, latency-bound products (few tiles, one workgroup per CU), with no extra
// global traffic or second kernel (unlike split-K across workgroups).
// The kernel body as a device function: `bx` = tile index (before the XCD remap), `by` = split
// index, `S` = number of splits, `smem_all` = the launch's single LDS object.  gemm_kernel runs one
// product per launch; pair_kernel (below) runs two independent products in one grid.
template <int BM, int BN, bool A_KM, bool B_KN, int EPI, int STAGES, int W, int KS>
__device__ __forceinline__ void gemm_body(const Args& p, int bx, int by, int S, uint8_t* smem_all) {
  constexpr int NTW = 64 * W * KS, WM = 2, WN = W / 2;
  constexpr int FM = BM / (16 * WM), FN = BN / (16 * WN);  // 16-wide fragments per wave along m / n
  using SM = Smem<BM, BN, STAGES, KS>;
  constexpr int A_BYTES = BM * BK * 2, BUF = SM::BUF, LDC = SM::LDC;
  constexpr int NPT = (BM + BN) / (8 * W);  // glds per thread per K-tile

  const int lane = threadIdx.x & 63, wave_all = threadIdx.x >> 6;
  const int kg = wave_all / W, wave = wave_all % W;  // K-split group, wave within the group
  const int wm = wave / WN, wn = wave % WN;
  uint8_t* smem = smem_all + kg * (ring_of(STAGES) * BUF);  // this group's pipeline buffers

  int tm, tn;
  tile_coords<8>(p.tiles_m, p.tiles_n, tm, tn, bx);
  const int m0 = tm * BM, n0 = tn * BN;

  // split-K: `by` selects the K range
  const int64_t kz = (int64_t)by * p.K;
  const uint16_t* A = p.a + (A_KM ? kz * p.lda : kz);
  const uint16_t* B = p.b + (B_KN ? kz * p.ldb : kz);

  f4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // EPI_ROWSUM: the waves of the first column of tiles (tn == 0, wn == 0) own the row sums
  constexpr bool ROWSUM = EPI == EPI_ROWSUM;
  const bool do_rs = ROWSUM && tn == 0 && wn == 0;  // uniform per wave
  f4 accb[FM];
#pragma unroll
  for (int j = 0; j < FM; ++j) accb[j] = f4{0.f, 0.f, 0.f, 0.f};
  s8v ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;  // bf16 1.0

  const int nk = p.K / BK / KS;  // K-tiles of this group: t_global = t * KS + kg
  auto compute = [&](const uint8_t* cur) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s8v af[FM], bf[FN];
#pragma unroll
      for (int j = 0; j < FM; ++j) af[j] = frag<BM, A_KM>(cur, wm * (BM / WM) + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < FN; ++i) bf[i] = frag<BN, B_KN>(cur + A_BYTES, wn * (BN / WN) + 16 * i, kk, lane);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[i], af[j], acc[i][j], 0, 0, 0);
      if constexpr (ROWSUM) {
        if (do_rs) {  // D[i][m] = Σ_k 1·A[m][k], identical in every row i
#pragma unroll
          for (int j = 0; j < FM; ++j) accb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[j], accb[j], 0, 0, 0);
        }
      }
    }
  };
  // DMA addressing: per-lane 32-bit offsets computed once, a scalar base per K-step
  const Pieces<BM, A_KM, W> pa(p.lda, wave, lane);
  const Pieces<BN, B_KN, W> pb(p.ldb, wave, lane, EPI == EPI_SWIGLU ? (int64_t)(p.N / 2) : 0);
  auto stage_tile = [&](int t, uint8_t* buf) {
    pa.stage(A, p.lda, m0, (t * KS + kg) * BK, buf, wave);
    pb.stage(B, p.ldb, EPI == EPI_SWIGLU ? n0 / 2 : n0, (t * KS + kg) * BK, buf + A_BYTES, wave);
  };

  if constexpr (STAGES >= 100) {
    // Ping-pong (cdna_hip_programming.md §5 256² template's staggered groups, MI355X_MICROARCH.md
    // "Two waves per SIMD"), one 512-thread workgroup per CU: waves 0-3 (rows 0-63 of the tile)
    // and 4-7 (rows 64-127) share the SIMDs pairwise (w, w+4) and run one barrier apart, so on
    // every SIMD one wave issues its 16 MFMAs while its partner reads the next K-tile's
    // fragments and issues its share of a DMA.  Per group and K-tile t:
    //   R(t):  fragments of tile t -> registers; DMA of tile t+2 into the buffer tile t-1 used;
    //          counted vmcnt retires tile t+1 (tile t+2 stays in flight); lgkmcnt(0)
    //   s_barrier (A_t) — MFMA(t) at priority 1 — s_barrier (B_t)
    // The lagging group's A_t is the leading group's B_t.  RAW: a wave's wait for tile t+1 comes
    // before its A_t, and both groups read tile t+1 only after a barrier every wave passed after
    // that wait.  WAR: tile t+2's DMA (issued in R(t), after the issuer's B_{t-1}) overwrites
    // tile t-1, whose reads both groups retired before barriers at or before that B_{t-1}.
    constexpr int S = ring_of(STAGES);
    static_assert(S == 3 && W == 8 && KS == 1, "ping-pong: 3-buffer ring, 8 waves, no K-split groups");
    const bool lag = __builtin_amdgcn_readfirstlane(threadIdx.x) >= NTW / 2;
    stage_tile(0, smem);
    if (nk > 1) {
      stage_tile(1, smem + BUF);
      wait_barrier<NPT>();  // tile 0 landed everywhere
    } else {
      wait_barrier<0>();
    }
    if (lag) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    s8v af[2][FM], bf[2][FN];
    auto pp_step = [&](int t, auto cur_c) {
      constexpr int CUR = decltype(cur_c)::value, NXT2 = (CUR + 2) % S;
      const uint8_t* cur = smem + CUR * BUF;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int j = 0; j < FM; ++j) af[kk][j] = frag<BM, A_KM>(cur, wm * (BM / WM) + 16 * j, kk, lane);
#pragma unroll
        for (int i = 0; i < FN; ++i) bf[kk][i] = frag<BN, B_KN>(cur + A_BYTES, wn * (BN / WN) + 16 * i, kk, lane);
      }
      if (t + 2 < nk) {
        stage_tile(t + 2, smem + NXT2 * BUF);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPT) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[kk][i], af[kk][j], acc[i][j], 0, 0, 0);
        if constexpr (ROWSUM) {
          if (do_rs) {
#pragma unroll
            for (int j = 0; j < FM; ++j)
              accb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[kk][j], accb[j], 0, 0, 0);
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    };
    for (int t = 0; t < nk; t += S) {
      pp_step(t, std::integral_constant<int, 0>{});
      if (t + 1 < nk) pp_step(t + 1, std::integral_constant<int, 1>{});
      if (t + 2 < nk) pp_step(t + 2, std::integral_constant<int, 2>{});
    }
    if (!lag) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else if constexpr (STAGES == 2) {
    stage_tile(0, smem);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      uint8_t* cur = smem + (t & 1) * BUF;
      if (t + 1 < nk) stage_tile(t + 1, smem + ((t + 1) & 1) * BUF);
      compute(cur);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // S-stage ring (S = STAGES >= 3): buffer t % S holds tile t; tiles t+1 .. t+S-2 are in flight
    // while tile t is computed, and tile t+S-1 is issued into the buffer tile t-1 occupied (every
    // wave finished reading it before step t-1's barrier).  The barrier that ends step t waits
    // for tile t+1 only (counted vmcnt: the younger tiles' NPT loads each stay in flight).  Deep
    // rings are for latency-bound products: with K ≤ (S-1)·64 every K-tile is requested at once.
    constexpr int S = STAGES;
    // wait until at most n younger tiles are outstanding (n ≤ S-2, runtime only at the tail)
    static_assert(S <= 9 && (S - 2) * NPT <= 63, "vmcnt range");
    auto wait_tiles = [&](int n) {
      switch (n) {
        case 0: wait_barrier<0>(); break;
        case 1: wait_barrier<NPT>(); break;
        case 2: wait_barrier<2 * NPT>(); break;
        case 3: wait_barrier<3 * NPT>(); break;
        case 4: wait_barrier<4 * NPT>(); break;
        case 5: wait_barrier<5 * NPT>(); break;
        case 6: wait_barrier<6 * NPT>(); break;
        default: wait_barrier<(S - 2) * NPT>(); break;
      }
    };
    const int pro = nk < S - 1 ? nk : S - 1;
    for (int t = 0; t < pro; ++t) stage_tile(t, smem + t * BUF);
    wait_tiles(pro - 1);
    // unrolled by S so every buffer offset is a compile-time constant: the compiler can then
    // prove the in-flight DMA and this step's ds_reads disjoint and does not drain vmcnt(0)
    // before the reads (it did with a rotating runtime index)
    auto step = [&](int t, auto cur_c) {
      constexpr int CUR = decltype(cur_c)::value, PREV = (CUR + S - 1) % S;
      const bool issue = t + S - 1 < nk;
      if (issue) stage_tile(t + S - 1, smem + PREV * BUF);
      compute(smem + CUR * BUF);
      // tiles t+2 .. min(t+S-1, nk-1) may stay outstanding
      const int last = issue ? t + S - 1 : nk - 1;
      wait_tiles(last - (t + 1) > 0 ? last - (t + 1) : 0);
    };
#define NBD_STEP(J) \
  if constexpr (J < S) { if (t + J < nk) step(t + J, std::integral_constant<int, J>{}); }
    for (int t = 0; t < nk; t += S) {
      NBD_STEP(0) NBD_STEP(1) NBD_STEP(2) NBD_STEP(3) NBD_STEP(4) NBD_STEP(5) NBD_STEP(6) NBD_STEP(7) NBD_STEP(8)
    }
#undef NBD_STEP
  }

  // ---- epilogue ------------------------------------------------------------------------------
  constexpr int CPR = BN / 8;  // 8-column chunks per row
  if constexpr (EPI == EPI_NONE && KS == 1) {
    // A plain (+ bias) bf16 result with nothing to add to it: bias added and rounded to bf16 in
    // registers (the one rounding the fp32 path does too), the bf16 tile staged through LDS —
    // half the bytes of the fp32 image: 8-B ds_write_b64 at ≈85 B/clk instead of 64 KiB of
    // ds_write_b128 at ≈79 B/clk per 128x128 tile (MI355X_MICROARCH.md LDS table).
    if (S == 1 && !(p.accum & 1)) {
      constexpr int LDB = BN + 8;  // bf16 row stride: 16 rows x 8 B of one write hit distinct banks
      uint16_t* cb = reinterpret_cast<uint16_t*>(smem_all);
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int n = wn * (BN / WN) + 16 * i + 4 * (lane >> 4);
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if (p.bias != nullptr) {
          const uint2 w = *reinterpret_cast<const uint2*>(p.bias + n0 + n);
          bv[0] = __uint_as_float(w.x << 16); bv[1] = __uint_as_float(w.x & 0xffff0000u);
          bv[2] = __uint_as_float(w.y << 16); bv[3] = __uint_as_float(w.y & 0xffff0000u);
        }
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          const int m = wm * (BM / WM) + 16 * j + (lane & 15);
          const f4 v = acc[i][j];
          uint2 w;
          w.x = pack2_bf16(v[0] + bv[0], v[1] + bv[1]);
          w.y = pack2_bf16(v[2] + bv[2], v[3] + bv[3]);
          *reinterpret_cast<uint2*>(cb + m * LDB + n) = w;
        }
      }
      __syncthreads();
      for (int c = threadIdx.x; c < BM * CPR; c += NTW) {
        const int r = c / CPR, cn = (c % CPR) * 8;
        const uint4 v = *reinterpret_cast<const uint4*>(cb + r * LDB + cn);
        *reinterpret_cast<uint4*>(p.c + (int64_t)(m0 + r) * p.ldc + n0 + cn) = v;
      }
      return;
    }
  }
  // The fp32 tile goes through LDS (the loop's last barrier retired every operand read) so the
  // global traffic is row-contiguous: each thread then owns 8 consecutive columns of a row —
  // 16-B bf16 stores / aux loads, 32-B fp32 slab stores.  acc[i][j] element e = C[m][n] with
  // m = .. + (lane&15), n = .. + 4(lane>>4) + e.
  float* ct = reinterpret_cast<float*>(smem_all);
  float* rsb = ct + BM * LDC;  // K-split row-sum scratch
  auto cslot = [&](int i, int j) -> f4* {
    return reinterpret_cast<f4*>(ct + (wm * (BM / WM) + 16 * j + (lane & 15)) * LDC + wn * (BN / WN) + 16 * i +
                                 4 * (lane >> 4));
  };
  if (kg == 0) {
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) *cslot(i, j) = acc[i][j];
  } else if constexpr (ROWSUM) {
    if (do_rs && lane < 16)
#pragma unroll
      for (int j = 0; j < FM; ++j) rsb[wm * (BM / WM) + 16 * j + lane] = accb[j][0];
  }
  __syncthreads();
  if constexpr (KS > 1) {  // the second group adds its partial tile (and row sums)
    if (kg == 1) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) {
          f4 v = *cslot(i, j);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += acc[i][j][e];
          *cslot(i, j) = v;
        }
    } else if constexpr (ROWSUM) {
      if (do_rs && lane < 16)
#pragma unroll
        for (int j = 0; j < FM; ++j) accb[j][0] += rsb[wm * (BM / WM) + 16 * j + lane];
    }
    __syncthreads();
  }

  if constexpr (ROWSUM) {
    // lanes 0..15 hold row m = .. + lane in element 0 (all four elements are equal)
    if (do_rs && kg == 0 && lane < 16) {
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = m0 + wm * (BM / WM) + 16 * j + lane;
        if (S > 1)
          p.ws[(int64_t)S * p.M * p.ldc + (int64_t)by * p.M + m] = accb[j][0];
        else
          p.aux_out[m] = f32_to_bf16((p.accum & 2) ? accb[j][0] + bf16_to_f32(p.aux_out[m]) : accb[j][0]);
      }
    }
  }
  if (S > 1) {
    // split-K: this split's fp32 slab; reduce_kernel sums the slabs.  (A last-arriver in-kernel
    // reduction measured slower here: its serial read of S-1 slabs of 16-64 KiB per tile costs
    // more than the extra launch — profiles/gemm_bench_r1.txt.)
    float* slab = p.ws + (int64_t)by * p.M * p.ldc;
    for (int c = threadIdx.x; c < BM * CPR; c += NTW) {
      const int r = c / CPR, cn = (c % CPR) * 8;
      float* dst = slab + (int64_t)(m0 + r) * p.ldc + n0 + cn;
      *reinterpret_cast<f4*>(dst) = *reinterpret_cast<const f4*>(ct + r * LDC + cn);
      *reinterpret_cast<f4*>(dst + 4) = *reinterpret_cast<const f4*>(ct + r * LDC + cn + 4);
    }
    return;
  }

  if constexpr (EPI == EPI_SWIGLU) {
    // tile columns [0, BN/2) = gate features n0/2.., [BN/2, BN) = up features of the same indices
    constexpr int HPR = BN / 16;  // 8-column chunks per half row
    const int I = p.N / 2;
    for (int c = threadIdx.x; c < BM * HPR; c += NTW) {
      const int r = c / HPR, cn = (c % HPR) * 8;
      float g[8], u[8];
      {
        const f4 g0 = *reinterpret_cast<const f4*>(ct + r * LDC + cn);
        const f4 g1 = *reinterpret_cast<const f4*>(ct + r * LDC + cn + 4);
        const f4 u0 = *reinterpret_cast<const f4*>(ct + r * LDC + BN / 2 + cn);
        const f4 u1 = *reinterpret_cast<const f4*>(ct + r * LDC + BN / 2 + cn + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          g[e] = g0[e]; g[e + 4] = g1[e]; u[e] = u0[e]; u[e + 4] = u1[e];
        }
      }
      const int64_t m = m0 + r, j = n0 / 2 + cn;
      store8_nt<bf16_t>(reinterpret_cast<bf16_t*>(p.aux_out) + m * p.N + j, g);
      store8_nt<bf16_t>(reinterpret_cast<bf16_t*>(p.aux_out) + m * p.N + I + j, u);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = g[e] * sigm(g[e]) * u[e];
      store8<bf16_t>(reinterpret_cast<bf16_t*>(p.c) + m * p.ldc + j, g);
    }
    return;
  }
  if constexpr (EPI == EPI_DSWIGLU) {
    // v = dact[m][j]; pre-activations [g|u] and the output d[g|u] are [M][2N]
    for (int c = threadIdx.x; c < BM * CPR; c += NTW) {
      const int r = c / CPR, cn = (c % CPR) * 8;
      float d[8], g[8], u[8];
      {
        const f4 lo = *reinterpret_cast<const f4*>(ct + r * LDC + cn);
        const f4 hi = *reinterpret_cast<const f4*>(ct + r * LDC + cn + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          d[e] = lo[e]; d[e + 4] = hi[e];
        }
      }
      const int64_t off = (int64_t)(m0 + r) * 2 * p.N + n0 + cn;
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(p.aux_in) + off, g);
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(p.aux_in) + off + p.N, u);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float sg = sigm(g[e]);
        const float du = d[e] * g[e] * sg;
        d[e] = d[e] * u[e] * sg * (1.f + g[e] * (1.f - sg));
        u[e] = du;
      }
      store8<bf16_t>(reinterpret_cast<bf16_t*>(p.c) + off, d);
      store8<bf16_t>(reinterpret_cast<bf16_t*>(p.c) + off + p.N, u);
    }
    return;
  }
  for (int c = threadIdx.x; c < BM * CPR; c += NTW) {
    const int r = c / CPR, cn = (c % CPR) * 8;
    float v[8];
    {
      const f4 lo = *reinterpret_cast<const f4*>(ct + r * LDC + cn);
      const f4 hi = *reinterpret_cast<const f4*>(ct + r * LDC + cn + 4);
      v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
      v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    }
    const int64_t off = (int64_t)(m0 + r) * p.ldc + n0 + cn;
    if (EPI != EPI_DGELU && p.bias) {
      float b[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(p.bias) + n0 + cn, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += b[e];
    }
    if constexpr (EPI == EPI_GELU) {
      store8_nt<bf16_t>(reinterpret_cast<bf16_t*>(p.aux_out) + off, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
    } else if constexpr (EPI == EPI_DGELU) {
      float h[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(p.aux_in) + off, h);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= dgelu_tanh(h[e]);
    } else if constexpr (EPI == EPI_ADELTA) {
      // δ of (row, head) from the 8 consecutive lanes holding that row's 64 columns of the head
      // (CPR % 8 == 0 and BM·CPR % NTW == 0: every lane runs every iteration, groups aligned)
      static_assert(CPR % 8 == 0 && (BM * CPR) % NTW == 0, "EPI_ADELTA: whole heads per 8 lanes, no idle lanes");
      float o[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(p.aux_in) + off, o);
      float dsum = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum = fmaf(bf16_to_f32(f32_to_bf16(v[e])), o[e], dsum);
      dsum += __shfl_xor(dsum, 1, 64);
      dsum += __shfl_xor(dsum, 2, 64);
      dsum += __shfl_xor(dsum, 4, 64);
      if ((c & 7) == 0) {
        const int64_t m = m0 + r;
        const int64_t hh = (n0 + cn) / 64, H = p.ldc / 64;
        p.delta[((m / p.dT) * H + hh) * p.dT + (m % p.dT)] = dsum;
      }
    } else {
      if (p.accum & 1) {  // gradient accumulation: c += A·B (one bf16 rounding of the fp32 sum)
        float o[8];
        load8<bf16_t>(reinterpret_cast<const bf16_t*>(p.c) + off, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += o[e];
      }
    }
    store8<bf16_t>(reinterpret_cast<bf16_t*>(p.c) + off, v);
  }
}

// Warm-up block r of P: one 4-byte load per 128-B line of its share of p.pf — the line lands in
// the XCD's L2 and the MALL, which is all the next launch needs (its first round of workgroups
// then hits the MALL instead of waiting on HBM for every K-tile).  Four lines per thread in
// flight per iteration; the values only feed an empty asm, so nothing is stored.
template <int NTH>
__device__ __forceinline__ void warm_lines(const Args& p, int r, int P) {
  const int64_t per = (p.pf_lines + P - 1) / P;
  const int64_t lo = (int64_t)r * per, hi = min(p.pf_lines, lo + per);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p.pf);
  uint32_t x = 0;
  for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += 4 * NTH) {
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + (int64_t)u * NTH;
      v[u] = i < hi ? q[i * 32] : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) x ^= v[u];
  }
  asm volatile("" ::"v"(x));
}

template <int BM, int BN, bool A_KM, bool B_KN, int EPI, int STAGES, int W, int KS>
__global__ __launch_bounds__(64 * W * KS, KS == 1 ? 2 : 1) void gemm_kernel(Args p) {
  // one __shared__ array for everything (a second LDS object de-pipelines the glds loop:
  // cdna_hip_programming.md §5 "Projection GEMM" item 4a)
  __shared__ __attribute__((aligned(1024))) uint8_t smem_all[Smem<BM, BN, STAGES, KS>::BYTES];
  // warm_blocks is a multiple of 8: the tile blocks keep their XCD (block id mod 8)
  const int bx = (int)blockIdx.x - p.warm_blocks;
  if (bx < 0) {
    if (blockIdx.y == 0) warm_lines<64 * W * KS>(p, blockIdx.x, p.warm_blocks);
    return;
  }
  gemm_body<BM, BN, A_KM, B_KN, EPI, STAGES, W, KS>(p, bx, blockIdx.y, gridDim.y, smem_all);
}

// A Linear layer's backward as one launch: blocks [0, nb1) compute the input gradient
// dx = dy·W (dgrad layout, optional GELU′ / SwiGLU′ epilogue), blocks [nb1, …) the weight
// gradient dW = dyᵀ·x (split s2 ways, optional bias-gradient row sums).  The weight-gradient
// products of a GPT-2 block alone have 144-576 work units — too few for 256 CUs at two
// workgroups each — and the two products are independent, so one grid lets them share the chip
// (two streams do too, but a graph with a parallel branch slowed every later eager step:
// docs/FINDINGS.md §12).  Both halves use the same tile / waves / stages, so the workgroups are
// interchangeable (128x128 / 8 waves / 2 stages; 64x64 / 4 waves / 3 stages for 64-granular
// shapes such as SmolLM2's).  nb1 is rounded up to a multiple of 8 so each half's block ids keep
// the XCD mapping.
// `first` = blocks of the half dispatched first (rounded up to a multiple of 8 so each half's
// block ids keep the XCD mapping); wfirst = 1 puts the weight-gradient units first.  The
// dispatcher hands out blocks in id order as slots free up, so the half with the longer units
// goes first (longest-processing-time order): a short-unit half dispatched first leaves the
// long units as a serial tail once it drains (ops/gemm.py pair_plan).
// A split-K reduce carried into a launch (graddst.h defer::take_carry): out[i] (+)= Σ_s ws[s][i]
// over the launch's last `blocks` workgroups — reduce_kernel's sums, in its order.
struct Red {
  const float* ws;
  uint16_t* out;
  uint16_t* rs_out;
  int64_t n8, m8, slab;
  int splits, accum, blocks;
};
constexpr int kRedMax = 4;  // reduces per launch (kernel-argument table)
struct RedTable {
  Red d[kRedMax];
  int n, blocks;  // descriptors, their workgroups in total
};

__device__ __forceinline__ void reduce_body(const Red& r, int blk, int nthreads) {
  for (int64_t i = (int64_t)blk * nthreads + threadIdx.x; i < r.n8 + r.m8; i += (int64_t)r.blocks * nthreads) {
    const bool rs = i >= r.n8;
    const float* src = rs ? r.ws + r.splits * r.slab + 8 * (i - r.n8) : r.ws + 8 * i;
    const int64_t stride = rs ? r.m8 * 8 : r.slab;
    float v[8];
    load8<float>(src, v);
    for (int s = 1; s < r.splits; ++s) {
      float w[8];
      load8<float>(src + s * stride, w);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += w[e];
    }
    bf16_t* dst = reinterpret_cast<bf16_t*>(rs ? r.rs_out : r.out) + 8 * (rs ? i - r.n8 : i);
    if (r.accum & (rs ? 2 : 1)) {
      float o[8];
      load8<bf16_t>(dst, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += o[e];
    }
    store8<bf16_t>(dst, v);
  }
}

template <int BM, int BN, int W, int STAGES, int EPI1, int EPI2>
__global__ __launch_bounds__(64 * W, W == 8 ? 2 : 2) void pair_kernel(Args p1, int t1, int first, Args p2, int t2, int s2,
                                                                      int wfirst, RedTable red) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem_all[Smem<BM, BN, STAGES, 1>::BYTES];
  const int b = (int)blockIdx.x - p1.warm_blocks;  // warm-up blocks first (gemm_kernel)
  if (b < 0) {
    warm_lines<64 * W>(p1, blockIdx.x, p1.warm_blocks);
    return;
  }
  // the carried reduce in the grid's last workgroups: dispatched after every tile, they fill the
  // CUs the tail round leaves idle
  const int nmain = (int)gridDim.x - p1.warm_blocks - red.blocks;
  if (b >= nmain) {
    int r = b - nmain, d = 0;
    while (d + 1 < red.n && r >= red.d[d].blocks) r -= red.d[d++].blocks;  // (block-uniform)
    reduce_body(red.d[d], r, 64 * W);
    return;
  }
  const bool dgrad = wfirst ? b >= first : b < first;
  if (dgrad) {
    const int l = wfirst ? b - first : b;
    if (l >= t1) return;  // padding to the XCD boundary
    gemm_body<BM, BN, false, true, EPI1, STAGES, W, 1>(p1, l, 0, 1, smem_all);
  } else {
    const int l = wfirst ? b : b - first;
    if (l >= t2 * s2) return;
    gemm_body<BM, BN, true, true, EPI2, STAGES, W, 1>(p2, l % t2, l / t2, s2, smem_all);
  }
}

// out[i] = Σ_s ws[s][i] as bf16 (fixed order: deterministic); 8 elements per thread.  With
// rs_out, the EPI_ROWSUM partials ws[S*slab + s*M + m] are summed into rs_out[m] the same way.
__global__ __launch_bounds__(256) void reduce_kernel(const float* __restrict__ ws, int splits, int64_t n8, int64_t slab,
                                                     uint16_t* __restrict__ out, int64_t m8,
                                                     uint16_t* __restrict__ rs_out, int accum) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8 + m8; i += (int64_t)gridDim.x * blockDim.x) {
    const bool rs = i >= n8;
    const float* src = rs ? ws + splits * slab + 8 * (i - n8) : ws + 8 * i;
    const int64_t stride = rs ? m8 * 8 : slab;
    float v[8];
    load8<float>(src, v);
    for (int s = 1; s < splits; ++s) {
      float w[8];
      load8<float>(src + s * stride, w);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += w[e];
    }
    bf16_t* dst = reinterpret_cast<bf16_t*>(rs ? rs_out : out) + 8 * (rs ? i - n8 : i);
    if (accum & (rs ? 2 : 1)) {  // gradient accumulation into the destination
      float o[8];
      load8<bf16_t>(dst, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += o[e];
    }
    store8<bf16_t>(dst, v);
  }
}

// the split-K reduce of a product: queued when the caller's scope asks for it (a weight
// gradient written into its claimed bucket slice, autograd.hip), else launched now
static void splitk_reduce(const at::Tensor& ws, int S, int64_t n8, int64_t slab, uint16_t* out, int64_t m8,
                          uint16_t* rs_out, int accum, hipStream_t st) {
  if (defer::want() && (defer::push_splitk(ws, S, n8, m8, slab, out, rs_out, accum, st) ||
                         defer::push_carry(ws, S, n8, m8, slab, out, rs_out, accum, st)))
    return;
  const int blocks = (int)std::min<int64_t>((n8 + m8 + 255) / 256, 2048);
  hipLaunchKernelGGL(reduce_kernel, dim3(blocks), dim3(256), 0, st, ws.data_ptr<float>(), S, n8, slab, out, m8,
                     rs_out, accum);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// ---- host --------------------------------------------------------------------------------------
struct Tile {
  int bm, bn, stages, waves, ks;
};

template <bool A_KM, bool B_KN, int EPI>
static void launch_epi(const Tile& t, const Args& a, dim3 grid, hipStream_t st) {
#define NBD_GEMM_K(BM_, BN_, S_, W_, KS_)                                                              \
  hipLaunchKernelGGL((gemm_kernel<BM_, BN_, A_KM, B_KN, EPI, S_, W_, KS_>), grid, dim3(64 * W_ * KS_), 0, st, a)
#define NBD_GEMM_CASE(BM_, BN_, KS_)                                   \
  if (t.bm == BM_ && t.bn == BN_ && t.waves == 4 && t.ks == KS_) {     \
    if (t.stages == 3) NBD_GEMM_K(BM_, BN_, 3, 4, KS_);                \
    else if (t.stages == 2) NBD_GEMM_K(BM_, BN_, 2, 4, KS_);           \
    else break;                                                        \
    return;                                                            \
  }
  // (deeper rings — 4, 6 and 8 stages, most K-tiles of a small product in flight at once —
  // measured slower on every workload shape: one workgroup per CU then leaves the tail round
  // serial; profiles/gemm_bench_r1.txt history)
  do {
    NBD_GEMM_CASE(128, 128, 1)
    NBD_GEMM_CASE(128, 64, 1)
    NBD_GEMM_CASE(64, 128, 1)
    NBD_GEMM_CASE(64, 64, 1)
    NBD_GEMM_CASE(128, 64, 2)  // intra-workgroup K-split: small, latency-bound products
    NBD_GEMM_CASE(64, 128, 2)
    NBD_GEMM_CASE(64, 64, 2)
    // 128x96 (row images only: the transposed-image swizzles assume 64- or 128-wide tiles):
    // N = 768 / 2304 forwards fill whole rounds of 2 workgroups per CU (512 / 1536 tiles)
    // where 128x128 leaves 0.75 / 2.25 rounds
    if constexpr (!A_KM && !B_KN) NBD_GEMM_CASE(128, 96, 1)
  } while (0);
  // 128x192, 8 waves (forward layout, plain / GELU epilogue): N = 768 forwards are exactly one
  // round of 256 workgroups (8192 tokens), N = 2304 / 3072 three / four; each wave's 64x48 block
  // reads 7 fragments per 12 MFMAs (128x128: 6 per 8)
  if constexpr (!A_KM && !B_KN && (EPI == EPI_NONE || EPI == EPI_GELU)) {
    if (t.bm == 128 && t.bn == 192 && t.waves == 8 && t.ks == 1) {
      if (t.stages == 3) NBD_GEMM_K(128, 192, 3, 8, 1);
      else NBD_GEMM_K(128, 192, 2, 8, 1);
      return;
    }
  }
  if (t.bm == 128 && t.bn == 128 && t.waves == 8 && t.ks == 1) {  // 8 waves: 128x128 only
    if (t.stages == 9) NBD_GEMM_K(128, 128, 103, 8, 1);  // ping-pong, 3-buffer ring
    else if (t.stages == 3) NBD_GEMM_K(128, 128, 3, 8, 1);
    else NBD_GEMM_K(128, 128, 2, 8, 1);
    return;
  }
#undef NBD_GEMM_CASE
#undef NBD_GEMM_K
  TORCH_CHECK(false, "nbd::gemm: no kernel for tile ", t.bm, "x", t.bn, " with ", t.waves, " waves, ", t.stages,
              " stages, K-split ", t.ks);
}

template <bool A_KM, bool B_KN>
static void launch_layout(int epi, const Tile& t, const Args& a, dim3 grid, hipStream_t st) {
  switch (epi) {
    case EPI_NONE: launch_epi<A_KM, B_KN, EPI_NONE>(t, a, grid, st); return;
    case EPI_GELU:
      if constexpr (!A_KM && !B_KN) {
        launch_epi<false, false, EPI_GELU>(t, a, grid, st);
        return;
      }
      break;
    case EPI_DGELU:
      if constexpr (!A_KM && B_KN) {
        launch_epi<false, true, EPI_DGELU>(t, a, grid, st);
        return;
      }
      break;
    case EPI_SWIGLU:
      if constexpr (!A_KM && !B_KN) {
        launch_epi<false, false, EPI_SWIGLU>(t, a, grid, st);
        return;
      }
      break;
    case EPI_DSWIGLU:
      if constexpr (!A_KM && B_KN) {
        launch_epi<false, true, EPI_DSWIGLU>(t, a, grid, st);
        return;
      }
      break;
    case EPI_ROWSUM:
      if constexpr (A_KM && B_KN) {
        launch_epi<true, true, EPI_ROWSUM>(t, a, grid, st);
        return;
      }
      break;
    default: break;
  }
  TORCH_CHECK(false, "nbd::gemm: epilogue ", epi, " not built for this layout");
}

// ---- next-weight warm-up -------------------------------------------------------------------------
// Inside a training step a weight is cold when its product starts: the activations streamed since
// its last use evicted it from the L2s and the MALL, and the first round of workgroups (all
// reading the same weight panels) then waits on HBM for every K-tile.  Measured on the q|k|v
// forward (8192x2304x768) right after a graphed GPT-2 step: 56 µs cold, 49.5 µs with the weight
// touched beforehand, 46 µs with weight and input touched, 40-42 µs back to back
// (benchmarks/gemm_context.py, profiles/gemm_context_r3.txt).  The launches therefore learn the
// order in which weights are used — keyed by (weight address, direction): forward products
// (B = W [N][K]) and backward ones (dgrad / pair, B = W as [K][N]) form two different chains —
// and each launch's first workgroups touch the weight the NEXT launch used the previous time
// round, so it arrives in the MALL while this product computes.
//
// Safety and stability rules:
// * the order is learned per HIP stream (a graph's capture stream, the default stream and a side
//   stream never splice their launch sequences together);
// * a link prev -> next is used only once it has been observed on two consecutive occurrences
//   of prev (a one-off transition — the last product of one model followed by the first of
//   another, or of a different cell — is never acted upon);
// * the weight is held weakly through its storage and re-validated at every eager lookup: only
//   bytes inside a live storage are ever read;
// * under stream capture the pointer is frozen into the graph, so the looked-up storage is also
//   kept alive STRONGLY until the capturer takes the references (gemm_warm_take_refs, called by
//   graphs.GraphedStep which holds them for the graph's lifetime).
// NBD_GEMM_WARM=0 disables it.
namespace warm {
constexpr int64_t kCapBytes = 8 << 20;  // the first 8 MiB: a product's first-round panels
struct Target {
  c10::weak_intrusive_ptr<c10::StorageImpl> storage{c10::intrusive_ptr<c10::StorageImpl>()};  // null: expired
  int64_t offset = 0, bytes = 0;
  uintptr_t key = 0;
};
struct Next {
  Target confirmed;     // acted upon
  Target cand;          // last observed successor
  int count = 0;        // consecutive observations of cand
  bool has_confirmed = false;
};
std::mutex g_mu;
std::unordered_map<uintptr_t, Next> g_next;         // key: weight address | direction
std::unordered_map<uintptr_t, uintptr_t> g_last;     // per (device, stream): the previous launch's key
std::vector<c10::intrusive_ptr<c10::StorageImpl>> g_capture_refs;  // warmed during capture

bool enabled() {
  const char* e = std::getenv("NBD_GEMM_WARM");
  return e == nullptr || e[0] != '0';
}

static bool capturing(hipStream_t st) {
  hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &s) != hipSuccess) return true;  // unknown: behave as under capture
  return s != hipStreamCaptureStatusNone;
}

// Record `w` as the weight of this launch on stream `st` (or of a library product announced by
// gemm_warm_hint; `cap` = how much of it the launch before may warm) and return the next launch's
// weight to touch (nullptr if none is confirmed).
const uint8_t* lookup(const at::Tensor& w, bool backward, hipStream_t st, int64_t& lines, int64_t cap = kCapBytes) {
  lines = 0;
  const int dev = w.get_device();
  if (dev < 0 || !w.has_storage()) return nullptr;
  const uintptr_t key = reinterpret_cast<uintptr_t>(w.data_ptr()) | (backward ? 1u : 0u);
  const uintptr_t skey = reinterpret_cast<uintptr_t>(st) ^ (uintptr_t)dev;
  const bool cap_mode = capturing(st);
  std::lock_guard<std::mutex> lk(g_mu);
  uintptr_t& last = g_last[skey];
  const uintptr_t prev = last;
  last = key;
  if (prev != 0 && prev != key) {
    if (g_next.size() > 4096) {  // forget dead weights (tests create many)
      for (auto it = g_next.begin(); it != g_next.end();)
        it = it->second.cand.storage.expired() && it->second.confirmed.storage.expired() ? g_next.erase(it) : ++it;
    }
    const at::Storage& s = w.storage();
    Target t;
    t.storage = s.getWeakStorageImpl();
    t.offset = static_cast<const uint8_t*>(w.data_ptr()) - static_cast<const uint8_t*>(s.data());
    t.bytes = std::min<int64_t>((int64_t)w.numel() * (int64_t)w.element_size(), cap);
    t.key = key;
    Next& n = g_next[prev];
    if (n.count > 0 && n.cand.key == key && !n.cand.storage.expired()) {
      if (++n.count >= 2) {
        n.confirmed = t;
        n.has_confirmed = true;
      }
    } else {
      n.cand = t;
      n.count = 1;
    }
  }
  auto it = g_next.find(key);
  if (it == g_next.end() || !it->second.has_confirmed) return nullptr;
  c10::intrusive_ptr<c10::StorageImpl> s = it->second.confirmed.storage.lock();
  if (!s) {
    it->second.has_confirmed = false;
    return nullptr;
  }
  const int64_t off = it->second.confirmed.offset, bytes = it->second.confirmed.bytes;
  if (s->device().index() != dev || off < 0 || off + bytes > (int64_t)s->nbytes() || s->data() == nullptr)
    return nullptr;
  const uint8_t* base = static_cast<const uint8_t*>(s->data()) + off;
  // whole 128-B lines inside [base, base + bytes): the 4-byte load at each line start stays in bounds
  const uintptr_t first = (reinterpret_cast<uintptr_t>(base) + 127) & ~uintptr_t(127);
  const uintptr_t end = reinterpret_cast<uintptr_t>(base) + bytes;
  if (end <= first) return nullptr;
  lines = (int64_t)((end - first) / 128);
  if (lines <= 0) return nullptr;
  if (cap_mode) g_capture_refs.push_back(std::move(s));  // frozen into the graph: keep it alive
  return reinterpret_cast<const uint8_t*>(first);
}

// warm-up blocks for `lines` lines at `nth` threads per block: ~4 lines per thread per pass, a
// multiple of 8 (block ids keep their XCD), at most 128 (a large weight takes several passes)
int blocks_for(int64_t lines, int nth) {
  if (lines <= 0) return 0;
  const int64_t b = (lines + 4LL * nth - 1) / (4LL * nth);
  return (int)std::min<int64_t>(128, (b + 7) / 8 * 8);
}
}  // namespace warm

// A library product (the LM head's hipBLASLt GEMMs) announces its weight: it joins the learned
// order, so the HIP launch before it warms up to max_bytes of that weight.  Host-side only.
void gemm_warm_hint(const at::Tensor& w, bool backward, int64_t max_bytes) {
  if (!warm::enabled() || !w.is_cuda()) return;
  int64_t lines = 0;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  warm::lookup(w, backward, st, lines, std::max<int64_t>(0, max_bytes));
}

// The storages whose bytes captured launches warm (one tensor aliasing each): the graph's owner
// keeps them for the graph's lifetime.  Clears the pending list.
std::vector<at::Tensor> gemm_warm_take_refs() {
  std::vector<c10::intrusive_ptr<c10::StorageImpl>> refs;
  {
    std::lock_guard<std::mutex> lk(warm::g_mu);
    refs.swap(warm::g_capture_refs);
  }
  std::vector<at::Tensor> out;
  out.reserve(refs.size());
  for (auto& s : refs) {
    at::Tensor t = at::empty({0}, at::TensorOptions().dtype(at::kByte).device(s->device()));
    t.set_(at::Storage(std::move(s)));
    out.push_back(std::move(t));
  }
  return out;
}

// Forget every learned link (tests; a notebook that wants a clean slate).
void gemm_warm_reset() {
  std::lock_guard<std::mutex> lk(warm::g_mu);
  warm::g_next.clear();
  warm::g_last.clear();
}

static bool tile_fits(const Tile& t, int M, int N) { return M % t.bm == 0 && N % t.bn == 0; }

// The largest tile that still gives about one workgroup per CU (256 CUs); a hint (BM*1000+BN)
// overrides it.
static Tile pick_tile(int M, int N, int64_t tile_hint) {
  if (tile_hint > 0) {
    // hint = ks*10^8 + waves*10^7 + stages*10^6 + BM*1000 + BN (ks 0 -> 1, waves 0 -> 4, stages 0 -> 2)
    // (stages digit 9: the ping-pong schedule with a 3-buffer ring, 128x128 / 8 waves)
    const int stg = (int)(tile_hint / 1000000 % 10), wv = (int)(tile_hint / 10000000 % 10);
    const int ks = (int)(tile_hint / 100000000);
    Tile t{(int)(tile_hint / 1000 % 1000), (int)(tile_hint % 1000), stg < 2 ? 2 : stg, wv == 8 ? 8 : 4, ks == 2 ? 2 : 1};
    TORCH_CHECK(t.stages != 9 || (t.bm == 128 && t.bn == 128 && t.waves == 8 && t.ks == 1),
                "nbd::gemm: the ping-pong schedule is built for 128x128 tiles with 8 waves");
    TORCH_CHECK(tile_fits(t, M, N), "nbd::gemm: tile ", t.bm, "x", t.bn, " does not divide ", M, "x", N);
    return t;
  }
  const Tile cands[4] = {{128, 128, 2, 4, 1}, {128, 64, 2, 4, 1}, {64, 128, 2, 4, 1}, {64, 64, 2, 4, 1}};
  int best = -1;
  for (int i = 0; i < 4; ++i) {
    if (!tile_fits(cands[i], M, N)) continue;
    best = i;
    if ((int64_t)(M / cands[i].bm) * (N / cands[i].bn) >= 256) break;
  }
  TORCH_CHECK(best >= 0, "nbd::gemm: M=", M, " N=", N, " not divisible by 64");
  return cands[best];
}

// Column split (tile hint >= kColSplit: hint - kColSplit = the tail's tile): the product's first
// N0 columns — as many as make WHOLE rounds of 256x256 tiles, one workgroup per CU — run on the
// 8-phase 256x256 kernel (gemm256.hip), the remaining N - N0 columns on the tail tile, as a second
// launch writing the same C (row stride N).  GPT-2 small's q|k|v (N = 2304 = 2048 + 256) and c_fc
// (N = 3072 = 2048 + 1024) forwards at 8192 tokens: 1.125 / 1.5 rounds of 256x256 tiles as one
// kernel, 2.25 / 3 rounds of 128x128 at two per CU (benchmarks/gemm_colsplit.py).  N0 = 0 when M
// is not a multiple of 256 or no whole round fits: the tail tile then runs the whole product.
constexpr int64_t kColSplit = 1000000000;
constexpr int kCUs = 256;

static int colsplit_head(int M, int N) {
  if (M % 256 != 0) return 0;
  const int64_t tm = M / 256;
  // columns per round of kCUs tiles; whole rounds only
  if ((int64_t)kCUs % tm != 0) return 0;
  const int per_round = (int)(kCUs / tm) * 256;
  return N / per_round * per_round;
}

void gemm_hip_one(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c, bool a_km, bool b_kn,
                  const c10::optional<at::Tensor>& bias, int64_t epi, const c10::optional<at::Tensor>& aux_in,
                  const c10::optional<at::Tensor>& aux_out, int64_t splits, int64_t tile_hint, int64_t accum);

// c = A·B with the layouts above; c is [M][N] bf16 (contiguous).
void gemm_hip(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c, bool a_km, bool b_kn,
              const c10::optional<at::Tensor>& bias, int64_t epi, const c10::optional<at::Tensor>& aux_in,
              const c10::optional<at::Tensor>& aux_out, int64_t splits, int64_t tile_hint, int64_t accum) {
  if (tile_hint >= kColSplit) {
    const int64_t tail = tile_hint - kColSplit;
    const int M = a_km ? a.size(1) : a.size(0);
    const int N = b_kn ? b.size(1) : b.size(0);
    const int N0 = (!a_km && (epi == EPI_NONE || epi == EPI_GELU || epi == EPI_DGELU) && splits <= 1 && accum == 0)
                       ? colsplit_head(M, N) : 0;
    if (N0 == 0 || N0 == N) {
      gemm_hip_one(a, b, c, a_km, b_kn, bias, epi, aux_in, aux_out, splits, N0 == N ? 86256256 : tail, accum);
      return;
    }
    // column blocks of B (rows of W [N][K], or columns of W as [K][N]), of C / the aux tensors
    // (row stride N) and of the bias
    auto cols = [&](const at::Tensor& t, int64_t lo, int64_t n) { return t.narrow(1, lo, n); };
    const at::Tensor b0 = b_kn ? cols(b, 0, N0) : b.narrow(0, 0, N0);
    const at::Tensor b1 = b_kn ? cols(b, N0, N - N0) : b.narrow(0, N0, N - N0);
    auto part = [&](const c10::optional<at::Tensor>& t, int64_t lo, int64_t n) -> c10::optional<at::Tensor> {
      if (!t) return c10::nullopt;
      return t->dim() == 1 ? t->narrow(0, lo, n) : cols(*t, lo, n);
    };
    gemm_hip_one(a, b0, cols(c, 0, N0), false, b_kn, part(bias, 0, N0), epi, part(aux_in, 0, N0),
                 part(aux_out, 0, N0), 1, 86256256, 0);
    gemm_hip_one(a, b1, cols(c, N0, N - N0), false, b_kn, part(bias, N0, N - N0), epi, part(aux_in, N0, N - N0),
                 part(aux_out, N0, N - N0), 1, tail, 0);
    return;
  }
  gemm_hip_one(a, b, c, a_km, b_kn, bias, epi, aux_in, aux_out, splits, tile_hint, accum);
}

// one launch (plus its split-K reduce).  C (and the aux tensors, which share its layout) may be a
// column block of a wider row-major matrix (unit inner stride, row stride >= N: the column split
// above) when there is no split-K; B [N][K] a row block, B as [K][N] a column block.
void gemm_hip_one(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c, bool a_km, bool b_kn,
                  const c10::optional<at::Tensor>& bias, int64_t epi, const c10::optional<at::Tensor>& aux_in,
                  const c10::optional<at::Tensor>& aux_out, int64_t splits, int64_t tile_hint, int64_t accum) {
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && c.dim() == 2, "nbd::gemm: 2-D operands");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && c.scalar_type() == at::kBFloat16,
              "nbd::gemm: bf16 operands");
  // A may be a row-strided view (unit inner stride, row stride >= its width: a column block of a
  // wider matrix, e.g. the LM head's weight gradient split by vocabulary rows); B and C contiguous
  TORCH_CHECK(a.stride(1) == 1 && a.stride(0) >= a.size(1) && b.stride(1) == 1 && b.stride(0) >= b.size(1) &&
                  c.stride(1) == 1 && c.stride(0) >= c.size(1),
              "nbd::gemm: operands need a unit inner stride (row-strided blocks of wider matrices allowed)");
  const bool c_dense = c.is_contiguous();
  const int M = a_km ? a.size(1) : a.size(0);
  const int K = a_km ? a.size(0) : a.size(1);
  const int N = b_kn ? b.size(1) : b.size(0);
  const int Kb = b_kn ? b.size(0) : b.size(1);
  TORCH_CHECK(K == Kb, "nbd::gemm: K mismatch ", K, " vs ", Kb);
  // EPI_SWIGLU writes silu(g)·u: [M][N/2]; EPI_DSWIGLU writes d[g|u]: [M][2N]
  const int64_t cN = epi == EPI_SWIGLU ? N / 2 : epi == EPI_DSWIGLU ? 2 * (int64_t)N : N;
  TORCH_CHECK(c.size(0) == M && c.size(1) == cN, "nbd::gemm: output shape");
  TORCH_CHECK(K % BK == 0 && K > 0, "nbd::gemm: K % 64 != 0");
  TORCH_CHECK(!(a_km && !b_kn), "nbd::gemm: layout (A [K][M], B [N][K]) not built");
  for (const at::Tensor* x : {&a, &b, &c})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x->data_ptr()) % 16 == 0, "nbd::gemm: 16-byte aligned operands");
  if (bias) {
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == N && bias->scalar_type() == at::kBFloat16, "nbd::gemm: bias");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(bias->data_ptr()) % 8 == 0, "nbd::gemm: bias alignment");
  }
  // (the GELU / GELU′ operands are indexed with C's row stride)
  if (epi == EPI_GELU)
    TORCH_CHECK(aux_out && aux_out->sizes() == c.sizes() && aux_out->strides() == c.strides() &&
                    aux_out->scalar_type() == at::kBFloat16, "nbd::gemm: aux_out");
  if (epi == EPI_DGELU)
    TORCH_CHECK(aux_in && aux_in->sizes() == c.sizes() && aux_in->strides() == c.strides() &&
                    aux_in->scalar_type() == at::kBFloat16, "nbd::gemm: aux_in");
  TORCH_CHECK(c_dense || (epi == EPI_NONE || epi == EPI_GELU || epi == EPI_DGELU),
              "nbd::gemm: a row-strided C only with the plain / GELU / GELU' epilogues");
  if (epi == EPI_ROWSUM)
    TORCH_CHECK(aux_out && aux_out->numel() == M && aux_out->is_contiguous() &&
                    aux_out->scalar_type() == at::kBFloat16 && reinterpret_cast<uintptr_t>(aux_out->data_ptr()) % 16 == 0,
                "nbd::gemm: aux_out (row sums)");
  if (epi == EPI_SWIGLU) {
    TORCH_CHECK(!a_km && !b_kn && !bias, "nbd::gemm: SwiGLU epilogue: forward layout, no bias");
    TORCH_CHECK(aux_out && aux_out->size(0) == M && aux_out->size(1) == N && aux_out->is_contiguous() &&
                    aux_out->scalar_type() == at::kBFloat16 && reinterpret_cast<uintptr_t>(aux_out->data_ptr()) % 16 == 0,
                "nbd::gemm: aux_out ([g|u] pre-activations)");
  }
  if (epi == EPI_DSWIGLU) {
    TORCH_CHECK(!a_km && b_kn && !bias, "nbd::gemm: SwiGLU backward epilogue: dgrad layout, no bias");
    TORCH_CHECK(aux_in && aux_in->size(0) == M && aux_in->size(1) == 2 * (int64_t)N && aux_in->is_contiguous() &&
                    aux_in->scalar_type() == at::kBFloat16 && reinterpret_cast<uintptr_t>(aux_in->data_ptr()) % 16 == 0,
                "nbd::gemm: aux_in ([g|u] pre-activations)");
  }
  TORCH_CHECK(epi >= EPI_NONE && epi <= EPI_DSWIGLU, "nbd::gemm: epilogue ", epi);
  const Tile t = pick_tile(M, N, tile_hint);
  TORCH_CHECK(accum == 0 || ((epi == EPI_NONE || epi == EPI_ROWSUM) && !bias && t.bm != 256),
              "nbd::gemm: accumulation only for plain / row-sum products on the 64-128 tile kernels");
  // per-lane DMA offsets are 32-bit byte offsets within one tile's rows (gemm_common.h Pieces)
  {
    const int64_t ra = a_km ? BK : t.bm, rb = b_kn ? BK : (epi == EPI_SWIGLU ? N / 2 + t.bn : t.bn);
    TORCH_CHECK(ra * a.stride(0) * 2 < (1LL << 32) && rb * b.stride(0) * 2 < (1LL << 32),
                "nbd::gemm: row stride too large for 32-bit DMA offsets");
  }
  const int tiles = (M / t.bm) * (N / t.bn);
  const int S = splits > 0 ? (int)splits : 1;
  TORCH_CHECK(K % (BK * S * t.ks) == 0, "nbd::gemm: K not divisible into ", S, " splits x ", t.ks, " K-groups");
  TORCH_CHECK(S == 1 || ((epi == EPI_NONE || epi == EPI_ROWSUM) && !bias),
              "nbd::gemm: split-K only without an elementwise epilogue");
  TORCH_CHECK(S == 1 || c_dense, "nbd::gemm: split-K writes a contiguous C");
  TORCH_CHECK(c.stride(0) < (1LL << 31) && b.stride(0) < (1LL << 31), "nbd::gemm: row stride too large");

  const c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  Args p;
  p.a = static_cast<const uint16_t*>(a.data_ptr());
  p.b = static_cast<const uint16_t*>(b.data_ptr());
  p.bias = bias ? static_cast<const uint16_t*>(bias->data_ptr()) : nullptr;
  p.aux_in = aux_in ? static_cast<const uint16_t*>(aux_in->data_ptr()) : nullptr;
  p.aux_out = aux_out ? static_cast<uint16_t*>(aux_out->data_ptr()) : nullptr;
  p.M = M;
  p.N = N;
  p.K = K / S;
  p.lda = a.stride(0);
  p.ldb = b.stride(0);
  p.ldc = c.stride(0);  // = cN when C is contiguous
  p.tiles_m = M / t.bm;
  p.tiles_n = N / t.bn;
  p.accum = (int)accum;
  p.pf = nullptr;
  p.pf_lines = 0;
  p.warm_blocks = 0;
  if (!a_km && warm::enabled()) {  // B is a weight (forward / dgrad), not an activation (wgrad)
    const uint8_t* pf = warm::lookup(b, b_kn, st, p.pf_lines);
    if (pf != nullptr && t.bm != 256) {  // (the 256x256 kernel has no warm-up blocks)
      p.pf = pf;
      p.warm_blocks = warm::blocks_for(p.pf_lines, 64 * t.waves * t.ks);
    }
  }
  const dim3 grid(tiles + p.warm_blocks, S);
  p.c = static_cast<uint16_t*>(c.data_ptr());
  at::Tensor ws;
  p.ws = nullptr;
  if (S > 1) {
    // stream-ordered (caching allocator): S slabs [M][N] (+ S row-sum partials [M])
    ws = at::empty({(int64_t)S * M * N + (epi == EPI_ROWSUM ? (int64_t)S * M : 0)}, a.options().dtype(at::kFloat));
    p.ws = ws.data_ptr<float>();
  }
  if (t.bm == 256)
    launch_gemm256(p, a_km, b_kn, (int)epi, grid, st, t.stages - 2);
  else if (!a_km && !b_kn)
    launch_layout<false, false>((int)epi, t, p, grid, st);
  else if (!a_km && b_kn)
    launch_layout<false, true>((int)epi, t, p, grid, st);
  else
    launch_layout<true, true>((int)epi, t, p, grid, st);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  if (S > 1)
    splitk_reduce(ws, S, (int64_t)M * N / 8, (int64_t)M * N, p.c, epi == EPI_ROWSUM ? M / 8 : 0, p.aux_out, p.accum,
                  st);
}

// A Linear layer's two backward products in one launch (pair_kernel): c1 = a1·b1 in the dgrad
// layout (a1 [M1][K1], b1 as [K1][N1]) with epi1 ∈ {none, GELU′ (aux_in1 = pre-activation)}, and
// c2 = a2ᵀ·b2 in the wgrad layout (a2 as [K2][M2], b2 as [K2][N2]) with epi2 ∈ {none, row sums
// into aux_out2}, split s2 ways along K2 (fp32 slabs + reduce_kernel).  128x128 tiles only.
void gemm_pair_hip(const at::Tensor& a1, const at::Tensor& b1, const at::Tensor& c1, int64_t epi1,
                   const c10::optional<at::Tensor>& aux_in1, const at::Tensor& a2, const at::Tensor& b2,
                   const at::Tensor& c2, int64_t epi2, const c10::optional<at::Tensor>& aux_out2, int64_t splits2,
                   int64_t accum2, const c10::optional<at::Tensor>& delta1, int64_t delta_T) {
  for (const at::Tensor* x : {&a1, &b1, &c1, &a2, &b2, &c2}) {
    TORCH_CHECK(x->dim() == 2 && x->scalar_type() == at::kBFloat16 && x->is_contiguous() && x->is_cuda() &&
                    reinterpret_cast<uintptr_t>(x->data_ptr()) % 16 == 0,
                "nbd::gemm_pair: contiguous 16-B aligned bf16 2-D GPU operands");
  }
  TORCH_CHECK(epi1 == EPI_NONE || epi1 == EPI_DGELU || epi1 == EPI_DSWIGLU || epi1 == EPI_ADELTA,
              "nbd::gemm_pair: epi1 must be none, GELU', SwiGLU' or the attention delta");
  TORCH_CHECK(epi2 == EPI_NONE || epi2 == EPI_ROWSUM, "nbd::gemm_pair: epi2 must be none or row sums");
  // product 1: dgrad layout
  const int M1 = a1.size(0), K1 = a1.size(1), N1 = b1.size(1);
  // SwiGLU′ writes d[g|u] [M][2N] from the saved pre-activations [g|u] [M][2N]
  const int64_t c1N = epi1 == EPI_DSWIGLU ? 2 * (int64_t)N1 : N1;
  TORCH_CHECK(b1.size(0) == K1 && c1.size(0) == M1 && c1.size(1) == c1N, "nbd::gemm_pair: product 1 shapes");
  // product 2: wgrad layout
  const int K2 = a2.size(0), M2 = a2.size(1), N2 = b2.size(1);
  TORCH_CHECK(b2.size(0) == K2 && c2.size(0) == M2 && c2.size(1) == N2, "nbd::gemm_pair: product 2 shapes");
  // splits2 = S | wfirst << 4 | small << 5 (the plan's encoding: ops/gemm.py pair_plan)
  const int S = (splits2 & 15) > 0 ? (int)(splits2 & 15) : 1;
  const int wfirst = (int)((splits2 >> 4) & 1);
  const bool small = (splits2 >> 5) & 1;  // bit 5: 64x64 tiles even where 128x128 would fit
  const bool big = !small && M1 % 128 == 0 && N1 % 128 == 0 && M2 % 128 == 0 && N2 % 128 == 0;
  const int TB = big ? 128 : 64;
  TORCH_CHECK(M1 % TB == 0 && N1 % TB == 0 && M2 % TB == 0 && N2 % TB == 0 && K1 % BK == 0 && K1 > 0 &&
                  K2 % (BK * S) == 0 && K2 > 0,
              "nbd::gemm_pair: 64-granular shapes and K divisible into 64-deep tiles (x ", S, " splits)");
  if (epi1 != EPI_NONE)
    TORCH_CHECK(aux_in1 && aux_in1->sizes() == c1.sizes() && aux_in1->is_contiguous() &&
                    aux_in1->scalar_type() == at::kBFloat16 && reinterpret_cast<uintptr_t>(aux_in1->data_ptr()) % 16 == 0,
                "nbd::gemm_pair: aux_in1 (pre-activations)");
  if (epi2 == EPI_ROWSUM)
    TORCH_CHECK(aux_out2 && aux_out2->numel() == M2 && aux_out2->is_contiguous() &&
                    aux_out2->scalar_type() == at::kBFloat16 && reinterpret_cast<uintptr_t>(aux_out2->data_ptr()) % 16 == 0,
                "nbd::gemm_pair: aux_out2 (row sums)");
  // per-lane DMA offsets are 32-bit byte offsets within one tile's rows (gemm_common.h Pieces)
  TORCH_CHECK((int64_t)TB * a1.size(1) * 2 < (1LL << 32) && (int64_t)BK * b1.size(1) * 2 < (1LL << 32) &&
                  (int64_t)BK * a2.size(1) * 2 < (1LL << 32) && (int64_t)BK * b2.size(1) * 2 < (1LL << 32),
              "nbd::gemm_pair: row stride too large for 32-bit DMA offsets");
  Args p1{}, p2{};
  p1.a = static_cast<const uint16_t*>(a1.data_ptr());
  p1.b = static_cast<const uint16_t*>(b1.data_ptr());
  p1.c = static_cast<uint16_t*>(c1.data_ptr());
  p1.aux_in = epi1 != EPI_NONE ? static_cast<const uint16_t*>(aux_in1->data_ptr()) : nullptr;
  p1.M = M1; p1.N = N1; p1.K = K1;
  p1.lda = a1.size(1); p1.ldb = b1.size(1); p1.ldc = c1N;
  if (epi1 == EPI_ADELTA) {  // δ [M1 / T][N1 / 64][T] from dO (c1) and O (aux_in1)
    TORCH_CHECK(delta1 && delta1->is_cuda() && delta1->scalar_type() == at::kFloat && delta1->is_contiguous() &&
                    delta_T > 0 && M1 % delta_T == 0 && N1 % 64 == 0 && delta1->numel() == (int64_t)M1 / 64 * N1,
                "nbd::gemm_pair: the attention delta needs delta float32 [M / T, N / 64, T] and T dividing M");
    p1.delta = delta1->data_ptr<float>();
    p1.dT = (int)delta_T;
  }
  p1.tiles_m = M1 / TB; p1.tiles_n = N1 / TB;
  p2.a = static_cast<const uint16_t*>(a2.data_ptr());
  p2.b = static_cast<const uint16_t*>(b2.data_ptr());
  p2.c = static_cast<uint16_t*>(c2.data_ptr());
  p2.aux_out = epi2 == EPI_ROWSUM ? static_cast<uint16_t*>(aux_out2->data_ptr()) : nullptr;
  p2.M = M2; p2.N = N2; p2.K = K2 / S;
  p2.lda = a2.size(1); p2.ldb = b2.size(1); p2.ldc = N2;
  p2.tiles_m = M2 / TB; p2.tiles_n = N2 / TB;
  p2.accum = (int)accum2;  // the weight-gradient half may accumulate into its destination
  at::Tensor ws;
  if (S > 1) {
    ws = at::empty({(int64_t)S * M2 * N2 + (epi2 == EPI_ROWSUM ? (int64_t)S * M2 : 0)}, a1.options().dtype(at::kFloat));
    p2.ws = ws.data_ptr<float>();
  }
  const int t1 = p1.tiles_m * p1.tiles_n, t2 = p2.tiles_m * p2.tiles_n;
  const int nb1 = (t1 + 7) / 8 * 8, nb2 = (t2 * S + 7) / 8 * 8;
  const int first = wfirst ? nb2 : nb1;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(a1.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  if (warm::enabled()) {  // b1 = W: the backward chain (next-weight warm-up, above)
    const uint8_t* pf = warm::lookup(b1, true, st, p1.pf_lines);
    if (pf != nullptr) {
      p1.pf = pf;
      p1.warm_blocks = warm::blocks_for(p1.pf_lines, big ? 512 : 256);
    }
  }
  // a previous product's large split-K reduce rides in this grid's tail (defer::take_carry)
  // (NBD_GEMM_CARRY_QUEUED=1: also up to kRedMax - 1 queued small ones, which then need no flush
  // launch — measured no faster on the notebook step, whose flushes are few: FINDINGS §36)
  static const int take_max = [] {
    const char* e = std::getenv("NBD_GEMM_CARRY_QUEUED");
    return e != nullptr && e[0] == '1' ? kRedMax : 1;
  }();
  RedTable red{};
  defer::Carry carried[kRedMax];
  red.n = defer::take_carry(st, carried, take_max);
  for (int i = 0; i < red.n; ++i) {
    const defer::Carry& c = carried[i];
    const int nt = big ? 512 : 256;  // threads per workgroup of this launch
    red.d[i] = Red{c.buf.data_ptr<float>(), c.out, c.rs_out, c.n8, c.m8, c.slab, c.splits, c.accum,
                   (int)std::max<int64_t>(1, std::min<int64_t>((c.n8 + c.m8 + 4LL * nt - 1) / (4LL * nt), 1024))};
    red.blocks += red.d[i].blocks;
  }
  const int64_t nblocks = (int64_t)p1.warm_blocks + nb1 + nb2 + red.blocks;
  TORCH_CHECK(nblocks < (1LL << 31), "nbd::gemm_pair: grid too large");
  const dim3 grid((unsigned)nblocks);
  // NBD_GEMM_PAIR_PP=1: the 128x128 halves on the ping-pong schedule (one workgroup per CU)
  const char* pp_env = std::getenv("NBD_GEMM_PAIR_PP");
  const bool pp = pp_env != nullptr && pp_env[0] == '1';
  auto launch = [&](auto e1, auto e2) {
    constexpr int E1 = decltype(e1)::value, E2 = decltype(e2)::value;
    if (big && pp)
      hipLaunchKernelGGL((pair_kernel<128, 128, 8, 103, E1, E2>), grid, dim3(512), 0, st, p1, t1, first, p2, t2, S, wfirst,
                         red);
    else if (big)
      hipLaunchKernelGGL((pair_kernel<128, 128, 8, 2, E1, E2>), grid, dim3(512), 0, st, p1, t1, first, p2, t2, S, wfirst,
                         red);
    else
      hipLaunchKernelGGL((pair_kernel<64, 64, 4, 3, E1, E2>), grid, dim3(256), 0, st, p1, t1, first, p2, t2, S, wfirst,
                         red);
  };
  using I0 = std::integral_constant<int, EPI_NONE>;
  using I2 = std::integral_constant<int, EPI_DGELU>;
  using I3 = std::integral_constant<int, EPI_ROWSUM>;
  using I5 = std::integral_constant<int, EPI_DSWIGLU>;
  using I6 = std::integral_constant<int, EPI_ADELTA>;
  if (epi2 == EPI_NONE) {
    if (epi1 == EPI_NONE) launch(I0{}, I0{});
    else if (epi1 == EPI_DGELU) launch(I2{}, I0{});
    else if (epi1 == EPI_ADELTA) launch(I6{}, I0{});
    else launch(I5{}, I0{});
  } else {
    if (epi1 == EPI_NONE) launch(I0{}, I3{});
    else if (epi1 == EPI_DGELU) launch(I2{}, I3{});
    else if (epi1 == EPI_ADELTA) launch(I6{}, I3{});
    else launch(I5{}, I3{});
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  if (S > 1)
    splitk_reduce(ws, S, (int64_t)M2 * N2 / 8, (int64_t)M2 * N2, p2.c, epi2 == EPI_ROWSUM ? M2 / 8 : 0, p2.aux_out,
                  p2.accum, st);
}

}  // namespace gemm
}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("gemm", &nbd::gemm::gemm_hip);
  m.impl("gemm_pair", &nbd::gemm::gemm_pair_hip);
}

// bookkeeping only (no device work): a catch-all kernel
TORCH_LIBRARY_FRAGMENT(nbd, m) {
  m.def("gemm_warm_hint(Tensor w, bool backward, int max_bytes) -> ()", &nbd::gemm::gemm_warm_hint);
  m.def("gemm_warm_take_refs() -> Tensor[]", &nbd::gemm::gemm_warm_take_refs);
  m.def("gemm_warm_reset() -> ()", &nbd::gemm::gemm_warm_reset);
}
