// gemm_common.h — pieces shared by the two bf16 MFMA GEMM kernel families:
//   gemm.hip     2/3-stage pipelines, 64..128-wide tiles, 4/8 waves (small and mid-size products)
//   gemm256.hip  256x256 tile, 8 waves, phase-interleaved schedule (large products: LM head)
// Operand layouts, LDS image swizzles, the LDS-DMA helper, the fragment reads and the epilogue
// activations are identical in both, so a product gives the same bits whichever kernel runs it
// (up to the fp32 summation order of the tile sizes).
#pragma once
#include <stdint.h>

#include "nbd_common.h"

namespace nbd {
namespace gemm {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;

// EPI_ROWSUM (weight-gradient layout): also Σ_k A[m,k] -> aux_out[m] — the Linear's bias gradient
// (Σ over tokens of dy) from the A fragments already in registers, one extra MFMA per fragment.
// EPI_SWIGLU (forward layout, B = [gate; up] weights [2I][K]): tile column block tn stages gate
// rows tn·BN/2.. and up rows I + tn·BN/2.. side by side, so the epilogue has g and u of the same
// feature: c = silu(g)·u [M][I], aux_out = [g|u] pre-activations [M][2I].
// EPI_DSWIGLU (dgrad layout, C = dact [M][I] never stored): aux_in = [g|u] [M][2I];
// c = d[g|u] [M][2I] = [dact·u·σ(g)(1 + g(1−σ(g))) | dact·silu(g)].
// EPI_ADELTA (dgrad layout, the input gradient of an attention output projection: C = dO [M][H·64]):
//   also δ[b][h][t] = Σ_d dO[m][64h + d]·O[m][64h + d] (m = b·T + t, O = aux_in, same layout as C)
//   into `delta` — the flash backward's pre-pass, from the tile's rounded outputs (attn.hip)
enum Epi : int { EPI_NONE = 0, EPI_GELU = 1, EPI_DGELU = 2, EPI_ROWSUM = 3, EPI_SWIGLU = 4, EPI_DSWIGLU = 5,
                 EPI_ADELTA = 6 };

struct Args {
  const uint16_t* a;
  const uint16_t* b;
  uint16_t* c;             // [M][ldc] bf16
  float* ws;               // split-K: [splits][M][ldc] fp32 slabs
  const uint16_t* bias;    // [N] or nullptr
  const uint16_t* aux_in;  // EPI_DGELU: pre-activation [M][ldc]; EPI_DSWIGLU: [g|u] [M][2N]
  uint16_t* aux_out;       // EPI_GELU: pre-activation out [M][ldc]; EPI_ROWSUM: row sums [M];
                           // EPI_SWIGLU: [g|u] out [M][N]
  int M, N, K;             // K = reduction length handled by one split
  int64_t lda, ldb, ldc;
  int tiles_m, tiles_n;
  int accum;               // bit 0: c += result (EPI_NONE / EPI_ROWSUM); bit 1: aux_out row sums +=
                           // (gradient accumulation into a DDP bucket slice: graddst.h)
  // weight warm-up (gemm.hip "next-weight warm-up"): blocks [0, warm_blocks) of the launch touch
  // the pf_lines 128-B lines at pf (the next launch's weight) instead of computing a tile
  const uint8_t* pf;
  int64_t pf_lines;
  int warm_blocks;
  float* delta;  // EPI_ADELTA: δ [M / dT][ldc / 64][dT] fp32
  int dT;
};

// ---- swizzles ---------------------------------------------------------------------------------
__device__ __forceinline__ int row_swz(int r) { return (r >> 1) & 7; }  // 16-B chunk XOR, row image
template <int R>
__device__ __forceinline__ int tr_swz(int k) {  // 8-B slot XOR, tr image with R-element rows
  if constexpr (R >= 128)
    return ((k & 3) | (((k >> 3) & 1) << 2)) << 2;
  else
    return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 2;
}

// 16-B global -> LDS DMA (global_load_lds_dwordx4: lane l lands at lds_wave_base + 16 l).
// Issued as inline asm on purpose: hipcc cannot prove that an in-flight DMA into one pipeline
// buffer and the ds_reads of another do not alias, and drains vmcnt(0) before the reads — which
// serialises the pipeline.  Hidden from it, the DMA is counted by our own vmcnt(N) waits
// (cdna_hip_programming.md §5.7 LDS-DMA recipe: M0 saved, written and restored in one statement).
__device__ __forceinline__ void glds16(const uint16_t* src, uint8_t* lds_wave_base) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(lds_wave_base));
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

// 16-B LDS DMA from a uniform (SGPR) base + a 32-bit per-lane byte offset: the saddr form of
// global_load_lds_dwordx4 — the per-lane part of the address is computed once per kernel, each
// K-step only moves the scalar base (no 64-bit VALU address arithmetic per DMA)
__device__ __forceinline__ void glds16s(const uint16_t* sbase_, uint32_t voff, uint8_t* lds_wave_base) {
  // the base is wave-uniform by construction; readfirstlane lets the compiler keep it in SGPRs
  const uint64_t b = (uint64_t)(uintptr_t)sbase_;
  // (the builtin returns int: widen through uint32_t, or the low half sign-extends into the high)
  const uint64_t sb = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint16_t* sbase = (const uint16_t*)(uintptr_t)sb;
  const uint32_t lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)(lds_wave_base));
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

// Per-lane byte offsets of one thread's DMA pieces of an R-row (or, TR, R-column) operand image
// (R x 64 K-tile = R/8 wave-pieces of 1 KiB, R/(8W) per wave) with the LDS swizzles above: row
// image [R][64] (16-B chunk ^ row_swz(row)), tr image [64][R] (16-B chunk ^ tr_swz(k)/2); R1 >= 0: rows R/2.. come from global rows r1.. (SwiGLU's
// up half), given as an element offset from the tile's first row.  stage() adds the uniform
// tile / K-step base.  Offsets must fit 32 bits: rows * ld * 2 bytes (asserted on the host).
template <int R, bool TR, int W>
struct Pieces {
  static constexpr int N = R / (8 * W);
  uint32_t off[N];
  __device__ __forceinline__ Pieces(int64_t ld, int wave, int lane, int64_t split_rows = 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int byte = (i * W + wave) * 1024 + lane * 16;
      int64_t e;
      if constexpr (!TR) {
        const int r = byte >> 7, pc = (byte >> 4) & 7;
        const int64_t row = (split_rows != 0 && r >= R / 2) ? split_rows + r - R / 2 : r;
        e = row * ld + 8 * (pc ^ row_swz(r));
      } else {
        constexpr int RB = 2 * R;
        const int k = byte / RB, pc = (byte % RB) >> 4;
        e = (int64_t)k * ld + 8 * (pc ^ (tr_swz<R>(k) >> 1));
      }
      off[i] = (uint32_t)(2 * e);
    }
  }
  // K-tile starting at k0 of the operand rows r0.. into img
  __device__ __forceinline__ void stage(const uint16_t* g, int64_t ld, int r0, int k0, uint8_t* img, int wave) const {
    const uint16_t* base = TR ? g + (int64_t)k0 * ld + r0 : g + (int64_t)r0 * ld + k0;
#pragma unroll
    for (int i = 0; i < N; ++i) glds16s(base, off[i], img + (i * W + wave) * 1024);
  }
};

// 16x16x32 operand fragment (lane l: rows/cols r0 + (l&15), k = 32kk + 8(l>>4) + 0..7) from an
// LDS image with R rows (row image [R][64], 128-B rows) or R columns (tr image [64][R]).
template <int R, bool TR>
__device__ __forceinline__ s8v frag(const uint8_t* img, int r0, int kk, int lane) {
  if constexpr (!TR) {
    const int r = r0 + (lane & 15), c = (lane >> 4) + 4 * kk;
    return *reinterpret_cast<const s8v*>(img + r * 128 + ((c ^ row_swz(r)) << 4));
  } else {
    constexpr int RB = 2 * R;
    const int i = lane & 15, g = lane >> 4;
    const int k = 32 * kk + 8 * g + (i >> 2);
    const int slot = ((r0 + 4 * (i & 3)) >> 2) ^ tr_swz<R>(k);
    const uint8_t* p = img + k * RB + slot * 8;
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(p));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(p + 4 * RB));
    s8v r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  }
}

constexpr float kBeta = 0.7978845608028654f;  // sqrt(2/pi)
constexpr float kKappa = 0.044715f;
// tanh(u) = 2σ(2u) − 1 with σ from v_exp_f32 + one reciprocal (libm tanhf's branchy slow path
// made the fused epilogue cost as much as a separate elementwise pass)
__device__ __forceinline__ float sig2(float u) { return __fdividef(1.f, 1.f + __expf(-2.f * u)); }
__device__ __forceinline__ float sigm(float x) { return __fdividef(1.f, 1.f + __expf(-x)); }
// The epilogue forms fold the constants: σ(2u) = 1 / (1 + 2^z), z = x·(c1 + c2·x²) with
// c1 = −2β·log2(e), c2 = −2βκ·log2(e) — 5 VALU + v_exp_f32 + v_rcp_f32 per element (the plain
// form above compiled to ~9 VALU + the two transcendentals; the GELU / GELU′ epilogues run 25 M
// of them per c_fc product)
constexpr float kLog2eF = 1.4426950408889634f;
constexpr float kGc1 = -2.f * kBeta * kLog2eF, kGc2 = -2.f * kBeta * kKappa * kLog2eF;
__device__ __forceinline__ float sig2_of(float x, float x2) {  // σ(2u(x)), x2 = x·x
  const float z = x * fmaf(kGc2, x2, kGc1);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z));
}
__device__ __forceinline__ float gelu_tanh(float x) {  // 0.5x(1 + tanh u) = x·σ(2u)
  return x * sig2_of(x, x * x);
}
__device__ __forceinline__ float dgelu_tanh(float x) {  // d gelu / dx = s + 2x·s(1−s)·β(1 + 3κx²), s = σ(2u)
  const float x2 = x * x;
  const float s = sig2_of(x, x2);
  const float w = x * fmaf(6.f * kBeta * kKappa, x2, 2.f * kBeta);  // 2xβ(1 + 3κx²)
  return fmaf(w, s - s * s, s);
}

// XCD-aware bijective remap of blockIdx.x (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"), then groups of G tile rows sweeping the column tiles, so the workgroups sharing
// an A row panel run on the same XCD's L2.
template <int G>
__device__ __forceinline__ void tile_coords(int tiles_m, int tiles_n, int& tm, int& tn, int id = -1) {
  const int nwg = tiles_m * tiles_n;
  int bid = id < 0 ? (int)blockIdx.x : id;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int per_group = G * tiles_n;
  const int first_m = (bid / per_group) * G;
  const int gsz = min(tiles_m - first_m, G);
  const int local = bid % per_group;
  tm = first_m + local % gsz;
  tn = local / gsz;
}

// out[i] = Σ_s ws[s][i] as bf16 (fixed order: deterministic); defined in gemm.hip
__global__ __launch_bounds__(256) void reduce_kernel(const float* __restrict__ ws, int splits, int64_t n8, int64_t slab,
                              uint16_t* __restrict__ out, int64_t m8, uint16_t* __restrict__ rs_out, int accum);

// gemm256.hip: the 256x256 phase-interleaved kernel for (a_km, b_kn, epi); grid (tiles, splits)
void launch_gemm256(const Args& p, bool a_km, bool b_kn, int epi, dim3 grid, hipStream_t st, int variant);

}  // namespace gemm
}  // namespace nbd
