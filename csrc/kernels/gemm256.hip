// gemm256.hip — 256x256-tile bf16 GEMM for the large products (the LM head's forward, input-
// and weight-gradient GEMMs: 8192 x 50k x 768), on v_mfma_f32_16x16x32_bf16.
//
// Same operand layouts, LDS image swizzles and fragment reads as gemm.hip (gemm_common.h); what
// differs is the schedule, built for one 512-thread workgroup per CU
// (cdna_hip_programming.md §5 "The 256² 8-phase template" + T3/T4/T5):
//   * 8 waves as 2 (M) x 4 (N); wave (wm, wn) owns rows wm·128.. and columns wn·64.. of the tile
//     and computes them as 4 quadrants of 64 x 32 (4 x 2 fragments x K 64 = 16 MFMAs each).
//   * Each operand K-tile is staged as two HALF images: A half h holds the 64-row halves h of
//     both waves' 128-row bands, B half h the 32-column halves h of the four 64-column bands —
//     so each half is read by exactly one quadrant row (A) or column (B) and frees up early.
//   * One K-tile = 4 phases, one quadrant each: {LDS fragment reads for the quadrant, issue the
//     DMA of a freed half of tile t+2} -> s_barrier -> lgkmcnt(0) -> 16 MFMAs at priority 1 ->
//     s_barrier.  Quadrant order (0,0) (0,1) (1,1) (1,0) with one register set per operand:
//     12 / 4 / 8 / 4 fragment reads (ds_read_b128 or 2 x ds_read_b64_tr_b16) per phase.
//   * Two LDS buffers (2 x 64 KiB).  Each half of tile t+2 goes into tile t's buffer once its
//     last reader phase has passed a barrier: A0 in phase 2, B1 in phase 3, A1 in phase 4, B0 in
//     phase 1 of tile t+1; phase 4 then waits with a COUNTED vmcnt(6) — tile t+1 landed, three
//     halves (6 DMAs per lane) of tile t+2 stay in flight across the barriers (never vmcnt(0) in
//     steady state).  Reads of tile t+1 start one phase after that wait (the "read a staged
//     buffer one phase AFTER the wait that retires it" rule).
//   * Epilogue through LDS as a bf16 [256][256] tile (bias added in fp32 first): 16-B row-
//     contiguous global stores; GELU / GELU′ applied on the way out.  Split-K (grid.y) writes
//     fp32 slabs straight from the accumulators; gemm.hip's reduce_kernel sums them.
#include <c10/util/Exception.h>

#include <type_traits>

#include "gemm_common.h"

namespace nbd {
namespace gemm {
namespace g256 {

constexpr int BM = 256, BN = 256, NTH = 512;
constexpr int HALF = 128 * BK * 2;  // one half image: 128 rows (or columns) x 64 k = 16 KiB
constexpr int BUF = 4 * HALF;       // A0 A1 B0 B1 = 64 KiB per K-tile buffer
constexpr int CST = BN * 2 + 16;    // epilogue bf16 C-tile row stride: +16 B keeps the 8-B writes conflict-free
constexpr int BYTES = (2 * BUF > BM * CST) ? 2 * BUF : BM * CST;

// image row lr of half X <-> tile row: bands of 2·GRP rows, half X is rows X·GRP.. of each band
template <int GRP>
__device__ __forceinline__ int hmap(int lr, int X) {
  return (lr / GRP) * (2 * GRP) + X * GRP + (lr % GRP);
}

// DMA one half image (16 KiB = 16 wave-pieces of 1 KiB; 2 per wave).  Row image [128][64] or
// tr image [64][128], the same swizzles as gemm_common.h's Pieces<128, TR, 8>.  The per-lane part
// of each piece's source address is a 32-bit byte offset computed once per kernel (HalfPieces);
// each stage only moves the wave-uniform base (SGPRs) — the saddr form of the DMA (glds16s).
// With 64-bit per-lane pointers the transposed layouts ran out of VGPRs: hipcc spilled three
// of them inside the K-loop and each reload's vmcnt(0) drained the DMA pipeline (docs/FINDINGS.md
// §33).
template <bool TR, int GRP>
struct HalfPieces {
  uint32_t off[2][2];  // [half X][piece]
  __device__ __forceinline__ HalfPieces(int64_t ld, int wave, int lane) {
#pragma unroll
    for (int X = 0; X < 2; ++X)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int byte = (i * 8 + wave) * 1024 + lane * 16;
        int64_t e;
        if constexpr (!TR) {
          const int r = byte >> 7, pc = (byte >> 4) & 7;
          e = (int64_t)hmap<GRP>(r, X) * ld + 8 * (pc ^ row_swz(r));
        } else {
          const int k = byte >> 8, pc = (byte & 255) >> 4;
          const int lc = 8 * (pc ^ (tr_swz<128>(k) >> 1));
          e = (int64_t)k * ld + hmap<GRP>(lc, X);
        }
        off[X][i] = (uint32_t)(2 * e);
      }
  }
  // K-tile at k0 of the operand rows (columns, TR) r0.. into img
  __device__ __forceinline__ void stage(const uint16_t* g, int64_t ld, int r0, int k0, uint8_t* img, int X,
                                        int wave) const {
    const uint16_t* base = TR ? g + (int64_t)k0 * ld + r0 : g + (int64_t)r0 * ld + k0;
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16s(base, off[X][i], img + (i * 8 + wave) * 1024);
  }
};

// Phase boundaries.  The LDS reads of a phase must be complete before its closing barrier (the
// WAR guard for the next DMA into the half they read): V = 0 waits lgkmcnt(0) right after the
// opening barrier (the template's order); V = 1, 2 let the compiler's counted waits feed the
// first MFMAs early and drain the reads only at the phase end (V = 2 without the s_setprio pair).
// V >= 4 STAGGER the two wave groups by one barrier (waves 4-7, the M-half wm = 1, run one
// barrier behind): the two waves sharing a SIMD (w and w+4) then alternate — one issues its
// MFMAs while the other reads its next fragments — and the reads are drained BEFORE the
// opening barrier, so a half is still free one phase after its last read in both groups
// (MI355X_MICROARCH.md "Two waves per SIMD"; cdna_hip_programming.md §5 template, `if(wr==1)
// s_barrier`).  V = 4 keeps the per-cluster setprio pair; V = 5 sets priority 1 once for the
// lagging group instead (T5 static form).
template <int V>
__device__ __forceinline__ void phase_open() {
  if constexpr (V >= 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if constexpr (V == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (V != 2 && V != 5) __builtin_amdgcn_s_setprio(1);
}
template <int V>
__device__ __forceinline__ void phase_close() {
  if constexpr (V == 1 || V == 2 || V == 3) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if constexpr (V != 2 && V != 5) __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return pack2_bf16(a, b);
}

// NTS: the C tile leaves with non-temporal stores (an output far larger than the L2s and the
// MALL — the LM head's logits — gains nothing from being cached on its way out: LM-head forward
// 659 -> 611 us, docs/FINDINGS.md §33).  Split-K slabs keep plain stores: the reduce kernel reads
// them right back.
template <bool A_KM, bool B_KN, int EPI, int V, bool NTS = false>
__global__ __launch_bounds__(NTH, 2) void kernel(Args p) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[BYTES];  // one LDS object (guide §5 item 4a)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  int tm, tn;
  tile_coords<8>(p.tiles_m, p.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int64_t kz = (int64_t)blockIdx.y * p.K;  // split-K: this split's K range
  const uint16_t* A = p.a + (A_KM ? kz * p.lda : kz);
  const uint16_t* B = p.b + (B_KN ? kz * p.ldb : kz);

  f4 acc[2][2][2][4];  // [quadrant mh][quadrant nh][n fragment][m fragment]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[a][b][i][j] = f4{0.f, 0.f, 0.f, 0.f};
  s8v af[2][4], bf[2][2], bq[2][2];  // [kk][fragment]: A, B (and, V = 3, the B0 fragments kept)

  const HalfPieces<A_KM, 64> pa(p.lda, wave, lane);
  const HalfPieces<B_KN, 32> pb(p.ldb, wave, lane);
  auto stage_a = [&](int t, uint8_t* buf, int X) { pa.stage(A, p.lda, m0, t * BK, buf + X * HALF, X, wave); };
  auto stage_b = [&](int t, uint8_t* buf, int X) { pb.stage(B, p.ldb, n0, t * BK, buf + (2 + X) * HALF, X, wave); };
  auto read_a = [&](const uint8_t* buf, int X) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j) af[kk][j] = frag<128, A_KM>(buf + X * HALF, wm * 64 + 16 * j, kk, lane);
  };
  auto read_b = [&](const uint8_t* buf, int X, s8v(&b)[2][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i) b[kk][i] = frag<128, B_KN>(buf + (2 + X) * HALF, wn * 32 + 16 * i, kk, lane);
  };
  auto mma = [&](f4(&c)[2][4], const s8v(&b)[2][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[kk][i], af[kk][j], c[i][j], 0, 0, 0);
  };

  const int nk = p.K / BK;
  // prologue: tiles 0 and 1 in flight, tile 0 landed
  stage_a(0, smem, 0); stage_b(0, smem, 0); stage_b(0, smem, 1); stage_a(0, smem, 1);
  if (nk > 1) {
    stage_a(1, smem + BUF, 0); stage_b(1, smem + BUF, 0); stage_b(1, smem + BUF, 1); stage_a(1, smem + BUF, 1);
    vm_wait<8>();  // tile 0 landed
  } else {
    vm_wait<0>();
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  // stagger (V >= 4): the lagging group (waves 4-7; readfirstlane keeps the branch scalar)
  // passes one extra barrier now and the leading group one after the loop
  const bool lagging = __builtin_amdgcn_readfirstlane(threadIdx.x) >= NTH / 2;
  if constexpr (V >= 4) {
    if (lagging) {
      if constexpr (V == 5) __builtin_amdgcn_s_setprio(1);
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("" ::: "memory");
  }

  // one K-tile (buffer CUR): 4 phases; the buffer index is a compile-time constant so the
  // compiler sees every LDS offset
  auto tile = [&](int t, auto cur_c) {
    constexpr int CUR = decltype(cur_c)::value;
    constexpr bool KEEP_B0 = V == 3;  // B0 fragments stay in registers (no phase-4 re-read)
    uint8_t* buf = smem + CUR * BUF;
    const bool pre = t + 2 < nk;
    s8v(&b0)[2][2] = KEEP_B0 ? bq : bf;
    // phase 1: quadrant (0,0) — reads A0, B0.  (Re-read B0:) B0 of tile t+1 goes into the other
    // buffer (its last reader, phase 4 of tile t-1, has passed a barrier; tile 1's came with the
    // prologue).
    read_b(buf, 0, b0);
    read_a(buf, 0);
    if (!KEEP_B0 && t >= 1 && t + 1 < nk) stage_b(t + 1, smem + (CUR ^ 1) * BUF, 0);
    phase_open<V>();
    mma(acc[0][0], b0);
    phase_close<V>();
    // phase 2: quadrant (0,1) — reads B1; A0 (and, kept, B0) are free: tile t+2's go in
    read_b(buf, 1, bf);
    if (pre) {
      stage_a(t + 2, buf, 0);
      if (KEEP_B0) stage_b(t + 2, buf, 0);
    }
    phase_open<V>();
    mma(acc[0][1], bf);
    phase_close<V>();
    // phase 3: quadrant (1,1) — reads A1; B1 is free
    read_a(buf, 1);
    if (pre) stage_b(t + 2, buf, 1);
    phase_open<V>();
    mma(acc[1][1], bf);
    phase_close<V>();
    // phase 4: quadrant (1,0) — (re-)reads B0; A1 is free.  Retire tile t+1: the younger DMAs of
    // tile t+2 (3 halves = 6 per lane; 4 halves = 8 with B0 kept) stay in flight; the first
    // reads of tile t+1 are in the next phase.
    if (!KEEP_B0) read_b(buf, 0, b0);
    if (pre) {
      stage_a(t + 2, buf, 1);
      vm_wait<KEEP_B0 ? 8 : 6>();
    } else {
      vm_wait<0>();
    }
    phase_open<V>();
    mma(acc[1][0], b0);
    phase_close<V>();
  };
  for (int t = 0; t < nk; t += 2) {
    tile(t, std::integral_constant<int, 0>{});
    if (t + 1 < nk) tile(t + 1, std::integral_constant<int, 1>{});
  }
  if constexpr (V >= 4) {
    if (!lagging) __builtin_amdgcn_s_barrier();
    if constexpr (V == 5) __builtin_amdgcn_s_setprio(0);
    asm volatile("" ::: "memory");
  }

  // ---- epilogue (every DMA retired: the last tile waited vmcnt(0)) ----------------------------
  // acc[mh][nh][i][j] element e = C[row][col + e], row = wm·128 + mh·64 + 16j + (lane&15),
  // col = wn·64 + nh·32 + 16i + 4(lane>>4)
  const int lr = lane & 15, lc = 4 * (lane >> 4);
  if (gridDim.y > 1) {
    float* slab = p.ws + (int64_t)blockIdx.y * p.M * p.ldc;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = wm * 128 + a * 64 + 16 * j + lr, col = wn * 64 + b * 32 + 16 * i + lc;
            *reinterpret_cast<f4*>(slab + (int64_t)(m0 + row) * p.ldc + n0 + col) = acc[a][b][i][j];
          }
    return;
  }
  const bool bias = EPI != EPI_DGELU && p.bias != nullptr;
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int col = wn * 64 + b * 32 + 16 * i + lc;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (bias) {
        const uint2 w = *reinterpret_cast<const uint2*>(p.bias + n0 + col);
        bv[0] = __uint_as_float(w.x << 16); bv[1] = __uint_as_float(w.x & 0xffff0000u);
        bv[2] = __uint_as_float(w.y << 16); bv[3] = __uint_as_float(w.y & 0xffff0000u);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = wm * 128 + a * 64 + 16 * j + lr;
          const f4 v = acc[a][b][i][j];
          uint2 w;
          w.x = pack2(v[0] + bv[0], v[1] + bv[1]);
          w.y = pack2(v[2] + bv[2], v[3] + bv[3]);
          *reinterpret_cast<uint2*>(smem + row * CST + col * 2) = w;
        }
    }
  __syncthreads();
  constexpr int CPR = BN / 8;  // 16-B chunks per row
  for (int c = threadIdx.x; c < BM * CPR; c += NTH) {
    const int r = c / CPR, cn = (c % CPR) * 8;
    float v[8];
    load8<bf16_t>(reinterpret_cast<const bf16_t*>(smem + r * CST + cn * 2), v);
    const int64_t off = (int64_t)(m0 + r) * p.ldc + n0 + cn;
    if constexpr (EPI == EPI_GELU) {
      store8<bf16_t>(reinterpret_cast<bf16_t*>(p.aux_out) + off, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = gelu_tanh(v[e]);
    } else if constexpr (EPI == EPI_DGELU) {
      float h[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(p.aux_in) + off, h);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= dgelu_tanh(h[e]);
    }
    if constexpr (NTS) store8_nt<bf16_t>(reinterpret_cast<bf16_t*>(p.c) + off, v);
    else store8<bf16_t>(reinterpret_cast<bf16_t*>(p.c) + off, v);
  }
}

template <bool A_KM, bool B_KN, int V>
static void launch_layout(const Args& p, int epi, dim3 grid, hipStream_t st) {
  switch (epi) {
    case EPI_NONE:
      hipLaunchKernelGGL((kernel<A_KM, B_KN, EPI_NONE, V>), grid, dim3(NTH), 0, st, p);
      return;
    case EPI_GELU:
      if constexpr (!A_KM && !B_KN) {
        hipLaunchKernelGGL((kernel<false, false, EPI_GELU, V>), grid, dim3(NTH), 0, st, p);
        return;
      }
      break;
    case EPI_DGELU:
      if constexpr (!A_KM && B_KN) {
        hipLaunchKernelGGL((kernel<false, true, EPI_DGELU, V>), grid, dim3(NTH), 0, st, p);
        return;
      }
      break;
    default: break;
  }
  TORCH_CHECK(false, "nbd::gemm: the 256x256 kernel has no epilogue ", epi, " for this layout");
}

template <bool A_KM, bool B_KN>
static void launch_nts(const Args& p, dim3 grid, hipStream_t st) {
  hipLaunchKernelGGL((kernel<A_KM, B_KN, EPI_NONE, 4, true>), grid, dim3(NTH), 0, st, p);
}

template <int V>
static void launch_v(const Args& p, bool a_km, bool b_kn, int epi, dim3 grid, hipStream_t st) {
  if (!a_km && !b_kn)
    launch_layout<false, false, V>(p, epi, grid, st);
  else if (!a_km && b_kn)
    launch_layout<false, true, V>(p, epi, grid, st);
  else
    launch_layout<true, true, V>(p, epi, grid, st);
}

}  // namespace g256

// variant (tile code "stages" digit - 2): schedule experiments, see phase_open / tile; 6 = 4 with
// non-temporal C stores
void launch_gemm256(const Args& p, bool a_km, bool b_kn, int epi, dim3 grid, hipStream_t st, int variant) {
  TORCH_CHECK(p.M % 256 == 0 && p.N % 256 == 0 && p.K % BK == 0, "nbd::gemm: 256x256 tiles need M, N % 256 == 0");
  TORCH_CHECK(grid.y == 1 || epi == EPI_NONE, "nbd::gemm: 256x256 split-K only without an epilogue");
  // every caller of this entry point passes one of the three built layouts; (A [K][M], B [N][K])
  // has no instantiation (launch_v / launch_nts would run the <true, true> kernel on it)
  TORCH_CHECK(!(a_km && !b_kn), "nbd::gemm: the 256x256 kernel has no (A [K][M], B [N][K]) layout");
  if (variant == 6) {  // 4 with non-temporal C stores (plain products; split-K slabs stay cached:
                       // the slab path returns before the C-tile stores)
    TORCH_CHECK(epi == EPI_NONE, "nbd::gemm: variant 6 stores plain products");
    if (!a_km && !b_kn)
      g256::launch_nts<false, false>(p, grid, st);
    else if (!a_km && b_kn)
      g256::launch_nts<false, true>(p, grid, st);
    else
      g256::launch_nts<true, true>(p, grid, st);
    return;
  }
  switch (variant) {
    case 1: g256::launch_v<1>(p, a_km, b_kn, epi, grid, st); break;
    case 2: g256::launch_v<2>(p, a_km, b_kn, epi, grid, st); break;
    case 3: g256::launch_v<3>(p, a_km, b_kn, epi, grid, st); break;
    case 4: g256::launch_v<4>(p, a_km, b_kn, epi, grid, st); break;
    case 5: g256::launch_v<5>(p, a_km, b_kn, epi, grid, st); break;
    default: g256::launch_v<0>(p, a_km, b_kn, epi, grid, st); break;
  }
}

}  // namespace gemm
}  // namespace nbd
