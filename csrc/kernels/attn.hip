// attn.hip — flash attention (forward + backward) for gfx950, head dim 64, bf16, optional causal.
//
// Used by the GPT-2 DDP workload (12 heads x 64, T = 1024): torch's SDPA path on this image ran
// at 5–7 % of the MFMA roof there (rocprof: attn_fwd 77 µs, bwd_kernel_dk_dv + dq 272 µs per
// layer, profiles/gpt2_step_rocprof_r1.md).  Everything below is v_mfma_f32_32x32x16_bf16 with
// the operand maps of cdna_hip_programming.md §3:
//   A: lane l (r = l&31, h = l>>5) holds A[r][8h + j];  B: lane l holds B[8h + j][r];
//   C/D (16 f32 per lane): col = l&31, row = (i&3) + 8(i>>2) + 4h  for register i.
//
// Forward (one workgroup = 4 waves = 128 queries of one (batch, head); a wave owns 32 queries):
//   S^T[key][q] = K·Q^T with the query on the lane, so each lane owns one query row's scores
//   (softmax max / sum = in-lane over 32 registers + one lane^32 exchange) and the S^T
//   accumulator, packed to bf16, is directly the B operand of O^T[d][q] += V^T[d][key]·P[key][q]
//   (§3 "accumulator tile as the next MFMA's operand").  Q lives in registers; K tiles in LDS
//   (144-B rows: conflict-free ds_read_b128 row reads); V tiles in LDS read transposed with
//   ds_read_b64_tr_b16 (T10).  The next K/V tile is fetched into registers while the current one
//   is computed (T14 issue-early / write-late), one LDS buffer.
// Backward (FA2 split, no atomics, deterministic):
//   pre   δ[q] = Σ_d dO·O
//   dkdv  one workgroup = 128 keys, wave = 32 keys on the lane; sweeps 64-query tiles:
//         S = Q·K^T, P = exp2(S·c − lse₂), dV^T += dO^T·P, dP = dO·V^T, dS = P(dP − δ),
//         dK^T += Q^T·dS — dK/dV stay in 64 accumulator registers; K, V in registers.
//   dq    one workgroup = 128 queries, wave = 32 queries on the lane; sweeps 64-key tiles:
//         S^T = K·Q^T, dP^T = V·dO^T, dS^T = P^T(dP^T − δ), dQ^T += K^T·dS^T.
// Causal: workgroups are launched heaviest-first; fully masked tiles are skipped per wave, and
// the mask is applied only to the 32x32 blocks the diagonal crosses (wave-uniform branches).
// Forward: the O / l rescale is deferred while the running max grows by <= 2^kDeferLog2.
// GQA: query head h reads key/value head h / group; dkdv runs per key/value head and sweeps its
// group of query heads, accumulating dK/dV in the same registers (no atomics).
// RoPE (optional, Llama family): q and k are rotated as they are loaded (Q/K fragments in
// registers; K/Q tiles between the global load and the LDS store, one thread holding both halves
// of a row chunk) and dQ/dK get the transpose rotation in the store epilogue — the packed
// projection stays unrotated and no separate rotary kernels or gradient copies run.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <numeric>
#include <queue>
#include <tuple>
#include <vector>
#include <type_traits>

#include "nbd_common.h"

namespace nbd {
namespace attn {

typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f16x __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

constexpr int D = 64;
constexpr int NT = 256;     // threads per workgroup (4 waves)
constexpr int BLK = 128;    // rows owned by a workgroup (queries in fwd/dq, keys in dkdv)
constexpr int TILE = 64;    // rows per swept tile
constexpr int RS = 72;      // LDS row stride (elements) of row-read images: 144 B
constexpr int RSV = 96;     // LDS row stride of transpose-only images: 192 B (tr reads conflict-free)
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kDeferLog2 = 4.f;  // forward: skip the O rescale while the max grows by <= 2^4

struct View {
  const uint16_t* p;
  int64_t sb, sh, st;  // element strides of batch, head, row; d is contiguous
  __device__ __forceinline__ const uint16_t* row(int b, int h, int t) const { return p + b * sb + h * sh + t * st; }
};
struct MView {
  uint16_t* p;
  int64_t sb, sh, st;
  __device__ __forceinline__ uint16_t* row(int b, int h, int t) const { return p + b * sb + h * sh + t * st; }
};

__device__ __forceinline__ f16x mfma(s8v a, s8v b, f16x c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ s8v ld16(const uint16_t* p) { return *reinterpret_cast<const s8v*>(p); }
__device__ __forceinline__ void st16(uint16_t* p, s8v v) { *reinterpret_cast<s8v*>(p) = v; }
__device__ __forceinline__ s4v tr4(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(p));
}
__device__ __forceinline__ s8v cat(s4v a, s4v b) {
  s8v r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
__device__ __forceinline__ uint16_t bf(float x) { return f32_to_bf16(x); }
// registers 8s .. 8s+7 of a C tile -> bf16 B/A fragment of k-step s (k order as §3)
__device__ __forceinline__ s8v pack_half(const f16x& c, int s) {
  u32x4 w;
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = pack2_bf16(c[8 * s + 2 * j], c[8 * s + 2 * j + 1]);
  return __builtin_bit_cast(s8v, w);
}
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
__device__ __forceinline__ f16x zero16() {
  f16x z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// store a 32x32 C tile whose rows are d (= db*32 + row) and columns a row index of `out`
// (lane&31): 4 consecutive d per 8-byte store
__device__ __forceinline__ void store_dT(uint16_t* rowp, const f16x& c, int db, int h, float mul) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const uint32_t lo = pack2_bf16(c[4 * g] * mul, c[4 * g + 1] * mul);
    const uint32_t hi = pack2_bf16(c[4 * g + 2] * mul, c[4 * g + 3] * mul);
    const int d = db * 32 + 8 * g + 4 * h;
    *reinterpret_cast<uint2*>(rowp + d) = make_uint2(lo, hi);
  }
}

// rotary embedding fused into the loads (HF rotate_half convention): dims d and d+32 of a row
// rotate by the angle of (row position, d); cos/sin = [T_max, 32] fp32 tables, nullptr = no RoPE
struct Rope {
  const float* cos;
  const float* sin;
};

// rotate 8 consecutive dims [d0, d0+8) of x (with their partners d+32 in y) for position t
__device__ __forceinline__ void rope8(s8v& x, s8v& y, const Rope& rp, int t, int d0) {
  const float4* c4 = reinterpret_cast<const float4*>(rp.cos + (int64_t)t * 32 + d0);
  const float4* s4 = reinterpret_cast<const float4*>(rp.sin + (int64_t)t * 32 + d0);
  const float4 ca = c4[0], cb = c4[1], sa = s4[0], sb = s4[1];
  const float c[8] = {ca.x, ca.y, ca.z, ca.w, cb.x, cb.y, cb.z, cb.w};
  const float sn[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float a = bf16_to_f32((uint16_t)x[j]), b = bf16_to_f32((uint16_t)y[j]);
    x[j] = (short)bf(a * c[j] - b * sn[j]);
    y[j] = (short)bf(b * c[j] + a * sn[j]);
  }
}

// Q or K fragments of one row held in registers (element s covers dims 16s + 8h + [0, 8)):
// pairs (f[0], f[2]) and (f[1], f[3])
__device__ __forceinline__ void rope_frag(s8v (&f)[4], const Rope& rp, int t, int h) {
  rope8(f[0], f[2], rp, t, 8 * h);
  rope8(f[1], f[3], rp, t, 16 + 8 * h);
}

// dQ/dK tiles: acc0 holds dims [0, 32), acc1 dims [32, 64) — a d/d+32 pair shares register i of
// one lane, so the transpose rotation (gradient of the forward rotation) is applied right here
__device__ __forceinline__ void store_dT_rope(uint16_t* rowp, const f16x& a0, const f16x& a1, int h, float mul,
                                              const Rope& rp, int t) {
  const float* cr = rp.cos + (int64_t)t * 32;
  const float* sr = rp.sin + (int64_t)t * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint16_t lo[4], hi[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int d = 8 * g + 4 * h + e;
      const float x = a0[4 * g + e] * mul, y = a1[4 * g + e] * mul;
      lo[e] = bf(x * cr[d] + y * sr[d]);
      hi[e] = bf(y * cr[d] - x * sr[d]);
    }
    const int d = 8 * g + 4 * h;
    *reinterpret_cast<uint2*>(rowp + d) =
        make_uint2((uint32_t)lo[0] | ((uint32_t)lo[1] << 16), (uint32_t)lo[2] | ((uint32_t)lo[3] << 16));
    *reinterpret_cast<uint2*>(rowp + 32 + d) =
        make_uint2((uint32_t)hi[0] | ((uint32_t)hi[1] << 16), (uint32_t)hi[2] | ((uint32_t)hi[3] << 16));
  }
}

// tile staging with the two halves of a row in one thread (row = tid/4, chunks q and q+4), so
// the rotation can be applied between the global load and the LDS store
struct StagePair {
  s8v a, b;
  __device__ __forceinline__ void load(const uint16_t* base, int64_t st, int tid) {
    const uint16_t* p = base + (tid >> 2) * st + (tid & 3) * 8;
    a = ld16(p);
    b = ld16(p + 32);
  }
  __device__ __forceinline__ void rope(const Rope& rp, int t0, int tid) {
    if (rp.cos != nullptr) rope8(a, b, rp, t0 + (tid >> 2), (tid & 3) * 8);
  }
  __device__ __forceinline__ void store(uint16_t* lds, int stride, int tid) const {
    uint16_t* p = lds + (tid >> 2) * stride + (tid & 3) * 8;
    st16(p, a);
    st16(p + 32, b);
  }
};

// cooperative tile staging: 64 rows x 64 d, 512 16-B chunks, 2 per thread
struct Stage2 {
  s8v a[2];
  __device__ __forceinline__ void load(const uint16_t* base, int64_t st, int tid) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * NT;
      a[i] = ld16(base + (c >> 3) * st + (c & 7) * 8);
    }
  }
  __device__ __forceinline__ void store(uint16_t* lds, int stride, int tid) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + i * NT;
      st16(lds + (c >> 3) * stride + (c & 7) * 8, a[i]);
    }
  }
};

// ============================================================================ forward
template <bool CAUSAL>
__global__ __launch_bounds__(NT, 2) void fwd_kernel(View q, View k, View v, MView o, float* __restrict__ lse,
                                                     int H, int T, int nblk, float sc2, int group, Rope rp,
                                                     const int* __restrict__ order) {
  __shared__ __attribute__((aligned(16))) uint16_t Ks[TILE * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[TILE * RSV];
  // work item (heaviest first under a causal mask); `order` places the items on the CUs (host: block_order)
  const int item = order != nullptr ? order[blockIdx.x] : (int)blockIdx.x;
  const int bh = item % (gridDim.x / nblk);
  const int qb = CAUSAL ? nblk - 1 - item / (gridDim.x / nblk) : item / (gridDim.x / nblk);
  const int b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int q0 = qb * BLK + w * 32;  // this wave's first query
  const int qi = q0 + r;             // this lane's query
  const int kh = hh / group;         // GQA: the key/value head of this query head
  s8v qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = ld16(q.row(b, hh, qi) + 16 * s + 8 * h);
  if (rp.cos != nullptr) rope_frag(qf, rp, qi, h);
  f16x acc_o[2] = {zero16(), zero16()};
  float m = -INFINITY, l = 0.f;
  const int ntiles = CAUSAL ? (qb * BLK + BLK) / TILE : T / TILE;
  StagePair sk;
  Stage2 sv;
  sk.load(k.row(b, kh, 0), k.st, tid);
  sv.load(v.row(b, kh, 0), v.st, tid);
  sk.rope(rp, 0, tid);
  sk.store(Ks, RS, tid);
  sv.store(Vs, RSV, tid);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) {  // issue the next tile's loads now, write them after this tile
      sk.load(k.row(b, kh, (t + 1) * TILE), k.st, tid);
      sv.load(v.row(b, kh, (t + 1) * TILE), v.st, tid);
    }
    const int k0 = t * TILE;
    // one tile; DIAG = the causal mask cuts through it (only those tiles pay for the compares)
    auto tile_body = [&](auto diag_c) {
      constexpr bool DIAG = decltype(diag_c)::value;
      // DIAG: the tile's second 32-key block lies wholly past this wave's queries for waves whose
      // diagonal falls in the first (skip1: no S / P·V MFMAs, P = 0), and a block wholly before
      // them needs no mask — only the block the diagonal crosses pays the compares (wave-uniform)
      const bool skip1 = DIAG && k0 + 32 > q0 + 31;
      f16x sacc[2] = {zero16(), zero16()};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        if (kb == 1 && skip1) break;
#pragma unroll
        for (int s = 0; s < 4; ++s) sacc[kb] = mfma(ld16(Ks + (kb * 32 + r) * RS + 16 * s + 8 * h), qf[s], sacc[kb]);
      }
      // running max on the raw scores (sc2 > 0), scaled once; p = exp2(s·sc2 − m) as one FMA + exp
      float mt = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        if constexpr (DIAG) {
          if (kb == 1 && skip1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) sacc[1][i] = -INFINITY;
            continue;
          }
          if (k0 + kb * 32 + 31 > q0) {  // the diagonal crosses this block
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if (k0 + kb * 32 + crow(i, h) > qi) sacc[kb][i] = -INFINITY;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) mt = fmaxf(mt, sacc[kb][i]);
      }
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64));
      // deferred rescale (cdna_hip_programming.md T13): the O / l rescale by exp2(m − m') runs
      // only when some query of the wave saw its running max grow by more than kDeferLog2;
      // otherwise the stale max is kept and this tile's p are bounded by 2^kDeferLog2 (bf16's
      // relative precision does not depend on the magnitude; O and l accumulate in fp32)
      const float mn = fmaxf(m, mt * sc2);
      if (__any(mn > m + kDeferLog2)) {
        const float alpha = __builtin_amdgcn_exp2f(m - mn);
        l *= alpha;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc_o[db][i] *= alpha;
        m = mn;
      }
      const float nmn = -m;
      float rs0 = 0.f, rs1 = 0.f;  // two chains; scalar adds (no v_pk_add_f32: -fno-slp-vectorize)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const float p0 = __builtin_amdgcn_exp2f(fmaf(sacc[kb][i], sc2, nmn));
          const float p1 = __builtin_amdgcn_exp2f(fmaf(sacc[kb][i + 1], sc2, nmn));
          sacc[kb][i] = p0;
          sacc[kb][i + 1] = p1;
          rs0 += p0;
          rs1 += p1;
        }
      float rs = rs0 + rs1;
      rs += __shfl_xor(rs, 32, 64);
      l += rs;
      // O^T[d][q] += V^T[d][key] . P[key][q]
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        if (kb == 1 && skip1) break;  // P = 0 there
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const s8v pb = pack_half(sacc[kb], s);
          const int key = kb * 32 + 16 * s + 4 * h + (lane & 15) / 4;
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            const uint16_t* base = Vs + key * RSV + db * 32 + (lane & 16) + 4 * (lane & 3);
            acc_o[db] = mfma(cat(tr4(base), tr4(base + 8 * RSV)), pb, acc_o[db]);
          }
        }
      }
    };
    if (!CAUSAL || k0 <= q0 + 31) {
      if (CAUSAL && k0 + TILE - 1 > q0)
        tile_body(std::true_type{});
      else
        tile_body(std::false_type{});
    }
    __syncthreads();
    if (t + 1 < ntiles) {
      sk.rope(rp, (t + 1) * TILE, tid);
      sk.store(Ks, RS, tid);
      sv.store(Vs, RSV, tid);
      __syncthreads();
    }
  }
  const float inv = 1.f / l;
  uint16_t* orow = o.row(b, hh, qi);
  store_dT(orow, acc_o[0], 0, h, inv);
  store_dT(orow, acc_o[1], 1, h, inv);
  if (h == 0) lse[(int64_t)bh * T + qi] = (m + __log2f(l)) * kLn2;
}

// ============================================================================ backward: δ
// δ[row] = Σ_d dO·O: 8 lanes per row, each a 16-B chunk of dO and of O (one 128-B line per row
// and operand: coalesced), reduced over the 8 lanes; 32 rows per workgroup
__global__ __launch_bounds__(NT) void bwd_pre_kernel(View dout, View out, float* __restrict__ delta, int H, int T,
                                                     int64_t rows) {
  const int64_t i = (int64_t)blockIdx.x * (NT / 8) + (threadIdx.x >> 3);
  const int c = threadIdx.x & 7;
  float acc = 0.f;
  if (i < rows) {
    const int t = (int)(i % T);
    const int64_t bh = i / T;
    const int b = (int)(bh / H), hh = (int)(bh % H);
    float x[8], y[8];
    load8<bf16_t>(reinterpret_cast<const bf16_t*>(dout.row(b, hh, t) + 8 * c), x);
    load8<bf16_t>(reinterpret_cast<const bf16_t*>(out.row(b, hh, t) + 8 * c), y);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc = fmaf(x[e], y[e], acc);
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (i < rows && c == 0) delta[i] = acc;
}

// ============================================================================ backward: dK, dV
// Block `blk` of `nblocks` (= B·H·gsplit·nblk).  gsplit > 1 (GQA with few key/value heads):
// the `group` query heads of a key/value head are split over gsplit workgroups, each writing a
// partial dK/dV (split index s at dk/dv + s·split_stride) that gqa_reduce_kernel sums — 3x the
// workgroups for SmolLM2 (9 query / 3 kv heads) instead of one workgroup sweeping all 3 heads.
// δ of a 64-row tile from register-staged dO and O chunks (Stage2 mapping: chunk c = tid + i·NT
// is row c/8, dims 8(c%8)..+8): 8-element partial dot, summed over the row's 8 consecutive lanes
__device__ __forceinline__ void tile_delta(const Stage2& dO, const Stage2& O, float* Ds, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      acc = fmaf(bf16_to_f32((uint16_t)dO.a[i][e]), bf16_to_f32((uint16_t)O.a[i][e]), acc);
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    if ((tid & 7) == 0) Ds[(tid + i * NT) >> 3] = -acc;  // stored negated: the dP accumulator's start
  }
}

// FD (fused δ, short sequences): δ = Σ_d dO·O is computed from the staged dO tile and an O tile
// loaded beside it, instead of by bwd_pre_kernel — one launch less where each (query head, tile)
// is swept by one key block anyway (T ≤ 256).
template <bool CAUSAL, bool FD>
__device__ __forceinline__ void dkdv_body(int blk, int nblocks, View q, View k, View v, View dout, View out,
                                          const float* __restrict__ lse, const float* __restrict__ delta, MView dk,
                                          MView dv, int H, int T, int nblk, float sc2, float scale, int group,
                                          Rope rp, int gsplit, int64_t split_stride) {
  // H = key/value heads; query heads hq = kvh·group + g, g < group
  __shared__ __attribute__((aligned(16))) uint16_t Qs[TILE * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Os[TILE * RS];  // dO tile
  __shared__ __attribute__((aligned(16))) float Ls[TILE];           // lse * log2(e)
  __shared__ __attribute__((aligned(16))) float Ds[TILE];           // -delta
  const int per = nblocks / nblk;
  const int bhs = blk % per;
  const int kb0 = blk / per;  // key block; block 0 has the most query tiles under a causal mask
  const int split = bhs % gsplit, bh = bhs / gsplit;
  const int b = bh / H, kvh = bh % H;
  const int gpw = group / gsplit;
  const int Hq = H * group;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int key0 = kb0 * BLK + w * 32;
  const int ki = key0 + r;  // this lane's key
  s8v kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = ld16(k.row(b, kvh, ki) + 16 * s + 8 * h);
    vf[s] = ld16(v.row(b, kvh, ki) + 16 * s + 8 * h);
  }
  if (rp.cos != nullptr) rope_frag(kf, rp, ki, h);
  f16x dvt[2] = {zero16(), zero16()}, dkt[2] = {zero16(), zero16()};
  const int t0 = CAUSAL ? (kb0 * BLK) / TILE : 0;
  const int nt = T / TILE;
  for (int g = split * gpw; g < (split + 1) * gpw; ++g) {
    const int hq = kvh * group + g;
    const float* lse_bh = lse + ((int64_t)b * Hq + hq) * T;
    const float* del_bh = FD ? nullptr : delta + ((int64_t)b * Hq + hq) * T;
    StagePair sq;
    Stage2 so, sov;  // dO tile; O tile (FD only)
    float lv = 0.f, dlv = 0.f;
    sq.load(q.row(b, hq, t0 * TILE), q.st, tid);
    so.load(dout.row(b, hq, t0 * TILE), dout.st, tid);
    if constexpr (FD) sov.load(out.row(b, hq, t0 * TILE), out.st, tid);
    if (tid < TILE) {
      lv = lse_bh[t0 * TILE + tid] * kLog2e;
      if constexpr (!FD) dlv = del_bh[t0 * TILE + tid];
    }
    if (g > split * gpw) __syncthreads();  // the previous head's last tile is still being read
    sq.rope(rp, t0 * TILE, tid);
    sq.store(Qs, RS, tid);
    so.store(Os, RS, tid);
    if (tid < TILE) {
      Ls[tid] = lv;
      if constexpr (!FD) Ds[tid] = -dlv;
    }
    if constexpr (FD) tile_delta(so, sov, Ds, tid);
    __syncthreads();
    for (int t = t0; t < nt; ++t) {
      if (t + 1 < nt) {
        sq.load(q.row(b, hq, (t + 1) * TILE), q.st, tid);
        so.load(dout.row(b, hq, (t + 1) * TILE), dout.st, tid);
        if constexpr (FD) sov.load(out.row(b, hq, (t + 1) * TILE), out.st, tid);
        if (tid < TILE) {
          lv = lse_bh[(t + 1) * TILE + tid] * kLog2e;
          if constexpr (!FD) dlv = del_bh[(t + 1) * TILE + tid];
        }
      }
      const int qt0 = t * TILE;
      if (!CAUSAL || qt0 + TILE - 1 >= key0) {
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          const int qr0 = qt0 + qb * 32;
          if (CAUSAL && qr0 + 31 < key0) continue;  // this 32-query block sees none of our keys
          // S[q][key] = Q . K^T (key on the lane); dP starts from -δ (row constant as the initial
          // accumulator: dS = P·(dP − δ) is then one multiply)
          f16x sacc = zero16(), dp;
#pragma unroll
          for (int i = 0; i < 16; ++i) dp[i] = Ds[qb * 32 + crow(i, h)];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            sacc = mfma(ld16(Qs + (qb * 32 + r) * RS + 16 * s + 8 * h), kf[s], sacc);
            dp = mfma(ld16(Os + (qb * 32 + r) * RS + 16 * s + 8 * h), vf[s], dp);
          }
          // causal mask only on the diagonal 32x32 block, behind a wave-uniform branch: a
          // per-element select in every block cost 3 VALU + 1 SALU per score
          if (CAUSAL && __builtin_amdgcn_readfirstlane((int)(qr0 < key0 + 31))) {
            const int thr = ki - qr0 - 4 * h;  // masked where (i&3) + 8(i>>2) < thr
#pragma unroll
            for (int i = 0; i < 16; ++i)
              if ((i & 3) + 8 * (i >> 2) < thr) sacc[i] = -INFINITY;
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int qrow = qb * 32 + crow(i, h);
            const float p = __builtin_amdgcn_exp2f(fmaf(sacc[i], sc2, -Ls[qrow]));
            sacc[i] = p;          // P
            dp[i] = p * dp[i];    // dS
          }
          // dV^T[d][key] += dO^T[d][q] . P[q][key];  dK^T[d][key] += Q^T[d][q] . dS[q][key]
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const s8v pb = pack_half(sacc, s);
            const s8v sb = pack_half(dp, s);
            const int qrow = qb * 32 + 16 * s + 4 * h + (lane & 15) / 4;
#pragma unroll
            for (int db = 0; db < 2; ++db) {
              const int col = db * 32 + (lane & 16) + 4 * (lane & 3);
              const uint16_t* ob = Os + qrow * RS + col;
              const uint16_t* qb_ = Qs + qrow * RS + col;
              dvt[db] = mfma(cat(tr4(ob), tr4(ob + 8 * RS)), pb, dvt[db]);
              dkt[db] = mfma(cat(tr4(qb_), tr4(qb_ + 8 * RS)), sb, dkt[db]);
            }
          }
        }
      }
      __syncthreads();
      if (t + 1 < nt) {
        sq.rope(rp, (t + 1) * TILE, tid);
        sq.store(Qs, RS, tid);
        so.store(Os, RS, tid);
        if (tid < TILE) {
          Ls[tid] = lv;
          if constexpr (!FD) Ds[tid] = -dlv;
        }
        if constexpr (FD) tile_delta(so, sov, Ds, tid);
        __syncthreads();
      }
    }
  }
  uint16_t* dkr = dk.row(b, kvh, ki) + split * split_stride;
  uint16_t* dvr = dv.row(b, kvh, ki) + split * split_stride;
  if (rp.cos != nullptr) {
    store_dT_rope(dkr, dkt[0], dkt[1], h, scale, rp, ki);
  } else {
    store_dT(dkr, dkt[0], 0, h, scale);
    store_dT(dkr, dkt[1], 1, h, scale);
  }
  store_dT(dvr, dvt[0], 0, h, 1.f);
  store_dT(dvr, dvt[1], 1, h, 1.f);
}

// ============================================================================ backward: dQ
template <bool CAUSAL, bool FD>
__device__ __forceinline__ void dq_body(int blk, int nblocks, View q, View k, View v, View dout, View out,
                                        const float* __restrict__ lse, const float* __restrict__ delta, MView dq,
                                        int H, int T, int nblk, float sc2, float scale, int group, Rope rp) {
  __shared__ __attribute__((aligned(16))) uint16_t Ks[TILE * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[TILE * RS];
  const int per = nblocks / nblk;
  const int bh = blk % per;
  const int qb = CAUSAL ? nblk - 1 - blk / per : blk / per;
  const int b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, h = lane >> 5;
  const int q0 = qb * BLK + w * 32;
  const int qi = q0 + r;
  const int kh = hh / group;
  s8v qf[4], of[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = ld16(q.row(b, hh, qi) + 16 * s + 8 * h);
    of[s] = ld16(dout.row(b, hh, qi) + 16 * s + 8 * h);
  }
  if (rp.cos != nullptr) rope_frag(qf, rp, qi, h);
  const float l2 = lse[(int64_t)bh * T + qi] * kLog2e;
  float dl;
  if constexpr (FD) {  // δ of this lane's query row: its 32 dims of dO·O + the partner lane's 32
    float acc = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const s8v ov = ld16(out.row(b, hh, qi) + 16 * s + 8 * h);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc = fmaf(bf16_to_f32((uint16_t)of[s][e]), bf16_to_f32((uint16_t)ov[e]), acc);
    }
    dl = acc + __shfl_xor(acc, 32, 64);
  } else {
    dl = delta[(int64_t)bh * T + qi];
  }
  f16x dqt[2] = {zero16(), zero16()};
  f16x ndl;  // −δ of this lane's query in every register: the dP^T accumulator's start (dS = P·dP)
#pragma unroll
  for (int i = 0; i < 16; ++i) ndl[i] = -dl;
  const int ntiles = CAUSAL ? (qb * BLK + BLK) / TILE : T / TILE;
  StagePair sk;
  Stage2 sv;
  sk.load(k.row(b, kh, 0), k.st, tid);
  sv.load(v.row(b, kh, 0), v.st, tid);
  sk.rope(rp, 0, tid);
  sk.store(Ks, RS, tid);
  sv.store(Vs, RS, tid);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) {
      sk.load(k.row(b, kh, (t + 1) * TILE), k.st, tid);
      sv.load(v.row(b, kh, (t + 1) * TILE), v.st, tid);
    }
    const int k0 = t * TILE;
    if (!CAUSAL || k0 <= q0 + 31) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const int kr0 = k0 + kb * 32;
        // a 32-key block wholly past this wave's queries contributes nothing (P = 0): skipped
        // (wave-uniform; the tile's first block always holds some key <= the wave's last query)
        if (CAUSAL && kb == 1 && __builtin_amdgcn_readfirstlane((int)(kr0 > q0 + 31))) break;
        f16x sacc = zero16(), dp = ndl;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sacc = mfma(ld16(Ks + (kb * 32 + r) * RS + 16 * s + 8 * h), qf[s], sacc);
          dp = mfma(ld16(Vs + (kb * 32 + r) * RS + 16 * s + 8 * h), of[s], dp);
        }
        // causal mask only where this 32-key block crosses the wave's queries (wave-uniform
        // branch; keys past every query of the wave were skipped with the whole tile)
        if (CAUSAL && __builtin_amdgcn_readfirstlane((int)(kr0 + 31 > q0))) {
          const int thr = qi - kr0 - 4 * h;  // masked where (i&3) + 8(i>>2) > thr
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if ((i & 3) + 8 * (i >> 2) > thr) sacc[i] = -INFINITY;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sacc[i], sc2, -l2));
          dp[i] = p * dp[i];  // dS^T[key][q]
        }
        // dQ^T[d][q] += K^T[d][key] . dS^T[key][q]
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const s8v sb = pack_half(dp, s);
          const int key = kb * 32 + 16 * s + 4 * h + (lane & 15) / 4;
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            const uint16_t* base = Ks + key * RS + db * 32 + (lane & 16) + 4 * (lane & 3);
            dqt[db] = mfma(cat(tr4(base), tr4(base + 8 * RS)), sb, dqt[db]);
          }
        }
      }
    }
    __syncthreads();
    if (t + 1 < ntiles) {
      sk.rope(rp, (t + 1) * TILE, tid);
      sk.store(Ks, RS, tid);
      sv.store(Vs, RS, tid);
      __syncthreads();
    }
  }
  uint16_t* dqr = dq.row(b, hh, qi);
  if (rp.cos != nullptr) {
    store_dT_rope(dqr, dqt[0], dqt[1], h, scale, rp, qi);
  } else {
    store_dT(dqr, dqt[0], 0, h, scale);
    store_dT(dqr, dqt[1], 1, h, scale);
  }
}

// One launch for both backward passes: blocks [0, nkv) compute dK/dV, the rest dQ — the two
// are independent, and for short sequences (SmolLM2: T = 128) neither fills the chip alone.
// (Pairing complementary causal blocks in one workgroup — key blocks kb and nblk-1-kb, query
// blocks qb and nblk-1-qb — was measured 14 % slower at B8 H12 T1024: docs/FINDINGS.md §31.)
template <bool CAUSAL, bool FD>
__global__ __launch_bounds__(NT, 2) void bwd_kernel(View q, View k, View v, View dout, View out,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ delta, MView dq, MView dk, MView dv,
                                                     int Hq, int Hkv, int T, int nblk, float sc2, float scale,
                                                     int group, Rope rp, int nkv, int gsplit, int64_t split_stride,
                                                     const int* __restrict__ order) {
  const int item = order != nullptr ? order[blockIdx.x] : (int)blockIdx.x;
  if (item < nkv)
    dkdv_body<CAUSAL, FD>(item, nkv, q, k, v, dout, out, lse, delta, dk, dv, Hkv, T, nblk, sc2, scale, group, rp,
                          gsplit, split_stride);
  else
    dq_body<CAUSAL, FD>(item - nkv, gridDim.x - nkv, q, k, v, dout, out, lse, delta, dq, Hq, T, nblk, sc2, scale,
                        group, rp);
}

// dk/dv[b, h, t, :] = Σ_s part[s][b][h][t][:] (fp32 sum of the gsplit partials); 8 elements per thread
__global__ __launch_bounds__(NT) void gqa_reduce_kernel(const uint16_t* __restrict__ pk, const uint16_t* __restrict__ pv,
                                                         MView dk, MView dv, int Hkv, int T, int gsplit,
                                                         int64_t split_stride, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < 2 * n8; i += (int64_t)gridDim.x * NT) {
    const bool isv = i >= n8;
    const int64_t j = isv ? i - n8 : i;
    const int d8 = (int)(j % (D / 8));
    const int64_t row = j / (D / 8);  // (b, h, t) row of the contiguous partial
    const int t = (int)(row % T), hh = (int)(row / T % Hkv), b = (int)(row / T / Hkv);
    const uint16_t* src = (isv ? pv : pk) + row * D + d8 * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < gsplit; ++sp) {
      float x[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(src + sp * split_stride), x);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += x[e];
    }
    uint16_t* dst = (isv ? dv : dk).row(b, hh, t) + d8 * 8;
    store8<bf16_t>(reinterpret_cast<bf16_t*>(dst), acc);
  }
}

// ============================================================================ host
// Extra dynamic LDS per workgroup (bytes) from an environment variable, read once: caps the
// workgroups resident per CU (160 KiB / (static + pad)) so that the hardware dispatcher, not
// the initial placement, balances the causal grid's unequal workgroups (experiment knob).
static int lds_pad(const char* name) {
  const char* e = std::getenv(name);
  return e == nullptr ? 0 : std::max(0, std::min(131072, std::atoi(e)));
}
static int fwd_pad() {
  static const int v = lds_pad("NBD_ATTN_FWD_LDS_PAD");
  return v;
}
static int bwd_pad() {
  static const int v = lds_pad("NBD_ATTN_BWD_LDS_PAD");
  return v;
}

// Block order for a causal grid (NBD_ATTN_ORDER=0: the plain heaviest-first order, A/B).
//
// A grid that the chip holds at once is placed round-robin: block w goes to CU w mod R (R = the
// CU count), so a CU's blocks are w, w + R, w + 2R, ... (benchmarks/dispatch_probe.hip,
// profiles/dispatch_probe_r6.txt: every CU, every grid size probed).  With causal work items of
// unequal cost, the time of such a grid is the most loaded CU's sum: GPT-2's forward (768
// blocks, 3 per CU) in the plain order puts 34 key tiles on its most loaded CU against a mean of
// 27.  The table maps block -> work item so that the first fill is an LPT assignment (heaviest
// item to the least loaded CU that still has a slot; 28 tiles there), and the blocks past the
// first fill keep the heaviest-first order for the dispatcher to hand out as slots free up.
// Built on the host once per (weights, slots) and kept in device memory; under stream capture
// an order not built yet is not built (a memcpy cannot be captured) and the plain order runs.
static bool order_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NBD_ATTN_ORDER");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

static int cu_count(int dev) {
  static int n[64] = {0};
  if (dev < 0 || dev >= 64) return 0;
  if (n[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) v = -1;
    n[dev] = v;
  }
  return n[dev];
}

// weights() = cost of each work item k (items indexed as the kernel reads them), called only
// when `shape` (everything the weights depend on) has no table yet; slots = resident blocks per
// CU.  Returns nullptr when the plain order is as good (equal weights) or unavailable.
template <typename W>
static const int* block_order(std::vector<int64_t> shape, W weights, int slots, int dev, hipStream_t st) {
  if (!order_enabled() || slots < 1) return nullptr;
  const int R = cu_count(dev);
  if (R < 1) return nullptr;
  static std::mutex mu;
  static std::map<std::vector<int64_t>, int*> cache;  // (nullptr: the plain order)
  shape.push_back(slots);
  shape.push_back(R);
  shape.push_back(dev);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(shape);
  if (it != cache.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
  const std::vector<int> weight = weights();
  if (weight.empty() || std::all_of(weight.begin(), weight.end(), [&](int x) { return x == weight[0]; })) {
    cache.emplace(std::move(shape), nullptr);
    return nullptr;
  }
  const int G = (int)weight.size();
  std::vector<int> items(G);
  std::iota(items.begin(), items.end(), 0);
  std::stable_sort(items.begin(), items.end(), [&](int a, int b) { return weight[a] > weight[b]; });
  const int F = std::min<int64_t>(G, (int64_t)R * slots);  // the first fill
  // CU c holds the first-fill blocks c, c + R, ... (< F): cap[c] of them
  std::vector<int> cap(R), load(R, 0);
  std::vector<std::vector<int>> held(R);
  for (int c = 0; c < R; ++c) cap[c] = F / R + (c < F % R ? 1 : 0);
  using E = std::pair<int, int>;  // (load, cu)
  std::priority_queue<E, std::vector<E>, std::greater<E>> pq;
  for (int c = 0; c < R; ++c)
    if (cap[c] > 0) pq.push({0, c});
  for (int i = 0; i < F; ++i) {
    const E e = pq.top();
    pq.pop();
    const int c = e.second;
    held[c].push_back(items[i]);
    load[c] += weight[items[i]];
    if ((int)held[c].size() < cap[c]) pq.push({load[c], c});
  }
  std::vector<int> perm(G);
  for (int c = 0; c < R; ++c)
    for (size_t r = 0; r < held[c].size(); ++r) perm[c + (int64_t)r * R] = held[c][r];
  for (int i = F; i < G; ++i) perm[i] = items[i];
  int* d = nullptr;
  if (hipMalloc(&d, sizeof(int) * G) != hipSuccess) return nullptr;
  if (hipMemcpy(d, perm.data(), sizeof(int) * G, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  cache.emplace(std::move(shape), d);
  if (const char* lg = std::getenv("NBD_ATTN_ORDER_LOG"); lg != nullptr && lg[0] == '1') {
    int plain = 0;  // the most loaded CU under the plain order (first fill)
    for (int c = 0; c < R; ++c) {
      int sum = 0;
      for (int64_t b = c; b < F; b += R) sum += weight[b];
      plain = std::max(plain, sum);
    }
    std::fprintf(stderr, "nbd attn block order: %d items, %d per CU x %d CUs, most loaded CU %d (plain order %d)\n", G,
                 slots, R, *std::max_element(load.begin(), load.end()), plain);
  }
  return d;
}

template <typename K>
static int resident_blocks(K kernel, int lds_bytes, const char* env = nullptr) {
  if (env != nullptr) {  // override for A/B runs
    const char* e = std::getenv(env);
    if (e != nullptr && std::atoi(e) > 0) return std::atoi(e);
  }
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(kernel), NT, lds_bytes) !=
      hipSuccess)
    return 0;
  return n;
}

static View view_of(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.size(3) == D && t.stride(3) == 1, "attn: ", name,
              " must be a [B, H, T, 64] GPU view with a contiguous last dim");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "attn: ", name, " must be bfloat16");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0 &&
                  ((uintptr_t)t.data_ptr() & 15) == 0,
              "attn: ", name, " strides must be multiples of 8 elements and its base 16-B aligned");
  return View{static_cast<const uint16_t*>(t.data_ptr()), t.stride(0), t.stride(1), t.stride(2)};
}
static MView mview_of(const at::Tensor& t, const char* name) {
  View v = view_of(t, name);
  return MView{const_cast<uint16_t*>(v.p), v.sb, v.sh, v.st};
}
static void check_shapes(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v) {
  TORCH_CHECK(k.sizes() == v.sizes() && q.size(0) == k.size(0) && q.size(2) == k.size(2),
              "attn: k and v must match, and share batch and length with q");
  TORCH_CHECK(k.size(1) > 0 && q.size(1) % k.size(1) == 0, "attn: query heads must be a multiple of key/value heads");
  TORCH_CHECK(q.size(2) % BLK == 0 && q.size(2) >= BLK, "attn: sequence length must be a positive multiple of 128");
  TORCH_CHECK(q.size(0) * q.size(1) * (q.size(2) / BLK) < (1LL << 31), "attn: grid too large");
}

static Rope rope_of(const c10::optional<at::Tensor>& c, const c10::optional<at::Tensor>& s, int64_t T) {
  const bool hc = c.has_value() && c->defined(), hs = s.has_value() && s->defined();
  TORCH_CHECK(hc == hs, "attn: rope_cos and rope_sin go together");
  if (!hc) return Rope{nullptr, nullptr};
  TORCH_CHECK(c->is_cuda() && s->is_cuda() && c->scalar_type() == at::kFloat && s->scalar_type() == at::kFloat &&
                  c->is_contiguous() && s->is_contiguous() && c->dim() == 2 && c->size(1) == D / 2 &&
                  s->sizes() == c->sizes() && c->size(0) >= T,
              "attn: rope tables must be contiguous float32 [>= T, 32]");
  return Rope{c->data_ptr<float>(), s->data_ptr<float>()};
}

std::tuple<at::Tensor, at::Tensor> attn_fwd_hip(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                bool causal, double scale, const c10::optional<at::Tensor>& rope_cos,
                                                const c10::optional<at::Tensor>& rope_sin) {
  check_shapes(q, k, v);
  const Rope rp = rope_of(rope_cos, rope_sin, q.size(2));
  const int B = q.size(0), H = q.size(1), T = q.size(2);
  View qv = view_of(q, "q"), kv = view_of(k, "k"), vv = view_of(v, "v");
  // output stored [B, T, H, D] (what the projection after attention reads), returned as [B, H, T, D]
  at::Tensor o = at::empty({B, T, H, D}, q.options()).permute({0, 2, 1, 3});
  at::Tensor lse = at::empty({B, H, T}, q.options().dtype(at::kFloat));
  MView ov = mview_of(o, "out");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int nblk = T / BLK;
  const dim3 grid((unsigned)(B * H * nblk));
  const float sc2 = (float)scale * kLog2e;
  const int group = H / (int)k.size(1);
  if (causal) {
    // item k: query block nblk - 1 - k / (B·H), 2·(that + 1) key tiles
    const int* order = nullptr;
    if (nblk > 1) {
      static const int slots = resident_blocks(fwd_kernel<true>, fwd_pad(), "NBD_ATTN_FWD_SLOTS");
      const int BH = B * H;
      order = block_order(
          {0, BH, nblk},
          [&] {
            std::vector<int> w((size_t)BH * nblk);
            for (size_t i = 0; i < w.size(); ++i) w[i] = 2 * (nblk - (int)(i / BH));
            return w;
          },
          slots, q.get_device(), st);
    }
    hipLaunchKernelGGL((fwd_kernel<true>), grid, dim3(NT), fwd_pad(), st, qv, kv, vv, ov, lse.data_ptr<float>(), H, T, nblk,
                       sc2, group, rp, order);
  } else {
    hipLaunchKernelGGL((fwd_kernel<false>), grid, dim3(NT), fwd_pad(), st, qv, kv, vv, ov, lse.data_ptr<float>(), H, T, nblk,
                       sc2, group, rp, static_cast<const int*>(nullptr));
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {o, lse};
}

void attn_bwd_hip(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                  const at::Tensor& out, const at::Tensor& lse, bool causal, double scale, const at::Tensor& dq,
                  const at::Tensor& dk, const at::Tensor& dv, const c10::optional<at::Tensor>& rope_cos,
                  const c10::optional<at::Tensor>& rope_sin, const c10::optional<at::Tensor>& delta_in) {
  check_shapes(q, k, v);
  const Rope rp = rope_of(rope_cos, rope_sin, q.size(2));
  TORCH_CHECK(dout.sizes() == q.sizes() && out.sizes() == q.sizes() && dq.sizes() == q.sizes() &&
                  dk.sizes() == k.sizes() && dv.sizes() == v.sizes(),
              "attn_bwd: shape mismatch");
  const int B = q.size(0), H = q.size(1), T = q.size(2);
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == (int64_t)B * H * T,
              "attn_bwd: lse must be float32 [B, H, T]");
  View qv = view_of(q, "q"), kv = view_of(k, "k"), vv = view_of(v, "v"), dov = view_of(dout, "dout"),
       ov = view_of(out, "out");
  MView dqv = mview_of(dq, "dq"), dkv = mview_of(dk, "dk"), dvv = mview_of(dv, "dv");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(q.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int nblk = T / BLK;
  // short sequences: δ inside the main kernel (each (query head, tile) is swept by <= 2 key blocks)
  static const int fd_env = [] {  // NBD_ATTN_FD=1 / 0: force the fused-δ path on / off (A/B)
    const char* e = std::getenv("NBD_ATTN_FD");
    return e == nullptr ? -1 : std::atoi(e);
  }();
  const bool fd = fd_env >= 0 ? fd_env == 1 : nblk <= 2;
  at::Tensor delta;
  if (!fd && delta_in.has_value() && delta_in->defined()) {
    // δ computed by the producer of dout (gemm.hip EPI_ADELTA: the output projection's input
    // gradient) — no pre-pass
    TORCH_CHECK(delta_in->is_cuda() && delta_in->scalar_type() == at::kFloat && delta_in->is_contiguous() &&
                    delta_in->numel() == (int64_t)B * H * T,
                "attn_bwd: delta must be float32 [B, H, T]");
    delta = *delta_in;
  } else if (!fd) {
    delta = at::empty({B, H, T}, lse.options());
    const int64_t rows = (int64_t)B * H * T;
    hipLaunchKernelGGL(bwd_pre_kernel, dim3((unsigned)((rows + NT / 8 - 1) / (NT / 8))), dim3(NT), 0, st, dov, ov,
                       delta.data_ptr<float>(), H, T, rows);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
  float* dptr = fd ? nullptr : delta.data_ptr<float>();
  const int Hkv = (int)k.size(1), group = H / Hkv;
  const float sc2 = (float)scale * kLog2e;
  // GQA with few key/value workgroups: split each kv head's query-head group over workgroups
  // (below 128 of them: SmolLM2 B16 T128 has 48 and runs its backward in 16.8 µs split against
  // 23.4 unsplit; at B64, 192, unsplit is faster, 24.9 against 39.0 — profiles/attn_nw_gsplit_r5.txt)
  static const int gsplit_env = [] {  // NBD_ATTN_GSPLIT=1: never split (A/B)
    const char* e = std::getenv("NBD_ATTN_GSPLIT");
    return e == nullptr ? 0 : std::atoi(e);
  }();
  const int gsplit = gsplit_env == 1 ? 1 : (group > 1 && B * Hkv * nblk < 128) ? group : 1;
  const int nkv = B * Hkv * nblk * gsplit, nq = B * H * nblk;
  MView dkw = dkv, dvw = dvv;
  at::Tensor pk, pv;
  int64_t split_stride = 0;
  if (gsplit > 1) {  // contiguous partials [gsplit][B][Hkv][T][D]
    pk = at::empty({gsplit, B, Hkv, T, D}, q.options());
    pv = at::empty({gsplit, B, Hkv, T, D}, q.options());
    split_stride = (int64_t)B * Hkv * T * D;
    dkw = MView{static_cast<uint16_t*>(pk.data_ptr()), (int64_t)Hkv * T * D, (int64_t)T * D, D};
    dvw = MView{static_cast<uint16_t*>(pv.data_ptr()), (int64_t)Hkv * T * D, (int64_t)T * D, D};
  }
  // causal items: dK/dV of key block kb sweeps (nblk - kb)·2 query tiles of gpw heads, ≈ 4 MFMA
  // products per tile; dQ of query block qb sweeps (qb + 1)·2 key tiles, 3 products per tile
  auto causal_order = [&](auto kernel) -> const int* {
    if (nblk <= 1) return nullptr;
    static const int slots = resident_blocks(kernel, bwd_pad(), "NBD_ATTN_BWD_SLOTS");
    const int gpw = group / gsplit;
    return block_order(
        {1, nkv, nq, nblk, gpw},
        [&] {
          std::vector<int> w((size_t)nkv + nq);
          const int per_kv = nkv / nblk, per_q = nq / nblk;
          for (int i = 0; i < nkv; ++i) w[i] = 4 * 2 * (nblk - i / per_kv) * gpw;
          for (int i = 0; i < nq; ++i) w[nkv + i] = 3 * 2 * (nblk - i / per_q);
          return w;
        },
        slots, q.get_device(), st);
  };
#define NBD_BWD(C_, F_, O_)                                                                                  \
  hipLaunchKernelGGL((bwd_kernel<C_, F_>), dim3((unsigned)(nkv + nq)), dim3(NT), bwd_pad(), st, qv, kv, vv, dov, ov,   \
                     lse.data_ptr<float>(), dptr, dqv, dkw, dvw, H, Hkv, T, nblk, sc2, (float)scale, group, rp, nkv, \
                     gsplit, split_stride, O_)
  const int* none = nullptr;
  if (causal) {
    if (fd) NBD_BWD(true, true, causal_order(bwd_kernel<true, true>));
    else NBD_BWD(true, false, causal_order(bwd_kernel<true, false>));
  } else {
    if (fd) NBD_BWD(false, true, none);
    else NBD_BWD(false, false, none);
  }
#undef NBD_BWD
  C10_HIP_KERNEL_LAUNCH_CHECK();
  if (gsplit > 1) {
    const int64_t n8 = (int64_t)B * Hkv * T * (D / 8);
    const int blocks = (int)std::min<int64_t>((2 * n8 + NT - 1) / NT, 1024);
    hipLaunchKernelGGL(gqa_reduce_kernel, dim3(blocks), dim3(NT), 0, st, static_cast<const uint16_t*>(pk.data_ptr()),
                       static_cast<const uint16_t*>(pv.data_ptr()), dkv, dvv, Hkv, T, gsplit, split_stride, n8);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
}

}  // namespace attn
}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("attn_fwd", &nbd::attn::attn_fwd_hip);
  m.impl("attn_bwd", &nbd::attn::attn_bwd_hip);
}
