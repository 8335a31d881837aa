// norm.hip — LayerNorm (with fused residual add) forward/backward and column sums, gfx950.
//
// GPT-2 small runs 25 LayerNorms over [8192, 768] bf16 rows per step plus a residual add before
// each; torch's kernels took ≈1.5 ms/step for the norms and 0.37 ms for the adds, and Linear's
// bias gradients (column sums of dY) another 1.0 ms through the generic reduce kernel
// (profiles/gpt2_step_rocprof_r1b.md) — all memory-bound work well below the HBM roof.
//
//   ln_fwd      one wave per row (4 rows per 256-thread workgroup); a lane owns 4-element
//               (8-B) chunks c = 4·lane + 256·k, held in registers between the mean and
//               variance passes (two wave64 reductions, no LDS); optional fused residual add
//               (writes x + delta once, normalises it) — 1 read (2 with the residual) + 1–2 writes.
//   ln_bwd      each workgroup sweeps 16 rows (4 per wave, loads of two rows in flight at once): dx = rstd·(g·dy − mean(g·dy) −
//               x̂·mean(g·dy·x̂)) (+ the residual stream's gradient, fused), and per-lane column
//               partials Σdy·x̂, Σdy reduced over the 4 waves in LDS → one [C] partial row per
//               workgroup; col_reduce sums the partials (fp32) into dγ, dβ.
//   colsum      bias gradients: [rows, C] → per-workgroup column partials (a lane owns 8
//               columns = one 16-B load per row) → col_reduce.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <cstdlib>

#include <tuple>
#include <type_traits>

#include "graddst.h"
#include "nbd_common.h"

namespace nbd {
namespace norm {

constexpr int NT = 256;
constexpr int kMaxCh = 8;  // 4-element chunks per lane: C <= 64 * 4 * 8 = 2048 (kernels are
                           // instantiated per chunk count NCH = ceil(C / 256) to keep registers low)

template <typename T>
__device__ __forceinline__ float round_to(float v) { return v; }
template <>
__device__ __forceinline__ float round_to<bf16_t>(float v) { return bf16_to_f32(f32_to_bf16(v)); }
template <>
__device__ __forceinline__ float round_to<f16_t>(float v) { return f16_to_f32(f32_to_f16(v)); }

template <typename T>
__device__ __forceinline__ void load4(const T* p, float (&v)[4]);
template <>
__device__ __forceinline__ void load4<bf16_t>(const bf16_t* p, float (&v)[4]) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(w.x << 16);
  v[1] = __uint_as_float(w.x & 0xffff0000u);
  v[2] = __uint_as_float(w.y << 16);
  v[3] = __uint_as_float(w.y & 0xffff0000u);
}
template <>
__device__ __forceinline__ void load4<f16_t>(const f16_t* p, float (&v)[4]) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
  v[0] = f16_to_f32((uint16_t)(w.x & 0xffffu));
  v[1] = f16_to_f32((uint16_t)(w.x >> 16));
  v[2] = f16_to_f32((uint16_t)(w.y & 0xffffu));
  v[3] = f16_to_f32((uint16_t)(w.y >> 16));
}
template <>
__device__ __forceinline__ void load4<float>(const float* p, float (&v)[4]) {
  const float4 w = *reinterpret_cast<const float4*>(p);
  v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
}
template <typename T>
__device__ __forceinline__ void store4(T* p, const float (&v)[4]);
template <>
__device__ __forceinline__ void store4<bf16_t>(bf16_t* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2(pack2_bf16(v[0], v[1]), pack2_bf16(v[2], v[3]));
}
template <>
__device__ __forceinline__ void store4<f16_t>(f16_t* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)f32_to_f16(v[0]) | ((uint32_t)f32_to_f16(v[1]) << 16),
                                            (uint32_t)f32_to_f16(v[2]) | ((uint32_t)f32_to_f16(v[3]) << 16));
}
template <>
__device__ __forceinline__ void store4<float>(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// ============================================================================ forward
template <typename T, typename W, bool RES, int NCH, bool RMS = false>
__global__ __launch_bounds__(NT) void ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ delta,
                                                    T* __restrict__ xsum, const W* __restrict__ gamma,
                                                    const W* __restrict__ beta, T* __restrict__ y,
                                                    float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                    int64_t rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (NT / kWave) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t base = row * C;
  float v[NCH][4], g[NCH][4], b[NCH][4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
      // γ / β first: their latency hides under the row's, not after the reductions
      load4<W>(gamma + c, g[k]);
      if (!RMS) load4<W>(beta + c, b[k]);
      load4<T>(x + base + c, v[k]);
      if (RES) {
        float d[4];
        load4<T>(delta + base + c, d);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[k][e] += d[e];
        store4<T>(xsum + base + c, v[k]);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[k][e] = round_to<T>(v[k][e]);  // normalise what was stored
      }
      s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
    }
  }
  const float mean = RMS ? 0.f : wsum(s) / (float)C;  // RMSNorm: no centring
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[k][e] - mean;
        q = fmaf(d, d, q);
      }
    }
  }
  const float rstd = rsqrtf(wsum(q) / (float)C + eps);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = fmaf((v[k][e] - mean) * rstd, g[k][e], RMS ? 0.f : b[k][e]);
      store4<T>(y + base + c, o);
    }
  }
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;  // RMSNorm: no mean (nullptr)
    rstd_out[row] = rstd;
  }
}

// ============================================================================ backward
constexpr int kBwdRows = 16;  // max rows per workgroup (4 per wave, two at a time)
// rows per wave iteration: 2 (ln_bwd_kernel's kRpi), or 1 with 4-row workgroups for small
// inputs (SmolLM2's 2048 rows: 512 workgroups of one row per wave instead of 256 of two)

// rows per workgroup: 16 for large inputs (GPT-2: 8192 rows -> 512 workgroups), fewer when that
// would leave the chip under-filled, but at least 8 so all four waves hold rows (SmolLM2 at
// 16 x 128 tokens: 2048 rows -> 8 per workgroup; with 4, two of the four waves idled and the
// weight-gradient partial rows doubled)
static bool small_rows_enabled() {  // NBD_LN_BWD_RPI1=0: keep 8-row workgroups (A/B)
  static const bool on = [] {
    const char* e = std::getenv("NBD_LN_BWD_RPI1");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}

static int bwd_rows_per_block(int64_t rows) {
  static const int forced = [] {  // NBD_LN_BWD_ROWS: A/B override (4 .. 64)
    const char* e = std::getenv("NBD_LN_BWD_ROWS");
    const int v = e ? std::atoi(e) : 0;
    return (v == 4 || v == 8 || v == 16 || v == 32 || v == 64) ? v : 0;
  }();
  if (forced) return forced;
  int r = kBwdRows;
  while (r > 8 && (rows + r - 1) / r < 512) r /= 2;
  if (r == 8 && (rows + 7) / 8 < 512 && small_rows_enabled()) r = 4;  // one row per wave (kRpi 1)
  return r;
}

template <typename T, typename W, bool RES, int NCH, bool RMS = false, int kRpi = 2>
__global__ __launch_bounds__(NT) void ln_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                    const T* __restrict__ dres, const W* __restrict__ gamma,
                                                    const float* __restrict__ mean_in,
                                                    const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                    float* __restrict__ part_g, int64_t rows, int C, int rpb) {
  __shared__ float red[2][NT / kWave - 1][NCH * 256];  // waves 1..3 hand their column partials to wave 0
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float g[NCH][4], ag[NCH][4], ab[NCH][4];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
#pragma unroll
    for (int e = 0; e < 4; ++e) ag[k][e] = ab[k][e] = 0.f;
    if (c < C) load4<W>(gamma + c, g[k]);
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  // each wave takes kRpi rows at a time and issues all their loads before any arithmetic
  for (int i = wave * kRpi; i < rpb; i += (NT / kWave) * kRpi) {
    float xv[kRpi][NCH][4], dv[kRpi][NCH][4], rv[kRpi][NCH][4];
    float mean[kRpi], rstd[kRpi];
    bool live[kRpi];
#pragma unroll
    for (int j = 0; j < kRpi; ++j) {
      const int64_t row = r0 + i + j;
      live[j] = row < rows && i + j < rpb;
      const int64_t rr = live[j] ? row : r0;  // dead rows re-read a live one; their results are dropped
      mean[j] = RMS ? 0.f : mean_in[rr];
      rstd[j] = rstd_in[rr];
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < C) {
          load4<T>(x + rr * C + c, xv[j][k]);
          load4<T>(dy + rr * C + c, dv[j][k]);
          if (RES) load4<T>(dres + rr * C + c, rv[j][k]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kRpi; ++j) {
      if (!live[j]) continue;
      const int64_t base = (r0 + i + j) * C;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < C) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float xh = (xv[j][k][e] - mean[j]) * rstd[j];
            const float gy = dv[j][k][e] * g[k][e];
            xv[j][k][e] = xh;  // keep x̂ and g·dy in the load registers
            s1 += gy;
            s2 = fmaf(gy, xh, s2);
            ag[k][e] = fmaf(dv[j][k][e], xh, ag[k][e]);
            if (!RMS) ab[k][e] += dv[j][k][e];  // RMSNorm has no β: no Σdy partials
            dv[j][k][e] = gy;
          }
        }
      }
      const float m1 = RMS ? 0.f : wsum(s1) / (float)C, m2 = wsum(s2) / (float)C;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < C) {
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = rstd[j] * (dv[j][k][e] - m1 - xv[j][k][e] * m2);
            if (RES) o[e] += rv[j][k][e];
          }
          store4<T>(dx + base + c, o);
        }
      }
    }
  }
  // column partials of this workgroup: waves 1..3 -> LDS -> wave 0 sums and writes one row
  if (wave > 0) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = 4 * lane + 256 * k;
      if (c < C)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          red[0][wave - 1][c + e] = ag[k][e];
          if (!RMS) red[1][wave - 1][c + e] = ab[k][e];
        }
    }
  }
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = 4 * lane + 256 * k;
      if (c < C) {
#pragma unroll
        for (int w = 0; w < NT / kWave - 1; ++w)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ag[k][e] += red[0][w][c + e];
            if (!RMS) ab[k][e] += red[1][w][c + e];
          }
        store4<float>(part_g + (int64_t)blockIdx.x * 2 * C + c, ag[k]);                // [blk][0, C)
        if (!RMS) store4<float>(part_g + (int64_t)blockIdx.x * 2 * C + C + c, ab[k]);  // [blk][C, 2C)
      }
    }
  }
}

// ln_bwd for 2-byte types with C % 256 == 0 (GPT-2: 768): half a wave per row, so every lane
// moves 16 B per access (8 elements; the 64-lane version above moves 8 B) and a wave has four
// rows' loads in flight; row values stay packed (bf16 / f16) in registers until used.  Column
// partials are combined across the two halves, then across the waves as above.
template <typename T>
__device__ __forceinline__ void unpack8v(const u32x4& w, float (&v)[8]);
template <>
__device__ __forceinline__ void unpack8v<bf16_t>(const u32x4& w, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void unpack8v<f16_t>(const u32x4& w, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = f16_to_f32((uint16_t)(w[j] & 0xffffu));
    v[2 * j + 1] = f16_to_f32((uint16_t)(w[j] >> 16));
  }
}

__device__ __forceinline__ float hsum(float v) {  // sum over the 32 lanes of a half-wave
#pragma unroll
  for (int off = 16; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

constexpr int kRpi16 = 1;  // one row pair per wave iteration: 192 VGPRs (two pairs: 256, and slower — 16.8 vs 16.2 µs)

// Forward with 16-B accesses (2-byte types, C a multiple of 256): a half-wave per row, NCH
// 8-element chunks per lane (ln_fwd_kernel: a wave per row, 8-B chunks).  Same math; the partial
// sums group 8 elements per lane, so the last bits can differ from ln_fwd_kernel's.
template <typename T, typename W, bool RES, int NCH, bool RMS = false>
__global__ __launch_bounds__(NT) void ln_fwd16_kernel(const T* __restrict__ x, const T* __restrict__ delta,
                                                      T* __restrict__ xsum, const W* __restrict__ gamma,
                                                      const W* __restrict__ beta, T* __restrict__ y,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int64_t rows, int C, float eps) {
  static_assert(sizeof(T) == 2, "ln_fwd16: 2-byte element types");
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int64_t row = ((int64_t)blockIdx.x * (NT / kWave) + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  if (row >= rows) return;  // (whole half-waves: the reductions below stay within the live half)
  const int64_t base = row * C;
  float v[NCH][8], g[NCH][8], b[NCH][8];
  u32x4 xv[NCH], dv[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 8 * hl + 256 * k;
    xv[k] = *reinterpret_cast<const u32x4*>(x + base + c);
    if (RES) dv[k] = *reinterpret_cast<const u32x4*>(delta + base + c);
    load8<W>(gamma + c, g[k]);
    if (!RMS) load8<W>(beta + c, b[k]);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    unpack8v<T>(xv[k], v[k]);
    if (RES) {
      float d[8];
      unpack8v<T>(dv[k], d);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[k][e] += d[e];
      store8<T>(xsum + base + 8 * hl + 256 * k, v[k]);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[k][e] = round_to<T>(v[k][e]);  // normalise what was stored
    }
#pragma unroll
    for (int e = 0; e < 8; e += 4) s += (v[k][e] + v[k][e + 1]) + (v[k][e + 2] + v[k][e + 3]);
  }
  const float mean = RMS ? 0.f : hsum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[k][e] - mean;
      q = fmaf(d, d, q);
    }
  const float rstd = rsqrtf(hsum(q) / (float)C + eps);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = fmaf((v[k][e] - mean) * rstd, g[k][e], RMS ? 0.f : b[k][e]);
    store8<T>(y + base + 8 * hl + 256 * k, o);
  }
  if (hl == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <typename T, typename W, bool RES, int NCH, bool RMS = false>
__global__ __launch_bounds__(NT) void ln_bwd16_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                      const T* __restrict__ dres, const W* __restrict__ gamma,
                                                      const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                      float* __restrict__ part_g, int64_t rows, int C, int rpb) {
  static_assert(sizeof(T) == 2, "ln_bwd16: 2-byte element types");
  __shared__ float red[2][NT / kWave - 1][NCH * 256];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, hl = lane & 31;
  float g[NCH][8], ag[NCH][8], ab[NCH][8];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    load8<W>(gamma + 8 * hl + 256 * k, g[k]);
#pragma unroll
    for (int e = 0; e < 8; ++e) ag[k][e] = ab[k][e] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  for (int i = wave * 2 * kRpi16; i < rpb; i += (NT / kWave) * 2 * kRpi16) {
    u32x4 xv[kRpi16][NCH], dv[kRpi16][NCH], rv[kRpi16][NCH];
    float mean[kRpi16], rstd[kRpi16];
    bool live[kRpi16];
#pragma unroll
    for (int j = 0; j < kRpi16; ++j) {
      const int li = i + 2 * j + half;
      const int64_t row = r0 + li;
      live[j] = row < rows && li < rpb;
      const int64_t rr = live[j] ? row : r0;  // dead rows re-read a live one; nothing of theirs is kept
      mean[j] = RMS ? 0.f : mean_in[rr];
      rstd[j] = rstd_in[rr];
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int64_t o = rr * C + 8 * hl + 256 * k;
        xv[j][k] = *reinterpret_cast<const u32x4*>(x + o);
        dv[j][k] = *reinterpret_cast<const u32x4*>(dy + o);
        if (RES) rv[j][k] = *reinterpret_cast<const u32x4*>(dres + o);
      }
    }
#pragma unroll
    for (int j = 0; j < kRpi16; ++j) {
      const float lv = live[j] ? 1.f : 0.f;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        float xf[8], df[8];
        unpack8v<T>(xv[j][k], xf);
        unpack8v<T>(dv[j][k], df);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (xf[e] - mean[j]) * rstd[j];
          const float gy = df[e] * g[k][e];
          s1 += gy;
          s2 = fmaf(gy, xh, s2);
          ag[k][e] = fmaf(df[e] * lv, xh, ag[k][e]);
          if (!RMS) ab[k][e] = fmaf(df[e], lv, ab[k][e]);
        }
      }
      const float m1 = RMS ? 0.f : hsum(s1) / (float)C, m2 = hsum(s2) / (float)C;
      if (live[j]) {
        const int64_t base = (r0 + i + 2 * j + half) * C;
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
          float xf[8], df[8], o[8];
          unpack8v<T>(xv[j][k], xf);
          unpack8v<T>(dv[j][k], df);
          float rf[8];
          if (RES) unpack8v<T>(rv[j][k], rf);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float xh = (xf[e] - mean[j]) * rstd[j];
            o[e] = rstd[j] * (df[e] * g[k][e] - m1 - xh * m2);
            if (RES) o[e] += rf[e];
          }
          store8<T>(dx + base + 8 * hl + 256 * k, o);
        }
      }
    }
  }
  // the two halves hold the same columns: fold, then waves 1..3 -> LDS -> wave 0
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ag[k][e] += __shfl_xor(ag[k][e], 32, kWave);
      if (!RMS) ab[k][e] += __shfl_xor(ab[k][e], 32, kWave);
    }
  if (wave > 0 && half == 0) {
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[0][wave - 1][8 * hl + 256 * k + e] = ag[k][e];
        if (!RMS) red[1][wave - 1][8 * hl + 256 * k + e] = ab[k][e];
      }
  }
  __syncthreads();
  if (wave == 0 && half == 0) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = 8 * hl + 256 * k;
#pragma unroll
      for (int w = 0; w < NT / kWave - 1; ++w)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ag[k][e] += red[0][w][c + e];
          if (!RMS) ab[k][e] += red[1][w][c + e];
        }
      store8<float>(part_g + (int64_t)blockIdx.x * 2 * C + c, ag[k]);
      if (!RMS) store8<float>(part_g + (int64_t)blockIdx.x * 2 * C + C + c, ab[k]);
    }
  }
}

// ============================================================================ column sums
constexpr int kColRows = 64;  // rows per workgroup

template <typename T>
__global__ __launch_bounds__(NT) void colsum_kernel(const T* __restrict__ x, int64_t rows, int C,
                                                    float* __restrict__ part) {
  // a lane owns 8 columns (one 16-B load per row); 256 threads = 2048 columns per workgroup
  // tile; blockIdx.y = column tile, blockIdx.x = row block
  const int c = (blockIdx.y * NT + threadIdx.x) * 8;
  if (c >= C) return;
  const int64_t r0 = (int64_t)blockIdx.x * kColRows;
  const int64_t r1 = r0 + kColRows < rows ? r0 + kColRows : rows;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int64_t r = r0;
  for (; r + 4 <= r1; r += 4) {  // four rows in flight per lane
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) load8<T>(x + (r + u) * C + c, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[u][e];
  }
  for (; r < r1; ++r) {
    float v[8];
    load8<T>(x + r * C + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += v[e];
  }
  store8<float>(part + (int64_t)blockIdx.x * C + c, acc);
}

// Sum of `nparts` partial rows of width W (= C, or 2C for LayerNorm's [dγ | dβ] partials) into
// out0[c] (c < C) / out1[c - C].  Workgroup = 16 columns x 16 partial-row groups: every thread's
// loads are independent and issued together, the 16 groups are combined in LDS — no serial
// per-column loop (a one-thread-per-column version spent 18 µs per call, latency-bound).
template <typename O>
__global__ __launch_bounds__(NT) void col_reduce_kernel(const float* __restrict__ part, int nparts, int ld, int W,
                                                        int C, O* __restrict__ out0, O* __restrict__ out1,
                                                        int accum) {
  __shared__ float red[16][17];
  const int cx = threadIdx.x & 15, pg = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cx;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < W) {
    int p = pg;
    for (; p + 48 < nparts; p += 64) {
      a0 += part[(int64_t)p * ld + c];
      a1 += part[(int64_t)(p + 16) * ld + c];
      a2 += part[(int64_t)(p + 32) * ld + c];
      a3 += part[(int64_t)(p + 48) * ld + c];
    }
    for (; p < nparts; p += 16) a0 += part[(int64_t)p * ld + c];
  }
  red[pg][cx] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (pg == 0 && c < W) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) s += red[g][cx];
    // accum bit 0 / 1: add to out0 / out1 (gradient accumulation in a bucket slice)
    if (c < C) Elem<O>::store(out0, c, (accum & 1) ? s + Elem<O>::load(out0, c) : s);
    else Elem<O>::store(out1, c - C, (accum & 2) ? s + Elem<O>::load(out1, c - C) : s);
  }
}

// ============================================================================ host
// A Llama model's token embedding and its first RMSNorm in one pass (a wave per row):
// x0[r] = table[ids[r]] (stored: the residual stream) and y[r] = RMSNorm(x0[r])·g, with the same
// arithmetic as F.embedding + ln_fwd_kernel<RMS> (identical bits).  Out-of-range ids read as zero
// rows and set `err` (the host reads the flag lazily, ops/embedding.py), as embedding_tokpos does.
template <typename T, typename W, int NCH>
__global__ __launch_bounds__(NT) void embed_rms_kernel(const int64_t* __restrict__ ids, const T* __restrict__ table,
                                                       int64_t V, const W* __restrict__ gamma, T* __restrict__ x0,
                                                       T* __restrict__ y, float* __restrict__ rstd_out, int64_t rows,
                                                       int C, float eps, int* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (NT / kWave) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t id = ids[row];
  const bool ok = id >= 0 && id < V;
  if (!ok && err != nullptr && lane == 0) atomicOr(err, 1);  // (a vector-memory atomic)
  const T* src = table + (ok ? id : 0) * (int64_t)C;
  const int64_t base = row * C;
  float v[NCH][4], g[NCH][4];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
      load4<W>(gamma + c, g[k]);
      if (ok) {
        load4<T>(src + c, v[k]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[k][e] = 0.f;
      }
      store4<T>(x0 + base + c, v[k]);
    }
  }
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[k][e] - 0.f;
        q = fmaf(d, d, q);
      }
    }
  }
  const float rstd = rsqrtf(wsum(q) / (float)C + eps);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = fmaf((v[k][e] - 0.f) * rstd, g[k][e], 0.f);
      store4<T>(y + base + c, o);
    }
  }
  if (lane == 0) rstd_out[row] = rstd;
}

// GPT-2's input and its first LayerNorm in one pass (a wave per row): x0[r] = wte[idx[r]] +
// wpe[pos[r % Tp]] (fp32 add, stored rounded — embedding_tokpos's bits) and y[r] = LayerNorm(x0[r])
// with ln_fwd_kernel's arithmetic on the rounded row.  Out-of-range ids (outside [0, V)) read as
// zero rows and set `err`; out-of-range positions read as zero rows.
template <typename T, typename W, int NCH>
__global__ __launch_bounds__(NT) void tokpos_ln_kernel(const int64_t* __restrict__ idx, const T* __restrict__ wte,
                                                       int64_t V, const int64_t* __restrict__ pos, int Tp,
                                                       const T* __restrict__ wpe, int64_t P,
                                                       const W* __restrict__ gamma, const W* __restrict__ beta,
                                                       T* __restrict__ x0, T* __restrict__ y, float* __restrict__ mean_out,
                                                       float* __restrict__ rstd_out, int64_t rows, int C, float eps,
                                                       int* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (NT / kWave) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int64_t id = idx[row], q = pos[row % Tp];
  const bool ok = id >= 0 && id < V, okp = q >= 0 && q < P;
  if (!ok && err != nullptr && lane == 0) atomicOr(err, 1);  // (a vector-memory atomic)
  const T* ta = wte + (ok ? id : 0) * (int64_t)C;
  const T* tb = wpe + (okp ? q : 0) * (int64_t)C;
  const int64_t base = row * C;
  float v[NCH][4], g[NCH][4], b[NCH][4];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
      load4<W>(gamma + c, g[k]);
      load4<W>(beta + c, b[k]);
      float e2[4];
      if (ok) {
        load4<T>(ta + c, v[k]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[k][e] = 0.f;
      }
      if (okp) {
        load4<T>(tb + c, e2);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) e2[e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[k][e] += e2[e];
      store4<T>(x0 + base + c, v[k]);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[k][e] = round_to<T>(v[k][e]);  // normalise what was stored
      s += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
    }
  }
  const float mean = wsum(s) / (float)C;
  float qq = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[k][e] - mean;
        qq = fmaf(d, d, qq);
      }
    }
  }
  const float rstd = rsqrtf(wsum(qq) / (float)C + eps);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = fmaf((v[k][e] - mean) * rstd, g[k][e], b[k][e]);
      store4<T>(y + base + c, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

static void check_rows(const at::Tensor& t, int64_t C, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.size(-1) == C, "norm: ", name, " must be contiguous [..., C]");
  TORCH_CHECK(((uintptr_t)t.data_ptr() & 15) == 0, "norm: ", name, " must be 16-B aligned");
}

template <typename F>
static void dispatch_nch(int64_t C, F&& f) {
  const int64_t n = (C + 255) / 256;
  if (n <= 1) f(std::integral_constant<int, 1>{});
  else if (n == 2) f(std::integral_constant<int, 2>{});
  else if (n == 3) f(std::integral_constant<int, 3>{});
  else if (n == 4) f(std::integral_constant<int, 4>{});
  else if (n <= 6) f(std::integral_constant<int, 6>{});
  else f(std::integral_constant<int, 8>{});
}

template <typename F>
static void dispatch_tw(at::ScalarType t, at::ScalarType w, F&& f) {
  TORCH_CHECK(t == at::kBFloat16 || t == at::kHalf || t == at::kFloat, "norm: unsupported dtype ", t);
  TORCH_CHECK(w == t, "norm: weight dtype must match the input dtype");
  if (t == at::kBFloat16) f(bf16_t{}, bf16_t{});
  else if (t == at::kHalf) f(f16_t{}, f16_t{});
  else f(float{}, float{});
}

template <typename O>
static void launch_reduce(const at::Tensor& part, int nparts, int ld, int W, int C, const at::Tensor& out0,
                          const at::Tensor& out1, int accum, hipStream_t st) {
  hipLaunchKernelGGL((col_reduce_kernel<O>), dim3((W + 15) / 16), dim3(NT), 0, st, part.data_ptr<float>(), nparts, ld,
                     W, C, static_cast<O*>(out0.data_ptr()), out1.defined() ? static_cast<O*>(out1.data_ptr()) : nullptr,
                     accum);
}
// part [nparts][ld] -> out0 = columns [0, C), out1 = columns [C, W) (same dtype; W == C: no out1),
// adding to out0 / out1 for accum bit 0 / 1.  Queued instead (defer.hip) when the caller's
// scope says both outputs are claimed bucket slices.
static void reduce_into(const at::Tensor& part, int nparts, int ld, int W, int C, const at::Tensor& out0,
                        const at::Tensor& out1, int accum, hipStream_t st) {
  if (defer::want() && out0.scalar_type() == at::kBFloat16 &&
      defer::push_colred(part, nparts, ld, W, C, static_cast<uint16_t*>(out0.data_ptr()),
                         out1.defined() ? static_cast<uint16_t*>(out1.data_ptr()) : nullptr, accum, st))
    return;
  switch (out0.scalar_type()) {
    case at::kFloat: launch_reduce<float>(part, nparts, ld, W, C, out0, out1, accum, st); break;
    case at::kBFloat16: launch_reduce<bf16_t>(part, nparts, ld, W, C, out0, out1, accum, st); break;
    case at::kHalf: launch_reduce<f16_t>(part, nparts, ld, W, C, out0, out1, accum, st); break;
    default: TORCH_CHECK(false, "norm: unsupported output dtype");
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

// The 16-B forward (ln_fwd16_kernel) for 2-byte types, C a multiple of 256 (NCH = C / 256 in
// {1, 2, 3, 4, 6, 8}) and 16-B aligned operands; false: use ln_fwd_kernel.  NBD_LN_FWD16=0 (A/B).
template <bool RMS>
static bool launch_fwd16(const at::Tensor& x, const c10::optional<at::Tensor>& delta, const at::Tensor& xsum,
                         const at::Tensor& weight, const at::Tensor* bias, const at::Tensor& y, const at::Tensor& mean,
                         const at::Tensor& rstd, int64_t rows, int64_t C, double eps, hipStream_t st) {
  static const bool on = [] {
    const char* e = std::getenv("NBD_LN_FWD16");
    return e == nullptr || e[0] != '0';
  }();
  const auto dt = x.scalar_type();
  if (!on || (dt != at::kBFloat16 && dt != at::kHalf) || weight.scalar_type() != dt || C % 256 != 0) return false;
  const int nch = (int)(C / 256);
  if (nch != 1 && nch != 2 && nch != 3 && nch != 4 && nch != 6 && nch != 8) return false;
  const bool res = delta.has_value() && delta->defined();
  auto a16 = [](const at::Tensor& t) { return !t.defined() || ((uintptr_t)t.data_ptr() & 15) == 0; };
  if (!a16(x) || !a16(y) || !a16(weight) || (bias != nullptr && (bias->scalar_type() != dt || !a16(*bias))) ||
      (res && (!a16(*delta) || !a16(xsum))))
    return false;
  const dim3 grid((unsigned)((rows + 7) / 8));
  auto go = [&](auto t, auto nc) {
    using T = decltype(t);
    constexpr int N = decltype(nc)::value;
    const T* dp = res ? static_cast<const T*>(delta->data_ptr()) : nullptr;
    T* sp = res ? static_cast<T*>(xsum.data_ptr()) : nullptr;
    const T* bp = bias != nullptr ? static_cast<const T*>(bias->data_ptr()) : nullptr;
    float* mp = RMS ? nullptr : mean.data_ptr<float>();
    if (res)
      hipLaunchKernelGGL((ln_fwd16_kernel<T, T, true, N, RMS>), grid, dim3(NT), 0, st,
                         static_cast<const T*>(x.data_ptr()), dp, sp, static_cast<const T*>(weight.data_ptr()), bp,
                         static_cast<T*>(y.data_ptr()), mp, rstd.data_ptr<float>(), rows, (int)C, (float)eps);
    else
      hipLaunchKernelGGL((ln_fwd16_kernel<T, T, false, N, RMS>), grid, dim3(NT), 0, st,
                         static_cast<const T*>(x.data_ptr()), dp, sp, static_cast<const T*>(weight.data_ptr()), bp,
                         static_cast<T*>(y.data_ptr()), mp, rstd.data_ptr<float>(), rows, (int)C, (float)eps);
  };
  auto by_n = [&](auto t) {
    switch (nch) {
      case 1: go(t, std::integral_constant<int, 1>{}); break;
      case 2: go(t, std::integral_constant<int, 2>{}); break;
      case 3: go(t, std::integral_constant<int, 3>{}); break;
      case 4: go(t, std::integral_constant<int, 4>{}); break;
      case 6: go(t, std::integral_constant<int, 6>{}); break;
      default: go(t, std::integral_constant<int, 8>{}); break;
    }
  };
  if (dt == at::kBFloat16) by_n(bf16_t{});
  else by_n(f16_t{});
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return true;
}

// returns (y, xsum or undefined, mean, rstd)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> ln_fwd_hip(const at::Tensor& x,
                                                                      const c10::optional<at::Tensor>& delta,
                                                                      const at::Tensor& weight,
                                                                      const at::Tensor& bias, double eps) {
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 4 == 0 && C <= 256 * kMaxCh && C > 0, "ln_fwd: C must be a multiple of 4 and <= 2048");
  check_rows(x, C, "x");
  TORCH_CHECK(weight.is_contiguous() && bias.is_contiguous() && weight.numel() == C && bias.numel() == C,
              "ln_fwd: weight/bias must be [C]");
  const bool res = delta.has_value() && delta->defined();
  if (res) {
    check_rows(*delta, C, "delta");
    TORCH_CHECK(delta->sizes() == x.sizes() && delta->scalar_type() == x.scalar_type(), "ln_fwd: delta mismatch");
  }
  const int64_t rows = x.numel() / C;
  at::Tensor y = at::empty_like(x);
  at::Tensor xsum = res ? at::empty_like(x) : at::Tensor();
  auto fo = x.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({rows}, fo), rstd = at::empty({rows}, fo);
  if (rows == 0) return {y, xsum, mean, rstd};
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  if (launch_fwd16<false>(x, delta, xsum, weight, &bias, y, mean, rstd, rows, C, eps, st)) return {y, xsum, mean, rstd};
  const dim3 grid((unsigned)((rows + 3) / 4));
  dispatch_tw(x.scalar_type(), weight.scalar_type(), [&](auto t, auto w) {
   dispatch_nch(C, [&](auto nch) {
    using T = decltype(t);
    using W = decltype(w);
    constexpr int N = decltype(nch)::value;
    if (res)
      hipLaunchKernelGGL((ln_fwd_kernel<T, W, true, N>), grid, dim3(NT), 0, st, static_cast<const T*>(x.data_ptr()),
                         static_cast<const T*>(delta->data_ptr()), static_cast<T*>(xsum.data_ptr()),
                         static_cast<const W*>(weight.data_ptr()), static_cast<const W*>(bias.data_ptr()),
                         static_cast<T*>(y.data_ptr()), mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, (int)C,
                         (float)eps);
    else
      hipLaunchKernelGGL((ln_fwd_kernel<T, W, false, N>), grid, dim3(NT), 0, st, static_cast<const T*>(x.data_ptr()),
                         nullptr, nullptr, static_cast<const W*>(weight.data_ptr()),
                         static_cast<const W*>(bias.data_ptr()), static_cast<T*>(y.data_ptr()),
                         mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, (int)C, (float)eps);
   });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {y, xsum, mean, rstd};
}

// one LayerNorm / RMSNorm backward launch: the 16-B half-wave kernel where it applies (2-byte
// types, C a multiple of 256; NBD_LN_BWD16=0 forces the 8-B kernel for A/B runs)
static bool bwd16_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NBD_LN_BWD16");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <typename T, typename W, int N, bool RMS>
static void launch_bwd(bool res, const at::Tensor& x, const at::Tensor& dy, const T* dr, const at::Tensor& weight,
                       const float* mean, const float* rstd, const at::Tensor& dx, const at::Tensor& pg, int64_t rows,
                       int64_t C, int rpb, int nblk, hipStream_t st) {
  const T* xp = static_cast<const T*>(x.data_ptr());
  const T* dyp = static_cast<const T*>(dy.data_ptr());
  const W* wp = static_cast<const W*>(weight.data_ptr());
  T* dxp = static_cast<T*>(dx.data_ptr());
  float* pgp = pg.data_ptr<float>();
  if constexpr (sizeof(T) == 2) {
    if (C == 256 * N && bwd16_enabled()) {
      if (res)
        hipLaunchKernelGGL((ln_bwd16_kernel<T, W, true, N, RMS>), dim3(nblk), dim3(NT), 0, st, xp, dyp, dr, wp, mean,
                           rstd, dxp, pgp, rows, (int)C, rpb);
      else
        hipLaunchKernelGGL((ln_bwd16_kernel<T, W, false, N, RMS>), dim3(nblk), dim3(NT), 0, st, xp, dyp, dr, wp, mean,
                           rstd, dxp, pgp, rows, (int)C, rpb);
      return;
    }
  }
  auto go = [&](auto rpi) {
    constexpr int R = decltype(rpi)::value;
    if (res)
      hipLaunchKernelGGL((ln_bwd_kernel<T, W, true, N, RMS, R>), dim3(nblk), dim3(NT), 0, st, xp, dyp, dr, wp, mean,
                         rstd, dxp, pgp, rows, (int)C, rpb);
    else
      hipLaunchKernelGGL((ln_bwd_kernel<T, W, false, N, RMS, R>), dim3(nblk), dim3(NT), 0, st, xp, dyp, dr, wp, mean,
                         rstd, dxp, pgp, rows, (int)C, rpb);
  };
  if (rpb == 4) go(std::integral_constant<int, 1>{});  // 4 rows = one per wave
  else go(std::integral_constant<int, 2>{});
}

// returns (dx, dweight, dbias); dx includes dres when given.  dw_dst / db_dst (optional): write
// the weight / bias gradients there (their bucket slices, autograd.hip), adding for accum bit 0 / 1
std::tuple<at::Tensor, at::Tensor, at::Tensor> ln_bwd_into(const at::Tensor& x, const at::Tensor& dy,
                                                           const c10::optional<at::Tensor>& dres,
                                                           const at::Tensor& weight, const at::Tensor& mean,
                                                           const at::Tensor& rstd, const at::Tensor& dw_dst,
                                                           const at::Tensor& db_dst, int accum) {
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 4 == 0 && C <= 256 * kMaxCh && C > 0, "ln_bwd: C must be a multiple of 4 and <= 2048");
  check_rows(x, C, "x");
  check_rows(dy, C, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "ln_bwd: dy mismatch");
  const bool res = dres.has_value() && dres->defined();
  if (res) {
    check_rows(*dres, C, "dres");
    TORCH_CHECK(dres->sizes() == x.sizes() && dres->scalar_type() == x.scalar_type(), "ln_bwd: dres mismatch");
  }
  const int64_t rows = x.numel() / C;
  TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows && mean.scalar_type() == at::kFloat &&
                  rstd.scalar_type() == at::kFloat,
              "ln_bwd: mean/rstd must be float32 [rows]");
  at::Tensor dx = at::empty_like(x);
  at::Tensor dw = dw_dst.defined() ? dw_dst.view({C}) : at::empty({C}, weight.options());
  at::Tensor db = db_dst.defined() ? db_dst.view({C}) : at::empty({C}, weight.options());
  const int rpb = bwd_rows_per_block(rows);
  const int nblk = (int)((rows + rpb - 1) / rpb);
  if (rows == 0) {
    if (!(accum & 1)) dw.zero_();
    if (!(accum & 2)) db.zero_();
    return {dx, dw, db};
  }
  auto fo = x.options().dtype(at::kFloat);
  at::Tensor pg = at::empty({nblk, 2 * C}, fo);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  dispatch_tw(x.scalar_type(), weight.scalar_type(), [&](auto t, auto w) {
   dispatch_nch(C, [&](auto nch) {
    using T = decltype(t);
    using W = decltype(w);
    constexpr int N = decltype(nch)::value;
    const T* dr = res ? static_cast<const T*>(dres->data_ptr()) : nullptr;
    launch_bwd<T, W, N, false>(res, x, dy, dr, weight, mean.data_ptr<float>(), rstd.data_ptr<float>(), dx, pg, rows,
                               C, rpb, nblk, st);
   });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  reduce_into(pg, nblk, (int)(2 * C), (int)(2 * C), (int)C, dw, db, accum, st);
  return {dx, dw, db};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> ln_bwd_hip(const at::Tensor& x, const at::Tensor& dy,
                                                          const c10::optional<at::Tensor>& dres,
                                                          const at::Tensor& weight, const at::Tensor& mean,
                                                          const at::Tensor& rstd) {
  return ln_bwd_into(x, dy, dres, weight, mean, rstd, at::Tensor(), at::Tensor(), 0);
}

// RMSNorm: y = x · rsqrt(mean(x²) + eps) · g  (optionally on x + delta, returned as xsum)
std::tuple<at::Tensor, at::Tensor, at::Tensor> rms_fwd_hip(const at::Tensor& x, const c10::optional<at::Tensor>& delta,
                                                           const at::Tensor& weight, double eps) {
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 4 == 0 && C <= 256 * kMaxCh && C > 0, "rms_fwd: C must be a multiple of 4 and <= 2048");
  check_rows(x, C, "x");
  TORCH_CHECK(weight.is_contiguous() && weight.numel() == C, "rms_fwd: weight must be [C]");
  const bool res = delta.has_value() && delta->defined();
  if (res) {
    check_rows(*delta, C, "delta");
    TORCH_CHECK(delta->sizes() == x.sizes() && delta->scalar_type() == x.scalar_type(), "rms_fwd: delta mismatch");
  }
  const int64_t rows = x.numel() / C;
  at::Tensor y = at::empty_like(x);
  at::Tensor xsum = res ? at::empty_like(x) : at::Tensor();
  auto fo = x.options().dtype(at::kFloat);
  at::Tensor rstd = at::empty({rows}, fo);
  if (rows == 0) return {y, xsum, rstd};
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  if (launch_fwd16<true>(x, delta, xsum, weight, nullptr, y, at::Tensor(), rstd, rows, C, eps, st)) return {y, xsum, rstd};
  const dim3 grid((unsigned)((rows + 3) / 4));
  dispatch_tw(x.scalar_type(), weight.scalar_type(), [&](auto t, auto w) {
   dispatch_nch(C, [&](auto nch) {
    using T = decltype(t);
    using W = decltype(w);
    constexpr int N = decltype(nch)::value;
    const T* dp = res ? static_cast<const T*>(delta->data_ptr()) : nullptr;
    T* sp = res ? static_cast<T*>(xsum.data_ptr()) : nullptr;
    if (res)
      hipLaunchKernelGGL((ln_fwd_kernel<T, W, true, N, true>), grid, dim3(NT), 0, st,
                         static_cast<const T*>(x.data_ptr()), dp, sp, static_cast<const W*>(weight.data_ptr()),
                         nullptr, static_cast<T*>(y.data_ptr()), nullptr, rstd.data_ptr<float>(), rows,
                         (int)C, (float)eps);
    else
      hipLaunchKernelGGL((ln_fwd_kernel<T, W, false, N, true>), grid, dim3(NT), 0, st,
                         static_cast<const T*>(x.data_ptr()), dp, sp, static_cast<const W*>(weight.data_ptr()),
                         nullptr, static_cast<T*>(y.data_ptr()), nullptr, rstd.data_ptr<float>(), rows,
                         (int)C, (float)eps);
   });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {y, xsum, rstd};
}

// (x0, y, rstd) of embed_rms_kernel: x0 / y shaped ids.shape + [C]
std::tuple<at::Tensor, at::Tensor, at::Tensor> embed_rms_fwd_hip(const at::Tensor& ids, const at::Tensor& table,
                                                                 const at::Tensor& weight, double eps,
                                                                 const c10::optional<at::Tensor>& err) {
  TORCH_CHECK(ids.is_cuda() && table.is_cuda() && weight.is_cuda(), "embed_rms: GPU tensors expected");
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous(), "embed_rms: contiguous int64 ids expected");
  TORCH_CHECK(table.dim() == 2 && table.is_contiguous(), "embed_rms: contiguous [V, C] table expected");
  const int64_t C = table.size(1), V = table.size(0);
  TORCH_CHECK(C % 4 == 0 && C <= 256 * kMaxCh && C > 0, "embed_rms: C must be a multiple of 4 and <= 2048");
  TORCH_CHECK(((uintptr_t)table.data_ptr() & 7) == 0, "embed_rms: 8-B aligned table expected");
  TORCH_CHECK(weight.is_contiguous() && weight.numel() == C, "embed_rms: weight must be [C]");
  if (err) TORCH_CHECK(err->is_cuda() && err->scalar_type() == at::kInt && err->numel() >= 1, "embed_rms: int32 error flag");
  std::vector<int64_t> shape(ids.sizes().begin(), ids.sizes().end());
  shape.push_back(C);
  at::Tensor x0 = at::empty(shape, table.options()), y = at::empty(shape, table.options());
  const int64_t rows = ids.numel();
  at::Tensor rstd = at::empty({rows}, table.options().dtype(at::kFloat));
  if (rows == 0) return {x0, y, rstd};
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(table.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const dim3 grid((unsigned)((rows + 3) / 4));
  dispatch_tw(table.scalar_type(), weight.scalar_type(), [&](auto t, auto w) {
   dispatch_nch(C, [&](auto nch) {
    using T = decltype(t);
    using W = decltype(w);
    constexpr int N = decltype(nch)::value;
    hipLaunchKernelGGL((embed_rms_kernel<T, W, N>), grid, dim3(NT), 0, st, ids.data_ptr<int64_t>(),
                       static_cast<const T*>(table.data_ptr()), V, static_cast<const W*>(weight.data_ptr()),
                       static_cast<T*>(x0.data_ptr()), static_cast<T*>(y.data_ptr()), rstd.data_ptr<float>(), rows,
                       (int)C, (float)eps, err ? err->data_ptr<int>() : nullptr);
   });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {x0, y, rstd};
}

// (x0, y, mean, rstd) of tokpos_ln_kernel: x0 / y shaped idx.shape + [C]; vocab < wte rows: the
// rows past it are padding (ids there are out of range)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> tokpos_ln_fwd_hip(
    const at::Tensor& idx, const at::Tensor& wte, const at::Tensor& pos, const at::Tensor& wpe, int64_t vocab,
    const at::Tensor& weight, const at::Tensor& bias, double eps, const c10::optional<at::Tensor>& err) {
  TORCH_CHECK(idx.is_cuda() && wte.is_cuda() && pos.is_cuda() && wpe.is_cuda(), "tokpos_ln: GPU tensors expected");
  TORCH_CHECK(idx.scalar_type() == at::kLong && pos.scalar_type() == at::kLong && idx.is_contiguous() &&
                  pos.is_contiguous() && pos.dim() == 1 && pos.numel() > 0 && idx.numel() % pos.numel() == 0,
              "tokpos_ln: int64 ids [..., T] and positions [T]");
  TORCH_CHECK(wte.dim() == 2 && wpe.dim() == 2 && wte.size(1) == wpe.size(1) && wte.is_contiguous() &&
                  wpe.is_contiguous() && wte.scalar_type() == wpe.scalar_type(),
              "tokpos_ln: contiguous [V, C] / [P, C] tables of one dtype");
  const int64_t C = wte.size(1);
  TORCH_CHECK(C % 4 == 0 && C <= 256 * kMaxCh && C > 0, "tokpos_ln: C must be a multiple of 4 and <= 2048");
  TORCH_CHECK(((uintptr_t)wte.data_ptr() & 7) == 0 && ((uintptr_t)wpe.data_ptr() & 7) == 0,
              "tokpos_ln: 8-B aligned tables expected");
  TORCH_CHECK(weight.is_contiguous() && bias.is_contiguous() && weight.numel() == C && bias.numel() == C,
              "tokpos_ln: weight / bias must be [C]");
  if (err) TORCH_CHECK(err->is_cuda() && err->scalar_type() == at::kInt && err->numel() >= 1, "tokpos_ln: int32 error flag");
  const int64_t V = vocab > 0 ? std::min<int64_t>(vocab, wte.size(0)) : wte.size(0);
  std::vector<int64_t> shape(idx.sizes().begin(), idx.sizes().end());
  shape.push_back(C);
  at::Tensor x0 = at::empty(shape, wte.options()), y = at::empty(shape, wte.options());
  const int64_t rows = idx.numel();
  auto fo = wte.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({rows}, fo), rstd = at::empty({rows}, fo);
  if (rows == 0) return {x0, y, mean, rstd};
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(wte.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const dim3 grid((unsigned)((rows + 3) / 4));
  dispatch_tw(wte.scalar_type(), weight.scalar_type(), [&](auto t, auto w) {
   dispatch_nch(C, [&](auto nch) {
    using T = decltype(t);
    using W = decltype(w);
    constexpr int N = decltype(nch)::value;
    hipLaunchKernelGGL((tokpos_ln_kernel<T, W, N>), grid, dim3(NT), 0, st, idx.data_ptr<int64_t>(),
                       static_cast<const T*>(wte.data_ptr()), V, pos.data_ptr<int64_t>(), (int)pos.numel(),
                       static_cast<const T*>(wpe.data_ptr()), wpe.size(0), static_cast<const W*>(weight.data_ptr()),
                       static_cast<const W*>(bias.data_ptr()), static_cast<T*>(x0.data_ptr()),
                       static_cast<T*>(y.data_ptr()), mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, (int)C,
                       (float)eps, err ? err->data_ptr<int>() : nullptr);
   });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {x0, y, mean, rstd};
}

std::tuple<at::Tensor, at::Tensor> rms_bwd_into(const at::Tensor& x, const at::Tensor& dy,
                                                const c10::optional<at::Tensor>& dres, const at::Tensor& weight,
                                                const at::Tensor& rstd, const at::Tensor& dw_dst, int accum) {
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 4 == 0 && C <= 256 * kMaxCh && C > 0, "rms_bwd: C must be a multiple of 4 and <= 2048");
  check_rows(x, C, "x");
  check_rows(dy, C, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.scalar_type() == x.scalar_type(), "rms_bwd: dy mismatch");
  const bool res = dres.has_value() && dres->defined();
  if (res) {
    check_rows(*dres, C, "dres");
    TORCH_CHECK(dres->sizes() == x.sizes() && dres->scalar_type() == x.scalar_type(), "rms_bwd: dres mismatch");
  }
  const int64_t rows = x.numel() / C;
  TORCH_CHECK(rstd.numel() == rows && rstd.scalar_type() == at::kFloat, "rms_bwd: rstd must be float32 [rows]");
  at::Tensor dx = at::empty_like(x);
  at::Tensor dw = dw_dst.defined() ? dw_dst.view({C}) : at::empty({C}, weight.options());
  const int rpb = bwd_rows_per_block(rows);
  const int nblk = (int)((rows + rpb - 1) / rpb);
  if (rows == 0) {
    if (!(accum & 1)) dw.zero_();
    return {dx, dw};
  }
  at::Tensor pg = at::empty({nblk, 2 * C}, x.options().dtype(at::kFloat));
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  dispatch_tw(x.scalar_type(), weight.scalar_type(), [&](auto t, auto w) {
   dispatch_nch(C, [&](auto nch) {
    using T = decltype(t);
    using W = decltype(w);
    constexpr int N = decltype(nch)::value;
    const T* dr = res ? static_cast<const T*>(dres->data_ptr()) : nullptr;
    launch_bwd<T, W, N, true>(res, x, dy, dr, weight, rstd.data_ptr<float>(), rstd.data_ptr<float>(), dx, pg, rows, C,
                              rpb, nblk, st);
   });
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  // the partial rows are [dγ | Σdy] (the kernel is LayerNorm's); RMSNorm sums the first half only
  reduce_into(pg, nblk, (int)(2 * C), (int)C, (int)C, dw, at::Tensor(), accum & 1, st);
  return {dx, dw};
}

std::tuple<at::Tensor, at::Tensor> rms_bwd_hip(const at::Tensor& x, const at::Tensor& dy,
                                               const c10::optional<at::Tensor>& dres, const at::Tensor& weight,
                                               const at::Tensor& rstd) {
  return rms_bwd_into(x, dy, dres, weight, rstd, at::Tensor(), 0);
}

// Σ over rows of a contiguous [..., C] tensor -> [C] in `dtype` (fp32 accumulation)
at::Tensor colsum_hip(const at::Tensor& x, at::ScalarType dtype) {
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && C > 0, "colsum: C must be a multiple of 8");
  check_rows(x, C, "x");
  const int64_t rows = x.numel() / C;
  at::Tensor out = at::empty({C}, x.options().dtype(dtype));
  if (rows == 0) return out.zero_();
  const int nblk = (int)((rows + kColRows - 1) / kColRows);
  at::Tensor part = at::empty({nblk, C}, x.options().dtype(at::kFloat));
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const dim3 grid((unsigned)nblk, (unsigned)((C / 8 + NT - 1) / NT));
  switch (x.scalar_type()) {
    case at::kFloat:
      hipLaunchKernelGGL((colsum_kernel<float>), grid, dim3(NT), 0, st, x.data_ptr<float>(), rows, (int)C,
                         part.data_ptr<float>());
      break;
    case at::kBFloat16:
      hipLaunchKernelGGL((colsum_kernel<bf16_t>), grid, dim3(NT), 0, st, static_cast<const bf16_t*>(x.data_ptr()),
                         rows, (int)C, part.data_ptr<float>());
      break;
    case at::kHalf:
      hipLaunchKernelGGL((colsum_kernel<f16_t>), grid, dim3(NT), 0, st, static_cast<const f16_t*>(x.data_ptr()), rows,
                         (int)C, part.data_ptr<float>());
      break;
    default: TORCH_CHECK(false, "colsum: unsupported dtype ", x.scalar_type());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  reduce_into(part, nblk, (int)C, (int)C, (int)C, out, at::Tensor(), 0, st);
  return out;
}

}  // namespace norm
}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("ln_fwd", &nbd::norm::ln_fwd_hip);
  m.impl("ln_bwd", &nbd::norm::ln_bwd_hip);
  m.impl("colsum", &nbd::norm::colsum_hip);
  m.impl("rms_fwd", &nbd::norm::rms_fwd_hip);
  m.impl("rms_bwd", &nbd::norm::rms_bwd_hip);
}
