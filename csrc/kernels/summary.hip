// summary.hip — one-pass on-device tensor summary for the REPL echo (K4).
//
// Computes count, sum, mean, std, L2 norm, min, max, absmax, #NaN and #Inf of a GPU tensor in a
// single HBM pass plus a one-block finalize, returning 12 float64s (one 96-byte D2H copy for the
// echo) instead of pulling tensor data to the host (reference: repr() of the cell's last value,
// worker.py:292, 341, and get_var's full value.cpu() copy, worker.py:414).
//
// bf16 / f16 inputs: the sum and the sum of squares run on the matrix cores.  One
// v_mfma_f32_16x16x32_bf16 consumes a 16x32 tile A held as 8 elements per lane — exactly one
// coalesced 16-byte load per lane (1 KiB per wave-instruction):
//   * mfma(A, ones)  -> every column of D holds the 16 row sums of A          (Σx)
//   * mfma(A, A)     -> the same registers as the B operand are Aᵀ (B[k][c] = A[c][k] by the
//                       gfx950 operand lane maps), so D = A·Aᵀ and its diagonal holds the 16
//                       row sums of squares                                    (Σx²)
// Both are permutation-invariant, so the tile layout is simply "lane l holds 16 contiguous
// bytes": no shuffles, no LDS.  Products of bf16/f16 are exact in f32 and accumulate in f32 in
// the matrix pipe, which runs beside the VALU: the VALU only does the conversions and the
// min/max/absmax/NaN/Inf bookkeeping.
// f32 inputs: the f32-input MFMA (16x16x4) runs at the VALU rate and would cost 2 matrix ops per
// 64 elements, so the f32 path uses shifted VALU sums (x - x0, better conditioned variance).
//
// Cross-block combine: per-block partials (f32, 8 values) -> finalize kernel in f64.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>
#include <cmath>

#include "nbd_common.h"

namespace nbd {

constexpr int kSumThreads = 256;
constexpr int kWavesPerBlock = kSumThreads / kWave;
constexpr int kMaxBlocks = 2048;  // 256 CUs x 8 resident blocks
constexpr int kNPart = 8;         // sum, sumsq, min, max, absmax, nan, inf, count

struct Acc {
  float mn, mx, amx, nan, inf;
};

__device__ __forceinline__ void acc_init(Acc& a) {
  a.mn = INFINITY;
  a.mx = -INFINITY;
  a.amx = 0.f;
  a.nan = 0.f;
  a.inf = 0.f;
}

__device__ __forceinline__ void acc_elem(Acc& a, float x) {
  // fminf/fmaxf ignore NaN (IEEE minNum/maxNum): min/max are over the non-NaN values
  a.mn = fminf(a.mn, x);
  a.mx = fmaxf(a.mx, x);
  a.amx = fmaxf(a.amx, fabsf(x));
  a.nan += (x != x) ? 1.f : 0.f;
  a.inf += (fabsf(x) == INFINITY) ? 1.f : 0.f;
}

// Block reduction of the 8 partials; thread 0 writes them.
__device__ __forceinline__ void block_store(float s, float q, const Acc& a, float cnt, float* part) {
  __shared__ float red[kWavesPerBlock][kNPart];
  s = wave_reduce(s, [](float x, float y) { return x + y; });
  q = wave_reduce(q, [](float x, float y) { return x + y; });
  float mn = wave_reduce(a.mn, [](float x, float y) { return fminf(x, y); });
  float mx = wave_reduce(a.mx, [](float x, float y) { return fmaxf(x, y); });
  float amx = wave_reduce(a.amx, [](float x, float y) { return fmaxf(x, y); });
  float nan = wave_reduce(a.nan, [](float x, float y) { return x + y; });
  float inf = wave_reduce(a.inf, [](float x, float y) { return x + y; });
  cnt = wave_reduce(cnt, [](float x, float y) { return x + y; });
  const int w = threadIdx.x / kWave, l = threadIdx.x % kWave;
  if (l == 0) {
    red[w][0] = s; red[w][1] = q; red[w][2] = mn; red[w][3] = mx;
    red[w][4] = amx; red[w][5] = nan; red[w][6] = inf; red[w][7] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float r[kNPart];
#pragma unroll
    for (int k = 0; k < kNPart; ++k) r[k] = red[0][k];
    for (int ww = 1; ww < kWavesPerBlock; ++ww) {
      r[0] += red[ww][0]; r[1] += red[ww][1];
      r[2] = fminf(r[2], red[ww][2]); r[3] = fmaxf(r[3], red[ww][3]); r[4] = fmaxf(r[4], red[ww][4]);
      r[5] += red[ww][5]; r[6] += red[ww][6]; r[7] += red[ww][7];
    }
    float* p = part + (size_t)blockIdx.x * kNPart;
#pragma unroll
    for (int k = 0; k < kNPart; ++k) p[k] = r[k];
  }
}

// ---- 16-bit inputs: MFMA sums --------------------------------------------------------------
// One wave tile = 512 elements = 64 lanes x 16 B.  Tiles are dealt round-robin to all waves of
// the grid; the (< 512-element) tail and any misaligned head are done on the VALU by block 0.
template <bool IS_BF16>
__global__ __launch_bounds__(kSumThreads) void summary16_kernel(const uint16_t* __restrict__ x, int64_t head,
                                                                int64_t ntiles, int64_t n, float* __restrict__ part) {
  const int lane = threadIdx.x % kWave;
  const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
  f32x4 acc_s = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc_q = {0.f, 0.f, 0.f, 0.f};
  Acc a;
  acc_init(a);
  const uint16_t* body = x + head;
  bf16x8 ones;
  {
    const short one = IS_BF16 ? (short)0x3F80 : (short)0x3C00;  // 1.0 in bf16 / f16
#pragma unroll
    for (int j = 0; j < 8; ++j) ones[j] = one;
  }
  int64_t t = wave;
  // two tiles per iteration: both loads in flight before the math
  for (; t + nwaves < ntiles; t += 2 * nwaves) {
    const u32x4 w0 = *reinterpret_cast<const u32x4*>(body + t * 512 + lane * 8);
    const u32x4 w1 = *reinterpret_cast<const u32x4*>(body + (t + nwaves) * 512 + lane * 8);
    const bf16x8 f0 = __builtin_bit_cast(bf16x8, w0);
    const bf16x8 f1 = __builtin_bit_cast(bf16x8, w1);
    if (IS_BF16) {
      acc_s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0, ones, acc_s, 0, 0, 0);
      acc_q = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0, f0, acc_q, 0, 0, 0);
      acc_s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1, ones, acc_s, 0, 0, 0);
      acc_q = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1, f1, acc_q, 0, 0, 0);
    } else {
      const f16x8 h0 = __builtin_bit_cast(f16x8, w0), h1 = __builtin_bit_cast(f16x8, w1);
      const f16x8 ho = __builtin_bit_cast(f16x8, ones);
      acc_s = __builtin_amdgcn_mfma_f32_16x16x32_f16(h0, ho, acc_s, 0, 0, 0);
      acc_q = __builtin_amdgcn_mfma_f32_16x16x32_f16(h0, h0, acc_q, 0, 0, 0);
      acc_s = __builtin_amdgcn_mfma_f32_16x16x32_f16(h1, ho, acc_s, 0, 0, 0);
      acc_q = __builtin_amdgcn_mfma_f32_16x16x32_f16(h1, h1, acc_q, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t u0 = w0[j], u1 = w1[j];
      if (IS_BF16) {
        acc_elem(a, __uint_as_float(u0 << 16)); acc_elem(a, __uint_as_float(u0 & 0xffff0000u));
        acc_elem(a, __uint_as_float(u1 << 16)); acc_elem(a, __uint_as_float(u1 & 0xffff0000u));
      } else {
        acc_elem(a, f16_to_f32((uint16_t)(u0 & 0xffffu))); acc_elem(a, f16_to_f32((uint16_t)(u0 >> 16)));
        acc_elem(a, f16_to_f32((uint16_t)(u1 & 0xffffu))); acc_elem(a, f16_to_f32((uint16_t)(u1 >> 16)));
      }
    }
  }
  for (; t < ntiles; t += nwaves) {
    const u32x4 w0 = *reinterpret_cast<const u32x4*>(body + t * 512 + lane * 8);
    const bf16x8 f0 = __builtin_bit_cast(bf16x8, w0);
    if (IS_BF16) {
      acc_s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0, ones, acc_s, 0, 0, 0);
      acc_q = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f0, f0, acc_q, 0, 0, 0);
    } else {
      const f16x8 h0 = __builtin_bit_cast(f16x8, w0), ho = __builtin_bit_cast(f16x8, ones);
      acc_s = __builtin_amdgcn_mfma_f32_16x16x32_f16(h0, ho, acc_s, 0, 0, 0);
      acc_q = __builtin_amdgcn_mfma_f32_16x16x32_f16(h0, h0, acc_q, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t u0 = w0[j];
      if (IS_BF16) {
        acc_elem(a, __uint_as_float(u0 << 16)); acc_elem(a, __uint_as_float(u0 & 0xffff0000u));
      } else {
        acc_elem(a, f16_to_f32((uint16_t)(u0 & 0xffffu))); acc_elem(a, f16_to_f32((uint16_t)(u0 >> 16)));
      }
    }
  }
  // D layout (16x16x32): col = lane & 15, row = 4*(lane >> 4) + reg.
  // Σx: the row sums are replicated over the 16 columns -> take column 0 (lanes 0, 16, 32, 48).
  // Σx²: diagonal elements row == col -> lanes with (lane & 15) >> 2 == lane >> 4, reg = (lane & 15) & 3.
  const int col = lane & 15, grp = lane >> 4;
  float s = (col == 0) ? (acc_s[0] + acc_s[1] + acc_s[2] + acc_s[3]) : 0.f;
  float q = 0.f;
  if ((col >> 2) == grp) {
    const int r = col & 3;
    q = (r == 0) ? acc_q[0] : (r == 1) ? acc_q[1] : (r == 2) ? acc_q[2] : acc_q[3];
  }
  // VALU part of the work: misaligned head + tail, block 0 only.
  if (blockIdx.x == 0) {
    const int64_t tail0 = head + ntiles * 512;
    for (int64_t i = threadIdx.x; i < head; i += kSumThreads) {
      const float v = IS_BF16 ? bf16_to_f32(x[i]) : f16_to_f32(x[i]);
      s += v; q = fmaf(v, v, q); acc_elem(a, v);
    }
    for (int64_t i = tail0 + threadIdx.x; i < n; i += kSumThreads) {
      const float v = IS_BF16 ? bf16_to_f32(x[i]) : f16_to_f32(x[i]);
      s += v; q = fmaf(v, v, q); acc_elem(a, v);
    }
  }
  block_store(s, q, a, 0.f, part);
}

// ---- f32 inputs: shifted VALU sums -----------------------------------------------------------
__device__ __forceinline__ float pick_shift(const float* x, int64_t n) {
  // shift by the first element (read on the device, no host sync) when it is finite
  if (n <= 0) return 0.f;
  const float v = x[0];
  return (fabsf(v) < INFINITY) ? v : 0.f;
}

__global__ __launch_bounds__(kSumThreads) void summary32_kernel(const float* __restrict__ x, int64_t head, int64_t nvec,
                                                                int64_t n, float* __restrict__ part) {
  const float shift = pick_shift(x, n);
  const int64_t tid = (int64_t)blockIdx.x * kSumThreads + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * kSumThreads;
  float s0 = 0.f, s1 = 0.f, q0 = 0.f, q1 = 0.f;
  Acc a;
  acc_init(a);
  const float* body = x + head;
  int64_t v = tid;
  for (; v + nth < nvec; v += 2 * nth) {
    const f32x4 p = *reinterpret_cast<const f32x4*>(body + v * 4);
    const f32x4 r = *reinterpret_cast<const f32x4*>(body + (v + nth) * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d0 = p[j] - shift, d1 = r[j] - shift;
      s0 += d0; q0 = fmaf(d0, d0, q0);
      s1 += d1; q1 = fmaf(d1, d1, q1);
      acc_elem(a, p[j]); acc_elem(a, r[j]);
    }
  }
  for (; v < nvec; v += nth) {
    const f32x4 p = *reinterpret_cast<const f32x4*>(body + v * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d0 = p[j] - shift;
      s0 += d0; q0 = fmaf(d0, d0, q0);
      acc_elem(a, p[j]);
    }
  }
  if (blockIdx.x == 0) {
    const int64_t tail0 = head + nvec * 4;
    for (int64_t i = threadIdx.x; i < head; i += kSumThreads) {
      const float d = x[i] - shift;
      s0 += d; q0 = fmaf(d, d, q0); acc_elem(a, x[i]);
    }
    for (int64_t i = tail0 + threadIdx.x; i < n; i += kSumThreads) {
      const float d = x[i] - shift;
      s0 += d; q0 = fmaf(d, d, q0); acc_elem(a, x[i]);
    }
  }
  block_store(s0 + s1, q0 + q1, a, 0.f, part);
}

// ---- finalize (one block, f64) ----------------------------------------------------------------
// out: [count, sum, mean, std, l2norm, min, max, absmax, nan, inf, numel_finite, shift]
__global__ __launch_bounds__(kSumThreads) void summary_finalize_kernel(const float* __restrict__ part, int nblocks,
                                                                       int64_t n, const float* __restrict__ xf32,
                                                                       double* __restrict__ out) {
  const double shift = xf32 != nullptr ? (double)pick_shift(xf32, n) : 0.0;
  __shared__ double red[kSumThreads][4];
  __shared__ float redf[kSumThreads][4];
  double s = 0, q = 0, nan = 0, inf = 0;
  float mn = INFINITY, mx = -INFINITY, amx = 0.f;
  for (int b = threadIdx.x; b < nblocks; b += kSumThreads) {
    const float* p = part + (size_t)b * kNPart;
    s += p[0]; q += p[1];
    mn = fminf(mn, p[2]); mx = fmaxf(mx, p[3]); amx = fmaxf(amx, p[4]);
    nan += p[5]; inf += p[6];
  }
  red[threadIdx.x][0] = s; red[threadIdx.x][1] = q; red[threadIdx.x][2] = nan; red[threadIdx.x][3] = inf;
  redf[threadIdx.x][0] = mn; redf[threadIdx.x][1] = mx; redf[threadIdx.x][2] = amx;
  __syncthreads();
  for (int off = kSumThreads / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      for (int k = 0; k < 4; ++k) red[threadIdx.x][k] += red[threadIdx.x + off][k];
      redf[threadIdx.x][0] = fminf(redf[threadIdx.x][0], redf[threadIdx.x + off][0]);
      redf[threadIdx.x][1] = fmaxf(redf[threadIdx.x][1], redf[threadIdx.x + off][1]);
      redf[threadIdx.x][2] = fmaxf(redf[threadIdx.x][2], redf[threadIdx.x + off][2]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double ds = red[0][0], dq = red[0][1];  // sums of (x - shift)
    const double cnt = (double)n;
    const double sum = ds + cnt * shift;
    const double mean = cnt > 0 ? sum / cnt : NAN;
    double var = cnt > 1 ? (dq - ds * ds / cnt) / (cnt - 1) : NAN;
    if (var < 0) var = 0;
    const double sumsq = dq + 2.0 * shift * ds + cnt * shift * shift;
    out[0] = cnt;
    out[1] = sum;
    out[2] = mean;
    out[3] = sqrt(var);
    out[4] = sqrt(sumsq > 0 ? sumsq : 0.0);
    out[5] = redf[0][0];
    out[6] = redf[0][1];
    out[7] = redf[0][2];
    out[8] = red[0][2];
    out[9] = red[0][3];
    out[10] = cnt - red[0][2] - red[0][3];
    out[11] = shift;
  }
}

at::Tensor tensor_summary_hip(const at::Tensor& x_) {
  TORCH_CHECK(x_.is_cuda(), "tensor_summary_hip: GPU tensor expected");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x_.device());
  at::Tensor x = x_.contiguous();
  const at::ScalarType dt = x.scalar_type();
  TORCH_CHECK(dt == at::kFloat || dt == at::kBFloat16 || dt == at::kHalf,
              "tensor_summary_hip: float32 / bfloat16 / float16 only (got ", dt, ")");
  const int64_t n = x.numel();
  auto out = at::empty({12}, x.options().dtype(at::kDouble));
  hipStream_t stream = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int64_t es = (int64_t)x.element_size();
  const uintptr_t addr = (uintptr_t)x.data_ptr();
  int64_t head = addr % 16 ? std::min<int64_t>(n, (int64_t)((16 - addr % 16) / es)) : 0;
  if (addr % es) head = n;  // not even element aligned: all on the VALU path
  const int64_t rest = n - head;
  int blocks;
  at::Tensor part;
  if (dt == at::kFloat) {
    const int64_t nvec = rest / 4;
    blocks = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxBlocks, (nvec + 2 * kSumThreads - 1) / (2 * kSumThreads)));
    part = at::empty({blocks * kNPart}, x.options().dtype(at::kFloat));
    // shifted sums (x - x[0]): well-conditioned variance for tensors whose mean is large
    // compared with their spread
    const float* xp = static_cast<const float*>(x.data_ptr());
    hipLaunchKernelGGL(summary32_kernel, dim3(blocks), dim3(kSumThreads), 0, stream, xp, head, nvec, n,
                       part.data_ptr<float>());
    C10_HIP_KERNEL_LAUNCH_CHECK();
    hipLaunchKernelGGL(summary_finalize_kernel, dim3(1), dim3(kSumThreads), 0, stream, part.data_ptr<float>(), blocks,
                       n, xp, out.data_ptr<double>());
  } else {
    const int64_t ntiles = rest / 512;
    const int64_t waves = std::max<int64_t>(1, (ntiles + 1) / 2);
    blocks = (int)std::max<int64_t>(1, std::min<int64_t>(kMaxBlocks, (waves + kWavesPerBlock - 1) / kWavesPerBlock));
    part = at::empty({blocks * kNPart}, x.options().dtype(at::kFloat));
    const uint16_t* p = static_cast<const uint16_t*>(x.data_ptr());
    if (dt == at::kBFloat16)
      hipLaunchKernelGGL(summary16_kernel<true>, dim3(blocks), dim3(kSumThreads), 0, stream, p, head, ntiles, n,
                         part.data_ptr<float>());
    else
      hipLaunchKernelGGL(summary16_kernel<false>, dim3(blocks), dim3(kSumThreads), 0, stream, p, head, ntiles, n,
                         part.data_ptr<float>());
    C10_HIP_KERNEL_LAUNCH_CHECK();
    hipLaunchKernelGGL(summary_finalize_kernel, dim3(1), dim3(kSumThreads), 0, stream, part.data_ptr<float>(), blocks,
                       n, static_cast<const float*>(nullptr), out.data_ptr<double>());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) { m.impl("tensor_summary", &nbd::tensor_summary_hip); }
