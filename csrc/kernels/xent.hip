// xent.hip — fused softmax cross-entropy over large-vocabulary logits (GPT-2: 8192 x 50257 bf16).
//
// The eager path (F.cross_entropy(logits.float(), y)) materialises an fp32 copy of the logits,
// a log_softmax output, its backward, a zero-filled grad and a bf16 cast: ~8 GB of HBM traffic
// per GPT-2 step (rocprof: ~3 ms of a 22.7 ms step, profiles/gpt2_step_rocprof_r1.md).  Here:
//
//   forward   one read of the logits.  One 256-thread workgroup per row keeps an online
//             (max, sum-of-exp) pair per lane in base 2 (v_exp_f32), merges lanes with wave64
//             shuffles and the 4 waves through LDS, and writes lse[row] and
//             loss[row] = lse - x[target] (0 for ignore_index rows).
//   backward  one read + one write: d x = (exp(x - lse) - onehot(target)) * scale, scale =
//             grad_out / n_valid read from device memory (no host sync), stored in the logits'
//             dtype — optionally in place over the logits (they are dead after the loss: the
//             LM-head GEMM's backward needs its inputs, not its output).
//
// Rows of an odd vocabulary are not 16-B aligned: each row runs a scalar head up to the first
// 16-B boundary, then 16-B-per-lane vector loads, then a scalar tail.  Grid = one workgroup per
// row (8192 rows = 32 workgroups per CU on 256 CUs).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <cmath>
#include <tuple>

#include "nbd_common.h"

namespace nbd {

constexpr int kXentThreads = 256;
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

struct OnlineLse {
  float m = -INFINITY;  // running max (base-2 scaled)
  float s = 0.f;        // sum of exp2(t - m)

  __device__ __forceinline__ void add(float t) {
    if (t > m) {
      s = s * __builtin_amdgcn_exp2f(m - t) + 1.f;  // exp2(-inf) = 0 on the first element
      m = t;
    } else if (m != -INFINITY) {
      s += __builtin_amdgcn_exp2f(t - m);
    }
  }
  __device__ __forceinline__ void add8(const float (&v)[8]) {
    float t[8];
    float cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      t[j] = v[j] * kLog2e;
      cm = fmaxf(cm, t[j]);
    }
    if (cm == -INFINITY) return;  // all masked
    if (cm > m) {
      s *= __builtin_amdgcn_exp2f(m - cm);
      m = cm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __builtin_amdgcn_exp2f(t[j] - m);
  }
  __device__ __forceinline__ void merge(float m2, float s2) {
    const float M = fmaxf(m, m2);
    if (M == -INFINITY) return;
    s = s * __builtin_amdgcn_exp2f(m - M) + s2 * __builtin_amdgcn_exp2f(m2 - M);
    m = M;
  }
};

template <typename T>
__device__ __forceinline__ int64_t head_elems(const T* p, int64_t V) {
  const int64_t h = (int64_t)(((16u - ((uintptr_t)p & 15u)) & 15u) / sizeof(T));
  return h < V ? h : V;
}

template <typename T>
__global__ __launch_bounds__(kXentThreads) void xent_fwd_kernel(const T* __restrict__ logits, int64_t ld,
                                                                const int64_t* __restrict__ target, int64_t V,
                                                                int64_t ignore_index, float* __restrict__ loss,
                                                                float* __restrict__ lse_out) {
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  const int tid = threadIdx.x;
  OnlineLse acc;
  const int64_t head = head_elems(x, V);
  if (tid < head) acc.add(Elem<T>::load(x, tid) * kLog2e);
  const T* xv = x + head;
  const int64_t nv = (V - head) / 8;
  for (int64_t k = tid; k < nv; k += kXentThreads) {
    float v[8];
    load8<T>(xv + k * 8, v);
    acc.add8(v);
  }
  for (int64_t i = head + nv * 8 + tid; i < V; i += kXentThreads) acc.add(Elem<T>::load(x, i) * kLog2e);
  // wave64 merge, then the 4 waves through LDS
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(acc.m, off, kWave);
    const float s2 = __shfl_xor(acc.s, off, kWave);
    acc.merge(m2, s2);
  }
  __shared__ float sm[kXentThreads / kWave], ss[kXentThreads / kWave];
  const int wave = tid / kWave;
  if ((tid & (kWave - 1)) == 0) {
    sm[wave] = acc.m;
    ss[wave] = acc.s;
  }
  __syncthreads();
  if (tid == 0) {
    OnlineLse tot;
#pragma unroll
    for (int w = 0; w < kXentThreads / kWave; ++w) tot.merge(sm[w], ss[w]);
    const float lse = (tot.m + log2f(tot.s)) * kLn2;
    const int64_t t = target[row];
    float l;
    if (t == ignore_index) l = 0.f;
    else if (t >= 0 && t < V) l = lse - Elem<T>::load(x, t);
    else l = NAN;  // out-of-range class index: poison the loss instead of reading out of bounds
    lse_out[row] = lse;
    loss[row] = l;
  }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(kXentThreads) void xent_bwd_kernel(const T* __restrict__ logits, int64_t ld,
                                                                const int64_t* __restrict__ target,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ scale, int64_t V,
                                                                int64_t ignore_index, T* dlogits) {
  // no __restrict__ on dlogits: it may alias logits (in-place backward; every element is read and
  // then written by the same lane)
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  T* dx = dlogits + row * ld;
  const int tid = threadIdx.x;
  const int64_t t = target[row];
  const bool valid = t != ignore_index && t >= 0 && t < V;
  const float sc = valid ? *scale : 0.f;
  const float l2 = lse[row] * kLog2e;
  if (!VEC) {
    for (int64_t i = tid; i < V; i += kXentThreads) {
      float g = __builtin_amdgcn_exp2f(Elem<T>::load(x, i) * kLog2e - l2) * sc;
      if (i == t) g -= sc;
      Elem<T>::store(dx, i, g);
    }
    return;
  }
  const int64_t head = head_elems(x, V);
  if (tid < head) {
    float g = __builtin_amdgcn_exp2f(Elem<T>::load(x, tid) * kLog2e - l2) * sc;
    if (tid == t) g -= sc;
    Elem<T>::store(dx, tid, g);
  }
  const int64_t nv = (V - head) / 8;
  for (int64_t k = tid; k < nv; k += kXentThreads) {
    const int64_t base = head + k * 8;
    float v[8];
    load8<T>(x + base, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __builtin_amdgcn_exp2f(v[j] * kLog2e - l2) * sc;
    const int64_t d = t - base;
    if (d >= 0 && d < 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j == d) v[j] -= sc;
    }
    if (sizeof(T) == 2) store8_nt<T>(dx + base, v);
    else store8<T>(dx + base, v);
  }
  for (int64_t i = head + nv * 8 + tid; i < V; i += kXentThreads) {
    float g = __builtin_amdgcn_exp2f(Elem<T>::load(x, i) * kLog2e - l2) * sc;
    if (i == t) g -= sc;
    Elem<T>::store(dx, i, g);
  }
}

// ---- forward and backward in one pass (the LM-head + loss path: logits are dead after the loss) --
// One read and one in-place write of each row: the row is held in registers between the two (NV
// 16-B chunks per lane, 256 lanes: V <= 256·8·NV), so the separate forward read of the two-kernel
// path disappears.  dx = (softmax(x) - onehot(t)) * scale with scale = 1/n_valid (or 1) read from
// device memory; grad_out is folded into the LM-head GEMMs' small operands by the caller.
template <typename T>
__device__ __forceinline__ void unpack8(const u32x4& w, float (&v)[8]);
template <>
__device__ __forceinline__ void unpack8<bf16_t>(const u32x4& w, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}
template <>
__device__ __forceinline__ void unpack8<f16_t>(const u32x4& w, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = f16_to_f32((uint16_t)(w[j] & 0xffffu));
    v[2 * j + 1] = f16_to_f32((uint16_t)(w[j] >> 16));
  }
}

constexpr int kFusedChunks = 32;  // at most 256 lanes x 32 x 8 = 65,536 columns (instances: 8, 16, 25, 32)

template <typename T, int NV>
__global__ __launch_bounds__(kXentThreads) void xent_fused_kernel(T* logits, int64_t ld,
                                                                  const int64_t* __restrict__ target, int64_t V,
                                                                  int64_t ignore_index,
                                                                  const float* __restrict__ scale,
                                                                  float* __restrict__ loss,
                                                                  float* __restrict__ lse_out) {
  const int64_t row = blockIdx.x;
  T* x = logits + row * ld;
  const int tid = threadIdx.x;
  const int64_t t = target[row];
  const bool valid = t != ignore_index && t >= 0 && t < V;
  float xt = 0.f;
  if (tid == 0 && valid) xt = Elem<T>::load(x, t);
  const int64_t head = head_elems(x, V);
  T* xv = x + head;
  const int64_t nv = (V - head) / 8;
  const int64_t tail0 = head + nv * 8;
  // lanes 0..7 own the unaligned head elements, lanes 8..15 the tail (each < 8)
  int64_t is = -1;
  if (tid < head) is = tid;
  else if (tid >= 8 && tid < 16 && tid - 8 < V - tail0) is = tail0 + tid - 8;
  const float xs = is >= 0 ? Elem<T>::load(x, is) : 0.f;
  u32x4 r[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int64_t k = tid + (int64_t)c * kXentThreads;
    if (k < nv) r[c] = *reinterpret_cast<const u32x4*>(xv + k * 8);
  }
  OnlineLse acc;
  if (is >= 0) acc.add(xs * kLog2e);
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int64_t k = tid + (int64_t)c * kXentThreads;
    if (k < nv) {
      float v[8];
      unpack8<T>(r[c], v);
      acc.add8(v);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float m2 = __shfl_xor(acc.m, off, kWave);
    const float s2 = __shfl_xor(acc.s, off, kWave);
    acc.merge(m2, s2);
  }
  __shared__ float sm[kXentThreads / kWave], ss[kXentThreads / kWave];
  const int wave = tid / kWave;
  if ((tid & (kWave - 1)) == 0) {
    sm[wave] = acc.m;
    ss[wave] = acc.s;
  }
  __syncthreads();  // every read of the row (registers, xs, xt) happened before any write below
  // keep the row packed between the passes: without this the compiler holds 8 unpacked floats per
  // chunk (306 VGPRs at NV = 32) instead of re-unpacking (a shift and a mask per pair)
#pragma unroll
  for (int c = 0; c < NV; ++c) asm volatile("" : "+v"(r[c]));
  OnlineLse tot;
#pragma unroll
  for (int w = 0; w < kXentThreads / kWave; ++w) tot.merge(sm[w], ss[w]);
  const float lse = (tot.m + log2f(tot.s)) * kLn2;
  if (tid == 0) {
    lse_out[row] = lse;
    loss[row] = valid ? lse - xt : (t == ignore_index ? 0.f : NAN);
  }
  const float sc = valid ? *scale : 0.f;
  const float l2 = lse * kLog2e;
  if (is >= 0) {
    float g = __builtin_amdgcn_exp2f(xs * kLog2e - l2) * sc;
    if (is == t) g -= sc;
    Elem<T>::store(x, is, g);
  }
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int64_t k = tid + (int64_t)c * kXentThreads;
    if (k < nv) {
      float v[8];
      unpack8<T>(r[c], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __builtin_amdgcn_exp2f(v[j] * kLog2e - l2) * sc;
      const int64_t d = t - (head + k * 8);
      if (d >= 0 && d < 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j == d) v[j] -= sc;
      }
      store8_nt<T>(xv + k * 8, v);
    }
  }
}

static void check_logits(const at::Tensor& logits, const at::Tensor& target) {
  TORCH_CHECK(logits.is_cuda() && target.is_cuda(), "xent: GPU tensors expected");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "xent: logits must be [N, V] with unit column stride");
  TORCH_CHECK(target.dim() == 1 && target.scalar_type() == at::kLong && target.is_contiguous() &&
                  target.size(0) == logits.size(0),
              "xent: target must be a contiguous int64 [N]");
  TORCH_CHECK(logits.size(0) < (1LL << 31), "xent: too many rows");
}

std::tuple<at::Tensor, at::Tensor> xent_fwd_hip(const at::Tensor& logits, const at::Tensor& target,
                                                int64_t ignore_index) {
  check_logits(logits, target);
  const int64_t N = logits.size(0), V = logits.size(1);
  auto opts = logits.options().dtype(at::kFloat);
  at::Tensor loss = at::empty({N}, opts), lse = at::empty({N}, opts);
  if (N == 0) return {loss, lse};
  TORCH_CHECK(V > 0, "xent: empty vocabulary");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int64_t ld = logits.stride(0);
  switch (logits.scalar_type()) {
#define NBD_XF(ATY, T)                                                                                           \
  case ATY:                                                                                                      \
    hipLaunchKernelGGL((xent_fwd_kernel<T>), dim3((unsigned)N), dim3(kXentThreads), 0, st,                       \
                       static_cast<const T*>(logits.data_ptr()), ld, target.data_ptr<int64_t>(), V, ignore_index, \
                       loss.data_ptr<float>(), lse.data_ptr<float>());                                          \
    break;
    NBD_XF(at::kFloat, float)
    NBD_XF(at::kBFloat16, bf16_t)
    NBD_XF(at::kHalf, f16_t)
#undef NBD_XF
    default: TORCH_CHECK(false, "xent: unsupported logits dtype ", logits.scalar_type());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {loss, lse};
}

void xent_bwd_hip(const at::Tensor& logits, const at::Tensor& target, const at::Tensor& lse, const at::Tensor& scale,
                  int64_t ignore_index, const at::Tensor& dlogits) {
  check_logits(logits, target);
  const int64_t N = logits.size(0), V = logits.size(1);
  TORCH_CHECK(dlogits.is_cuda() && dlogits.sizes() == logits.sizes() && dlogits.strides() == logits.strides() &&
                  dlogits.scalar_type() == logits.scalar_type(),
              "xent_bwd: dlogits must match the logits' shape, strides and dtype");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == N,
              "xent_bwd: lse must be float32 [N]");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() == 1,
              "xent_bwd: scale must be a 1-element float32 GPU tensor");
  if (N == 0) return;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int64_t ld = logits.stride(0);
  // the vector path needs dlogits to share the logits' 16-B phase (same strides, so one check)
  const bool vec = (((uintptr_t)dlogits.data_ptr() - (uintptr_t)logits.data_ptr()) & 15u) == 0;
  switch (logits.scalar_type()) {
#define NBD_XB(ATY, T)                                                                                         \
  case ATY:                                                                                                    \
    if (vec)                                                                                                   \
      hipLaunchKernelGGL((xent_bwd_kernel<T, true>), dim3((unsigned)N), dim3(kXentThreads), 0, st,             \
                         static_cast<const T*>(logits.data_ptr()), ld, target.data_ptr<int64_t>(),            \
                         lse.data_ptr<float>(), scale.data_ptr<float>(), V, ignore_index,                     \
                         static_cast<T*>(dlogits.data_ptr()));                                                \
    else                                                                                                       \
      hipLaunchKernelGGL((xent_bwd_kernel<T, false>), dim3((unsigned)N), dim3(kXentThreads), 0, st,            \
                         static_cast<const T*>(logits.data_ptr()), ld, target.data_ptr<int64_t>(),            \
                         lse.data_ptr<float>(), scale.data_ptr<float>(), V, ignore_index,                     \
                         static_cast<T*>(dlogits.data_ptr()));                                                \
    break;
    NBD_XB(at::kFloat, float)
    NBD_XB(at::kBFloat16, bf16_t)
    NBD_XB(at::kHalf, f16_t)
#undef NBD_XB
    default: TORCH_CHECK(false, "xent: unsupported logits dtype ", logits.scalar_type());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

std::tuple<at::Tensor, at::Tensor> xent_fused_hip(const at::Tensor& logits, const at::Tensor& target,
                                                  int64_t ignore_index, const at::Tensor& scale) {
  check_logits(logits, target);
  const int64_t N = logits.size(0), V = logits.size(1);
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kHalf,
              "xent_fused: bf16 / fp16 logits expected");
  TORCH_CHECK(V > 0 && V <= (int64_t)kXentThreads * 8 * kFusedChunks + 14, "xent_fused: vocabulary too large");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() == 1,
              "xent_fused: scale must be a 1-element float32 GPU tensor");
  auto opts = logits.options().dtype(at::kFloat);
  at::Tensor loss = at::empty({N}, opts), lse = at::empty({N}, opts);
  if (N == 0) return {loss, lse};
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(logits.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int64_t ld = logits.stride(0);
  // registers per lane scale with the chunk count: use the smallest instance covering the row
  const int64_t need = (V + (int64_t)kXentThreads * 8 - 1) / ((int64_t)kXentThreads * 8);
  const bool bf = logits.scalar_type() == at::kBFloat16;
#define NBD_XFU(NV)                                                                                              \
  if (bf)                                                                                                        \
    hipLaunchKernelGGL((xent_fused_kernel<bf16_t, NV>), dim3((unsigned)N), dim3(kXentThreads), 0, st,           \
                       static_cast<bf16_t*>(logits.data_ptr()), ld, target.data_ptr<int64_t>(), V, ignore_index, \
                       scale.data_ptr<float>(), loss.data_ptr<float>(), lse.data_ptr<float>());                 \
  else                                                                                                           \
    hipLaunchKernelGGL((xent_fused_kernel<f16_t, NV>), dim3((unsigned)N), dim3(kXentThreads), 0, st,            \
                       static_cast<f16_t*>(logits.data_ptr()), ld, target.data_ptr<int64_t>(), V, ignore_index,  \
                       scale.data_ptr<float>(), loss.data_ptr<float>(), lse.data_ptr<float>());
  if (need <= 8) {
    NBD_XFU(8)
  } else if (need <= 16) {
    NBD_XFU(16)
  } else if (need <= 25) {
    NBD_XFU(25)
  } else {
    NBD_XFU(32)
  }
#undef NBD_XFU
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {loss, lse};
}

// The mean reduction's two scalars, one launch each instead of torch's compare / sum / cast /
// reciprocal and sum / multiply chains (six small kernels around the GPT-2 LM head, ≈ 35 µs per
// step: docs/FINDINGS.md §36).  One 1024-thread workgroup; fixed summation order (deterministic).
constexpr int kScalarThreads = 1024;

__device__ __forceinline__ float block_sum_1024(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < kScalarThreads / 64; ++i) t += red[i];
  return t;  // (valid in thread 0)
}

// scale[0] = 1 / #(target != ignore_index)  (+inf when every row is ignored: the loss is then nan, as torch)
__global__ __launch_bounds__(kScalarThreads) void xent_mean_scale_kernel(const int64_t* __restrict__ target, int64_t n,
                                                                         int64_t ignore_index, float* __restrict__ scale) {
  __shared__ float red[kScalarThreads / 64];
  float c = 0.f;  // exact: counts < 2^24
  for (int64_t i = threadIdx.x; i < n; i += kScalarThreads) c += target[i] != ignore_index ? 1.f : 0.f;
  const float t = block_sum_1024(c, red);
  if (threadIdx.x == 0) scale[0] = 1.f / t;
}

// loss = Σ rows · scale[0]
__global__ __launch_bounds__(kScalarThreads) void xent_loss_total_kernel(const float* __restrict__ rows, int64_t n,
                                                                         const float* __restrict__ scale,
                                                                         float* __restrict__ out) {
  __shared__ float red[kScalarThreads / 64];
  float c = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += kScalarThreads) c += rows[i];
  const float t = block_sum_1024(c, red);
  if (threadIdx.x == 0) out[0] = t * scale[0];
}

at::Tensor xent_mean_scale_hip(const at::Tensor& target, int64_t ignore_index) {
  TORCH_CHECK(target.is_cuda() && target.scalar_type() == at::kLong && target.is_contiguous(),
              "xent_mean_scale: contiguous int64 GPU targets expected");
  at::Tensor scale = at::empty({1}, target.options().dtype(at::kFloat));
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(target.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  hipLaunchKernelGGL(xent_mean_scale_kernel, dim3(1), dim3(kScalarThreads), 0, st, target.data_ptr<int64_t>(),
                     target.numel(), ignore_index, scale.data_ptr<float>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return scale;
}

at::Tensor xent_loss_total_hip(const at::Tensor& rows, const at::Tensor& scale) {
  TORCH_CHECK(rows.is_cuda() && rows.scalar_type() == at::kFloat && rows.is_contiguous(),
              "xent_loss_total: contiguous float32 GPU rows expected");
  TORCH_CHECK(scale.is_cuda() && scale.scalar_type() == at::kFloat && scale.numel() == 1,
              "xent_loss_total: scale must be a 1-element float32 GPU tensor");
  at::Tensor out = at::empty({}, rows.options());
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(rows.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  hipLaunchKernelGGL(xent_loss_total_kernel, dim3(1), dim3(kScalarThreads), 0, st, rows.data_ptr<float>(), rows.numel(),
                     scale.data_ptr<float>(), out.data_ptr<float>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

// The LM head's backward scales by the incoming gradient g (a device fp32 scalar, 1 after
// loss.backward()): dh *= g in place and hg = h·g, one launch for both (torch ran a cast of g and
// two elementwise kernels, or two mixed-dtype ones at ≈ 25 µs each).  8 elements per thread.
template <typename T>
__global__ __launch_bounds__(256) void scale_pair_kernel(T* __restrict__ a, const T* __restrict__ b, T* __restrict__ bo,
                                                        const float* __restrict__ g, int64_t na8, int64_t nb8) {
  const float s = g[0];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float x[8];
  if (i < na8) {
    load8<T>(a + i * 8, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] *= s;
    store8<T>(a + i * 8, x);
  } else if (i < na8 + nb8) {
    const int64_t j = i - na8;
    load8<T>(b + j * 8, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] *= s;
    store8<T>(bo + j * 8, x);
  }
}

// a *= g (in place), returns b·g
at::Tensor scale_pair_hip(const at::Tensor& a, const at::Tensor& b, const at::Tensor& g) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.is_contiguous() && b.is_contiguous() && a.scalar_type() == b.scalar_type() &&
                  (a.scalar_type() == at::kBFloat16 || a.scalar_type() == at::kHalf) && a.numel() % 8 == 0 &&
                  b.numel() % 8 == 0,
              "scale_pair: contiguous bf16/fp16 GPU tensors with numel % 8 == 0");
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kFloat && g.numel() == 1, "scale_pair: g must be one float32 on the GPU");
  for (const at::Tensor* t : {&a, &b})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "scale_pair: 16-byte aligned tensors");
  at::Tensor out = at::empty_like(b);
  const int64_t na8 = a.numel() / 8, nb8 = b.numel() / 8, blocks = (na8 + nb8 + 255) / 256;
  if (blocks == 0) return out;
  TORCH_CHECK(blocks < (1LL << 31), "scale_pair: too large");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  if (a.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(scale_pair_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, st,
                       static_cast<bf16_t*>(a.data_ptr()), static_cast<const bf16_t*>(b.data_ptr()),
                       static_cast<bf16_t*>(out.data_ptr()), g.data_ptr<float>(), na8, nb8);
  else
    hipLaunchKernelGGL(scale_pair_kernel<f16_t>, dim3((unsigned)blocks), dim3(256), 0, st,
                       static_cast<f16_t*>(a.data_ptr()), static_cast<const f16_t*>(b.data_ptr()),
                       static_cast<f16_t*>(out.data_ptr()), g.data_ptr<float>(), na8, nb8);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("xent_fwd", &nbd::xent_fwd_hip);
  m.impl("xent_bwd", &nbd::xent_bwd_hip);
  m.impl("xent_fused", &nbd::xent_fused_hip);
  m.impl("xent_mean_scale", &nbd::xent_mean_scale_hip);
  m.impl("xent_loss_total", &nbd::xent_loss_total_hip);
  m.impl("scale_pair_", &nbd::scale_pair_hip);
}
