// act.hip — rotary position embedding (in place on a packed QKV projection) and SwiGLU, gfx950.
//
// Llama-family blocks (SmolLM2, the reference notebook's model) spend a small-batch step in
// dozens of tiny eager kernels per layer: rotate_half + cos/sin multiplies for q and k, SiLU,
// the gate·up product and their backward.  These kernels do each in one pass.
//
//   rope_      rows of a contiguous [B, T, H_total·D] projection; heads [0, n_rot) are rotated
//              (q heads then k heads), v heads untouched.  HF convention (rotate_half, not
//              interleaved): x'[i] = x[i]·cos − x[i+D/2]·sin, x'[i+D/2] = x[i+D/2]·cos + x[i]·sin,
//              cos/sin = [T, D/2] fp32 tables; `inverse` rotates by −θ (the backward of the
//              forward rotation is its transpose).  A lane owns 4 rotation pairs (two 8-B loads).
//   swiglu     act = silu(g)·u on a fused [N, 2I] gate|up projection; backward writes
//              d[g|u] = [dact·u·σ(g)(1 + g(1−σ(g))) | dact·silu(g)] into one [N, 2I] buffer, so
//              the fused projection's backward is a single GEMM pair.  16-B vectors.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "nbd_common.h"

namespace nbd {
namespace act {

constexpr int NT = 256;

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float (&v)[4]) {
  const uint2 w = *reinterpret_cast<const uint2*>(p);
  const uint16_t h[4] = {(uint16_t)(w.x & 0xffffu), (uint16_t)(w.x >> 16), (uint16_t)(w.y & 0xffffu),
                         (uint16_t)(w.y >> 16)};
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = Elem<T>::load(reinterpret_cast<const T*>(h), e);
}
template <typename T>
__device__ __forceinline__ void st4(T* p, const float (&v)[4]) {
  uint16_t h[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) Elem<T>::store(reinterpret_cast<T*>(h), e, v[e]);
  *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
}

// grid-stride over units = rows · n_rot · (D/8): one unit = 4 pairs of one head of one token
template <typename T>
__global__ __launch_bounds__(NT) void rope_kernel(T* __restrict__ x, int64_t rows, int T_, int width, int n_rot,
                                                  int D, const float* __restrict__ cos_t,
                                                  const float* __restrict__ sin_t, float sgn) {
  const int half = D / 2, upr = half / 4;  // units per head
  const int64_t units = rows * n_rot * upr;
  for (int64_t u = (int64_t)blockIdx.x * NT + threadIdx.x; u < units; u += (int64_t)gridDim.x * NT) {
    const int j = (int)(u % upr);
    const int64_t rh = u / upr;
    const int h = (int)(rh % n_rot);
    const int64_t row = rh / n_rot;
    const int t = (int)(row % T_);
    T* p = x + row * width + (int64_t)h * D + 4 * j;
    float a[4], b[4], c[4], s[4];
    ld4<T>(p, a);
    ld4<T>(p + half, b);
    const float4 cv = *reinterpret_cast<const float4*>(cos_t + (int64_t)t * half + 4 * j);
    const float4 sv = *reinterpret_cast<const float4*>(sin_t + (int64_t)t * half + 4 * j);
    c[0] = cv.x; c[1] = cv.y; c[2] = cv.z; c[3] = cv.w;
    s[0] = sgn * sv.x; s[1] = sgn * sv.y; s[2] = sgn * sv.z; s[3] = sgn * sv.w;
    float oa[4], ob[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      oa[e] = a[e] * c[e] - b[e] * s[e];
      ob[e] = b[e] * c[e] + a[e] * s[e];
    }
    st4<T>(p, oa);
    st4<T>(p + half, ob);
  }
}

__device__ __forceinline__ float sigm(float g) { return 1.f / (1.f + __expf(-g)); }

template <typename T>
__global__ __launch_bounds__(NT) void swiglu_fwd_kernel(const T* __restrict__ gu, int64_t rows, int I,
                                                        T* __restrict__ out) {
  const int per = I / 8;
  const int64_t units = rows * per;
  for (int64_t u = (int64_t)blockIdx.x * NT + threadIdx.x; u < units; u += (int64_t)gridDim.x * NT) {
    const int64_t r = u / per;
    const int c = (int)(u % per) * 8;
    float g[8], v[8], o[8];
    load8<T>(gu + r * 2 * I + c, g);
    load8<T>(gu + r * 2 * I + I + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = g[e] * sigm(g[e]) * v[e];
    store8<T>(out + r * I + c, o);
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void swiglu_bwd_kernel(const T* __restrict__ gu, const T* __restrict__ dact,
                                                        int64_t rows, int I, T* __restrict__ dgu) {
  const int per = I / 8;
  const int64_t units = rows * per;
  for (int64_t u = (int64_t)blockIdx.x * NT + threadIdx.x; u < units; u += (int64_t)gridDim.x * NT) {
    const int64_t r = u / per;
    const int c = (int)(u % per) * 8;
    float g[8], v[8], d[8], dg[8], dv[8];
    load8<T>(gu + r * 2 * I + c, g);
    load8<T>(gu + r * 2 * I + I + c, v);
    load8<T>(dact + r * I + c, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float s = sigm(g[e]);
      dv[e] = d[e] * g[e] * s;
      dg[e] = d[e] * v[e] * s * (1.f + g[e] * (1.f - s));
    }
    store8<T>(dgu + r * 2 * I + c, dg);
    store8<T>(dgu + r * 2 * I + I + c, dv);
  }
}

static int grid_for(int64_t units) { return (int)std::max<int64_t>(1, std::min<int64_t>((units + NT - 1) / NT, 4096)); }

void rope_hip(const at::Tensor& x, const at::Tensor& cos_t, const at::Tensor& sin_t, int64_t n_rot, int64_t D,
              bool inverse) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 3, "rope_: x must be a contiguous [B, T, W] GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kHalf, "rope_: bf16/f16 only");
  TORCH_CHECK(D % 8 == 0 && D > 0 && n_rot > 0 && n_rot * D <= x.size(2), "rope_: bad head layout");
  const int64_t T = x.size(1);
  TORCH_CHECK(cos_t.is_cuda() && sin_t.is_cuda() && cos_t.scalar_type() == at::kFloat && cos_t.is_contiguous() &&
                  sin_t.is_contiguous() && cos_t.size(0) >= T && cos_t.size(1) == D / 2 && sin_t.sizes() == cos_t.sizes(),
              "rope_: cos/sin must be float32 [>= T, D/2]");
  TORCH_CHECK(((uintptr_t)x.data_ptr() & 7) == 0 && (x.size(2) % 4) == 0, "rope_: alignment");
  const int64_t rows = x.size(0) * T;
  const int64_t units = rows * n_rot * (D / 8);
  if (units == 0) return;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const float sgn = inverse ? -1.f : 1.f;
  if (x.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL((rope_kernel<bf16_t>), dim3(grid_for(units)), dim3(NT), 0, st,
                       static_cast<bf16_t*>(x.data_ptr()), rows, (int)T, (int)x.size(2), (int)n_rot, (int)D,
                       cos_t.data_ptr<float>(), sin_t.data_ptr<float>(), sgn);
  else
    hipLaunchKernelGGL((rope_kernel<f16_t>), dim3(grid_for(units)), dim3(NT), 0, st, static_cast<f16_t*>(x.data_ptr()),
                       rows, (int)T, (int)x.size(2), (int)n_rot, (int)D, cos_t.data_ptr<float>(),
                       sin_t.data_ptr<float>(), sgn);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

static void check_gu(const at::Tensor& gu) {
  TORCH_CHECK(gu.is_cuda() && gu.is_contiguous() && gu.size(-1) % 16 == 0, "swiglu: gu must be contiguous [..., 2I], I % 8 == 0");
  TORCH_CHECK(gu.scalar_type() == at::kBFloat16 || gu.scalar_type() == at::kHalf || gu.scalar_type() == at::kFloat,
              "swiglu: unsupported dtype");
  TORCH_CHECK(((uintptr_t)gu.data_ptr() & 15) == 0, "swiglu: 16-B alignment");
}

at::Tensor swiglu_fwd_hip(const at::Tensor& gu) {
  check_gu(gu);
  const int64_t I = gu.size(-1) / 2, rows = gu.numel() / (2 * I);
  auto sizes = gu.sizes().vec();
  sizes.back() = I;
  at::Tensor out = at::empty(sizes, gu.options());
  const int64_t units = rows * (I / 8);
  if (units == 0) return out;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(gu.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  switch (gu.scalar_type()) {
    case at::kBFloat16:
      hipLaunchKernelGGL((swiglu_fwd_kernel<bf16_t>), dim3(grid_for(units)), dim3(NT), 0, st,
                         static_cast<const bf16_t*>(gu.data_ptr()), rows, (int)I, static_cast<bf16_t*>(out.data_ptr()));
      break;
    case at::kHalf:
      hipLaunchKernelGGL((swiglu_fwd_kernel<f16_t>), dim3(grid_for(units)), dim3(NT), 0, st,
                         static_cast<const f16_t*>(gu.data_ptr()), rows, (int)I, static_cast<f16_t*>(out.data_ptr()));
      break;
    default:
      hipLaunchKernelGGL((swiglu_fwd_kernel<float>), dim3(grid_for(units)), dim3(NT), 0, st, gu.data_ptr<float>(),
                         rows, (int)I, out.data_ptr<float>());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

at::Tensor swiglu_bwd_hip(const at::Tensor& gu, const at::Tensor& dact) {
  check_gu(gu);
  const int64_t I = gu.size(-1) / 2, rows = gu.numel() / (2 * I);
  TORCH_CHECK(dact.is_cuda() && dact.is_contiguous() && dact.scalar_type() == gu.scalar_type() &&
                  dact.numel() == rows * I && ((uintptr_t)dact.data_ptr() & 15) == 0,
              "swiglu_bwd: dact must be a contiguous [..., I] of the same dtype");
  at::Tensor dgu = at::empty_like(gu);
  const int64_t units = rows * (I / 8);
  if (units == 0) return dgu;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(gu.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  switch (gu.scalar_type()) {
    case at::kBFloat16:
      hipLaunchKernelGGL((swiglu_bwd_kernel<bf16_t>), dim3(grid_for(units)), dim3(NT), 0, st,
                         static_cast<const bf16_t*>(gu.data_ptr()), static_cast<const bf16_t*>(dact.data_ptr()), rows,
                         (int)I, static_cast<bf16_t*>(dgu.data_ptr()));
      break;
    case at::kHalf:
      hipLaunchKernelGGL((swiglu_bwd_kernel<f16_t>), dim3(grid_for(units)), dim3(NT), 0, st,
                         static_cast<const f16_t*>(gu.data_ptr()), static_cast<const f16_t*>(dact.data_ptr()), rows,
                         (int)I, static_cast<f16_t*>(dgu.data_ptr()));
      break;
    default:
      hipLaunchKernelGGL((swiglu_bwd_kernel<float>), dim3(grid_for(units)), dim3(NT), 0, st, gu.data_ptr<float>(),
                         dact.data_ptr<float>(), rows, (int)I, dgu.data_ptr<float>());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return dgu;
}

}  // namespace act
}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("rope_", &nbd::act::rope_hip);
  m.impl("swiglu_fwd", &nbd::act::swiglu_fwd_hip);
  m.impl("swiglu_bwd", &nbd::act::swiglu_bwd_hip);
}
