// tiny.hip — Linear layers with a tiny output dimension (classifier heads: SmolLM2's `score`,
// 576 -> 2 labels on 16 pooled rows), forward and backward, bf16 in / fp32 accumulate.
//
// Such a product is a few dot products: y[16, 2] = x[16, 576]·Wᵀ is 32 dots of 576.  A tiled
// MFMA GEMM (or the library's, which ran three Cijk launches per notebook step for it: 7-8 µs
// each, profiles/notebook_graph_prof_r5final2.md) pads it to a whole 64-wide tile and a K-loop;
// here it is one wave per output and one launch for the three backward products:
//   forward   y[m, n]  = Σ_k x[m, k]·W[n, k] (+ b[n])       one wave per (m, n), lanes over K
//   backward  dx[m, k] = Σ_n dy[m, n]·W[n, k]                one thread per (m, 8 k)
//             dW[n, k] = Σ_m dy[m, n]·x[m, k]                one thread per (n, 8 k)
//             db[n]    = Σ_m dy[m, n]                        one thread per n
// Every sum is fp32 in a fixed order (deterministic); outputs rounded once to bf16.  Loads are
// 16 B per lane (8 bf16).  For N ≤ 64 (and M·K, N·K ≤ 2^31); large M works but dW then loops
// over every row in one thread (ops/tiny.py routes only M ≤ 4096 here).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include "nbd_common.h"

namespace nbd {
namespace tiny {

constexpr int NT = 256;

// one wave per output element: lanes stride K in 8-element chunks
__global__ __launch_bounds__(NT) void fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                 const uint16_t* __restrict__ bias, uint16_t* __restrict__ y, int M,
                                                 int N, int K) {
  const int wave = (int)(blockIdx.x * (NT / kWave) + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  if (wave >= M * N) return;  // (wave-uniform: no wave is split by the exit)
  const int m = wave / N, n = wave % N;
  const uint16_t* xr = x + (int64_t)m * K;
  const uint16_t* wr = w + (int64_t)n * K;
  float acc = 0.f;
  for (int k = lane * 8; k < K; k += 64 * 8) {
    float a[8], b[8];
    load8<bf16_t>(reinterpret_cast<const bf16_t*>(xr + k), a);
    load8<bf16_t>(reinterpret_cast<const bf16_t*>(wr + k), b);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc = fmaf(a[e], b[e], acc);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) {
    if (bias != nullptr) acc += bf16_to_f32(bias[n]);
    y[(int64_t)m * N + n] = f32_to_bf16(acc);
  }
}

// blocks [0, bx) dx, [bx, bx + bw) dW, the last one db (when db != nullptr)
__global__ __launch_bounds__(NT) void bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                 const uint16_t* __restrict__ w, uint16_t* __restrict__ dx,
                                                 uint16_t* __restrict__ dw, uint16_t* __restrict__ db, int M, int N,
                                                 int K, int bx, int bw) {
  const int K8 = K / 8;
  const int b = (int)blockIdx.x;
  if (b < bx) {  // dx[m, 8c..8c+8] = Σ_n dy[m, n]·W[n, 8c..]
    const int64_t i = (int64_t)b * NT + threadIdx.x;
    if (i >= (int64_t)M * K8) return;
    const int m = (int)(i / K8), c = (int)(i % K8);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int n = 0; n < N; ++n) {
      const float g = bf16_to_f32(dy[(int64_t)m * N + n]);
      float v[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(w + (int64_t)n * K + 8 * c), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(g, v[e], acc[e]);
    }
    store8<bf16_t>(reinterpret_cast<bf16_t*>(dx + (int64_t)m * K + 8 * c), acc);
  } else if (b < bx + bw) {  // dW[n, 8c..] = Σ_m dy[m, n]·x[m, 8c..]
    const int64_t i = (int64_t)(b - bx) * NT + threadIdx.x;
    if (i >= (int64_t)N * K8) return;
    const int n = (int)(i / K8), c = (int)(i % K8);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int m = 0; m < M; ++m) {
      const float g = bf16_to_f32(dy[(int64_t)m * N + n]);
      float v[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(x + (int64_t)m * K + 8 * c), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(g, v[e], acc[e]);
    }
    store8<bf16_t>(reinterpret_cast<bf16_t*>(dw + (int64_t)n * K + 8 * c), acc);
  } else {  // db[n] = Σ_m dy[m, n]
    const int n = threadIdx.x;
    if (db == nullptr || n >= N) return;
    float acc = 0.f;
    for (int m = 0; m < M; ++m) acc += bf16_to_f32(dy[(int64_t)m * N + n]);
    db[n] = f32_to_bf16(acc);
  }
}

static void check_common(const at::Tensor& x, const at::Tensor& w) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.dim() == 2 && w.dim() == 2, "nbd::linear_tiny: 2-D GPU operands");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "nbd::linear_tiny: bf16 operands");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "nbd::linear_tiny: contiguous operands");
  TORCH_CHECK(x.size(1) == w.size(1) && x.size(1) % 8 == 0 && x.size(1) > 0, "nbd::linear_tiny: K mismatch or K % 8 != 0");
  TORCH_CHECK(w.size(0) >= 1 && w.size(0) <= 64, "nbd::linear_tiny: N must be in [1, 64]");
  TORCH_CHECK(x.size(0) * x.size(1) < (1LL << 31) && x.size(0) * w.size(0) < (1LL << 31), "nbd::linear_tiny: too large");
  for (const at::Tensor* t : {&x, &w})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "nbd::linear_tiny: 16-byte aligned operands");
}

at::Tensor linear_tiny_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias) {
  check_common(x, w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  if (bias)
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N,
                "nbd::linear_tiny: bias [N] bf16");
  at::Tensor y = at::empty({M, N}, x.options());
  if (M == 0) return y;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int waves = M * N, blocks = (waves + NT / kWave - 1) / (NT / kWave);
  hipLaunchKernelGGL(fwd_kernel, dim3(blocks), dim3(NT), 0, st, static_cast<const uint16_t*>(x.data_ptr()),
                     static_cast<const uint16_t*>(w.data_ptr()),
                     bias ? static_cast<const uint16_t*>(bias->data_ptr()) : nullptr,
                     static_cast<uint16_t*>(y.data_ptr()), M, N, K);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return y;
}

// (dx, dW, db) for the products asked for
std::tuple<at::Tensor, at::Tensor, at::Tensor> linear_tiny_bwd(const at::Tensor& dy, const at::Tensor& x,
                                                               const at::Tensor& w, bool want_dx, bool want_dw,
                                                               bool want_db) {
  check_common(x, w);
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.is_contiguous() && dy.size(0) == M &&
                  dy.size(1) == N,
              "nbd::linear_tiny: dy [M, N] bf16 contiguous");
  // (an output not asked for comes back as an empty [0] tensor)
  at::Tensor dx = at::empty({want_dx ? M : 0, K}, x.options());
  at::Tensor dw = at::empty({want_dw ? N : 0, K}, w.options());
  at::Tensor db = at::empty({want_db ? N : 0}, w.options());
  const int64_t K8 = K / 8;
  const int bx = want_dx ? (int)(((int64_t)M * K8 + NT - 1) / NT) : 0;
  const int bw = want_dw ? (int)(((int64_t)N * K8 + NT - 1) / NT) : 0;
  const int blocks = bx + bw + (want_db ? 1 : 0);
  if (blocks == 0 || M == 0) {
    if (want_dw) dw.zero_();
    if (want_db) db.zero_();
    return {dx, dw, db};
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  hipLaunchKernelGGL(bwd_kernel, dim3(blocks), dim3(NT), 0, st, static_cast<const uint16_t*>(dy.data_ptr()),
                     static_cast<const uint16_t*>(x.data_ptr()), static_cast<const uint16_t*>(w.data_ptr()),
                     want_dx ? static_cast<uint16_t*>(dx.data_ptr()) : nullptr,
                     want_dw ? static_cast<uint16_t*>(dw.data_ptr()) : nullptr,
                     want_db ? static_cast<uint16_t*>(db.data_ptr()) : nullptr, M, N, K, bx, bw);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {dx, dw, db};
}

}  // namespace tiny
}  // namespace nbd

TORCH_LIBRARY_FRAGMENT(nbd, m) {
  m.def("linear_tiny(Tensor x, Tensor w, Tensor? bias) -> Tensor");
  m.def("linear_tiny_bwd(Tensor dy, Tensor x, Tensor w, bool want_dx, bool want_dw, bool want_db) -> "
        "(Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("linear_tiny", &nbd::tiny::linear_tiny_fwd);
  m.impl("linear_tiny_bwd", &nbd::tiny::linear_tiny_bwd);
}
