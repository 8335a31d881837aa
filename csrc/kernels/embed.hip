// embed.hip — embedding backward (dense weight gradient) by counting sort, gfx950.
//
// torch's embedding backward sorts and uniques the token ids with rocprim once there are more
// than 3072 of them (GPT-2 small: 8192 per step); rocprim's temporary / virtual-shared-memory
// buffers are not taken from the caching allocator, so a HIP graph that captured them replays
// into freed memory (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in rocprim::partition_kernel,
// benchmarks/ddp_compare.py flatgraph).  This version only uses caching-allocator memory and
// fixed launch shapes, so it captures and replays, and it is cheaper:
//
//   count   counts[v] = #tokens with id v                (int atomics)
//   scan    offsets = exclusive_scan(counts), one 1024-thread workgroup (two passes over V)
//   place   slot = offsets[v] + atomicAdd(cursor[v]) ; order[slot] = token position
//   rows    one wave per vocabulary row: Σ dY[order[offsets[v] .. offsets[v+1])] in fp32, written
//           once in the weight's dtype (zeros for rows no token touched) — the gradient is written
//           exactly once, no zero-fill pass and no float atomics.
// Summation order inside a row follows the atomic slot order (not bitwise run-to-run stable; DDP
// ranks still agree after the all-reduce).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <type_traits>

#include "nbd_common.h"

namespace nbd {
namespace embed {

constexpr int NT = 256;
constexpr int kScanT = 1024;

__global__ __launch_bounds__(NT) void count_kernel(const int64_t* __restrict__ idx, int64_t n, int V,
                                                   int* __restrict__ counts, int* __restrict__ bad) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t v = idx[i];
    if (v >= 0 && v < V) atomicAdd(&counts[v], 1);
    else atomicOr(bad, 1);  // out-of-range id: flagged, never written out of bounds
  }
}

// exclusive scan of counts[0..V) into offsets[0..V]; one workgroup
__global__ __launch_bounds__(kScanT) void scan_kernel(const int* __restrict__ counts, int V,
                                                      int* __restrict__ offsets) {
  __shared__ int part[kScanT];
  const int t = threadIdx.x;
  const int per = (V + kScanT - 1) / kScanT;
  const int b = t * per, e = min(V, b + per);
  int s = 0;
  for (int i = b; i < e; ++i) s += counts[i];
  part[t] = s;
  __syncthreads();
  // Hillis-Steele inclusive scan over the 1024 partial sums
  for (int off = 1; off < kScanT; off <<= 1) {
    const int add = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += add;
    __syncthreads();
  }
  int run = part[t] - s;  // exclusive prefix of this thread's range
  for (int i = b; i < e; ++i) {
    offsets[i] = run;
    run += counts[i];
  }
  if (t == kScanT - 1) offsets[V] = part[t];
}

__global__ __launch_bounds__(NT) void place_kernel(const int64_t* __restrict__ idx, int64_t n, int V,
                                                   const int* __restrict__ offsets, int* __restrict__ cursor,
                                                   int* __restrict__ order) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
    const int64_t v = idx[i];
    if (v >= 0 && v < V) order[offsets[v] + atomicAdd(&cursor[v], 1)] = (int)i;
  }
}

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float (&v)[4]) {
  if constexpr (std::is_same<T, float>::value) {
    const float4 w = *reinterpret_cast<const float4*>(p);
    v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
  } else {
    const uint2 w = *reinterpret_cast<const uint2*>(p);
    const uint16_t h[4] = {(uint16_t)(w.x & 0xffffu), (uint16_t)(w.x >> 16), (uint16_t)(w.y & 0xffffu),
                           (uint16_t)(w.y >> 16)};
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = std::is_same<T, bf16_t>::value ? bf16_to_f32(h[e]) : f16_to_f32(h[e]);
  }
}
template <typename T>
__device__ __forceinline__ void st4(T* p, const float (&v)[4]) {
  if constexpr (std::is_same<T, float>::value) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else {
    uint16_t h[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) h[e] = std::is_same<T, bf16_t>::value ? f32_to_bf16(v[e]) : f32_to_f16(v[e]);
    *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16),
                                              (uint32_t)h[2] | ((uint32_t)h[3] << 16));
  }
}

// one wave per vocabulary row; a lane owns 4-column chunks c = 4·lane + 256·k, k < NCH
template <typename T, int NCH>
__global__ __launch_bounds__(NT) void rows_kernel(const T* __restrict__ dy, int C, const int* __restrict__ offsets,
                                                  const int* __restrict__ order, int V, T* __restrict__ grad) {
  const int lane = threadIdx.x & 63;
  const int64_t v = (int64_t)blockIdx.x * (NT / kWave) + (threadIdx.x >> 6);
  if (v >= V) return;
  float acc[NCH][4];
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[k][e] = 0.f;
  const int b = offsets[v], e = offsets[v + 1];
  for (int j = b; j < e; ++j) {
    const int64_t row = order[j];
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = 4 * lane + 256 * k;
      if (c < C) {
        float x[4];
        ld4<T>(dy + row * C + c, x);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[k][q] += x[q];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) st4<T>(grad + v * C + c, acc[k]);
  }
}

template <typename F>
static void dispatch_nch(int64_t C, F&& f) {
  const int64_t n = (C + 255) / 256;
  if (n <= 1) f(std::integral_constant<int, 1>{});
  else if (n == 2) f(std::integral_constant<int, 2>{});
  else if (n == 3) f(std::integral_constant<int, 3>{});
  else if (n == 4) f(std::integral_constant<int, 4>{});
  else if (n <= 6) f(std::integral_constant<int, 6>{});
  else if (n <= 8) f(std::integral_constant<int, 8>{});
  else f(std::integral_constant<int, 16>{});
}

// grad_weight [V, C] (dtype of dy) from dy [N, C] and int64 ids [N]
at::Tensor embedding_bwd_hip(const at::Tensor& dy, const at::Tensor& idx, int64_t V) {
  TORCH_CHECK(dy.is_cuda() && idx.is_cuda(), "embedding_bwd: GPU tensors expected");
  TORCH_CHECK(dy.dim() == 2 && dy.is_contiguous(), "embedding_bwd: dy must be a contiguous [N, C]");
  TORCH_CHECK(idx.dim() == 1 && idx.is_contiguous() && idx.scalar_type() == at::kLong && idx.size(0) == dy.size(0),
              "embedding_bwd: ids must be a contiguous int64 [N]");
  const int64_t N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(C % 4 == 0 && C <= 4096, "embedding_bwd: C must be a multiple of 4 and <= 4096");
  TORCH_CHECK(V > 0 && V < (1LL << 31) && N < (1LL << 31), "embedding_bwd: sizes out of range");
  TORCH_CHECK(((uintptr_t)dy.data_ptr() & 15) == 0, "embedding_bwd: dy must be 16-B aligned");
  at::Tensor grad = at::empty({V, C}, dy.options());
  auto io = idx.options().dtype(at::kInt);
  at::Tensor counts = at::zeros({V + 1}, io);  // [V] counts, [V] = out-of-range flag
  at::Tensor cursor = at::zeros({V}, io);
  at::Tensor offsets = at::empty({V + 1}, io);
  at::Tensor order = at::empty({std::max<int64_t>(N, 1)}, io);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int blocks = (int)std::min<int64_t>((N + NT - 1) / NT + 1, 1024);
  int* cnt = counts.data_ptr<int>();
  hipLaunchKernelGGL(count_kernel, dim3(blocks), dim3(NT), 0, st, idx.data_ptr<int64_t>(), N, (int)V, cnt, cnt + V);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(kScanT), 0, st, cnt, (int)V, offsets.data_ptr<int>());
  hipLaunchKernelGGL(place_kernel, dim3(blocks), dim3(NT), 0, st, idx.data_ptr<int64_t>(), N, (int)V,
                     offsets.data_ptr<int>(), cursor.data_ptr<int>(), order.data_ptr<int>());
  const dim3 rgrid((unsigned)((V + 3) / 4));
  dispatch_nch(C, [&](auto nch) {
    constexpr int K = decltype(nch)::value;
    switch (dy.scalar_type()) {
      case at::kFloat:
        hipLaunchKernelGGL((rows_kernel<float, K>), rgrid, dim3(NT), 0, st, dy.data_ptr<float>(), (int)C,
                           offsets.data_ptr<int>(), order.data_ptr<int>(), (int)V, grad.data_ptr<float>());
        break;
      case at::kBFloat16:
        hipLaunchKernelGGL((rows_kernel<bf16_t, K>), rgrid, dim3(NT), 0, st,
                           static_cast<const bf16_t*>(dy.data_ptr()), (int)C, offsets.data_ptr<int>(),
                           order.data_ptr<int>(), (int)V, static_cast<bf16_t*>(grad.data_ptr()));
        break;
      case at::kHalf:
        hipLaunchKernelGGL((rows_kernel<f16_t, K>), rgrid, dim3(NT), 0, st, static_cast<const f16_t*>(dy.data_ptr()),
                           (int)C, offsets.data_ptr<int>(), order.data_ptr<int>(), (int)V,
                           static_cast<f16_t*>(grad.data_ptr()));
        break;
      default: TORCH_CHECK(false, "embedding_bwd: unsupported dtype ", dy.scalar_type());
    }
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return grad;
}

}  // namespace embed
}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) { m.impl("embedding_bwd", &nbd::embed::embedding_bwd_hip); }
