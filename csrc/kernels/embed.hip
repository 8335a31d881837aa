// embed.hip — embedding backward (dense weight gradient) by counting sort, gfx950.
//
// torch's embedding backward sorts and uniques the token ids with rocprim once there are more
// than 3072 of them (GPT-2 small: 8192 per step); rocprim's temporary / virtual-shared-memory
// buffers are not taken from the caching allocator, so a HIP graph that captured them replays
// into freed memory (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in rocprim::partition_kernel,
// benchmarks/ddp_compare.py flatgraph).  This version only uses caching-allocator memory and
// fixed launch shapes, so it captures and replays, and it is cheaper:
//
//   count    counts[v] = #tokens with id v  (int atomics; the lanes of a wave that share its
//            first id — a padding run — count with one)
//   scan     offsets = exclusive_scan(counts): per-1024 block scans + block sums, then each block
//            adds the sum of the blocks before it (two fully parallel launches)
//   place    slot = offsets[v] + atomicAdd(cursor[v]) ; order[slot] = token position (same
//            one-atomic-per-wave rule for the first id, ranked by lane)
//   partial  one wave per 16 consecutive sorted slots: runs of equal ids are summed in fp32 and
//            stored into scratch row max(offsets[v], first slot of the wave) of a [N, C] scratch
//            — a frequent id (padding!) is spread over many waves instead of one wave looping
//            over hundreds of occurrences (550 µs per step on the notebook's right-padded
//            batches), and no float atomics: every scratch row has one writer, none is zeroed
//   rows     one wave per vocabulary row: the run's rows (one per wave it reached) summed and
//            cast into the gradient (or zeros) — written exactly once, no separate zero-fill.
// The order of equal ids inside a run follows the cursor atomics, so the fp32 summation order can
// differ run to run (DDP ranks still agree after the all-reduce).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <type_traits>
#include <vector>

#include "nbd_common.h"

namespace nbd {
namespace embed {

constexpr int NT = 256;
constexpr int kScanT = 1024;

// the id of the wave's first lane with a valid id (-1 if none): the wave's most likely repeat
__device__ __forceinline__ int wave_first_id(bool ok, int v) {
  const uint64_t m = __ballot(ok);
  if (m == 0) return -1;
  return __shfl(v, __ffsll((unsigned long long)m) - 1, kWave);
}

__global__ __launch_bounds__(NT) void count_kernel(const int64_t* __restrict__ idx, int64_t n, int V,
                                                   int* __restrict__ counts, int* __restrict__ bad) {
  for (int64_t i0 = (int64_t)blockIdx.x * NT; i0 < n; i0 += (int64_t)gridDim.x * NT) {
    const int64_t i = i0 + threadIdx.x;
    const int64_t v = i < n ? idx[i] : -1;
    const bool ok = i < n && v >= 0 && v < V;
    if (i < n && !ok) atomicOr(bad, 1);  // out-of-range id: flagged, never written out of bounds
    // lanes holding the wave's first valid id count it with one atomic (a padding run would
    // otherwise be hundreds of same-address atomics in a row)
    const int lead = wave_first_id(ok, (int)v);
    const uint64_t same = __ballot(ok && v == lead);
    if (ok && v == lead) {
      if (__lane_id() == (unsigned)(__ffsll((unsigned long long)same) - 1)) atomicAdd(&counts[v], (int)__popcll(same));
    } else if (ok) {
      atomicAdd(&counts[v], 1);
    }
  }
}

// exclusive scan of counts[0..V) into offsets[0..V], pass 1: block-local scans + block sums
__global__ __launch_bounds__(kScanT) void scan_local_kernel(const int* __restrict__ counts, int V,
                                                            int* __restrict__ offsets, int* __restrict__ bsum) {
  __shared__ int part[kScanT];
  const int t = threadIdx.x;
  const int i = blockIdx.x * kScanT + t;
  const int c = i < V ? counts[i] : 0;
  part[t] = c;
  __syncthreads();
  for (int off = 1; off < kScanT; off <<= 1) {  // Hillis-Steele inclusive scan
    const int add = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += add;
    __syncthreads();
  }
  if (i < V) offsets[i] = part[t] - c;
  if (t == kScanT - 1) bsum[blockIdx.x] = part[t];
}

// pass 2: add the sum of all earlier blocks; the last block also writes offsets[V]
__global__ __launch_bounds__(kScanT) void scan_add_kernel(int* __restrict__ offsets, int V,
                                                          const int* __restrict__ bsum, int nblk) {
  __shared__ int base;
  if (threadIdx.x == 0) {
    int s = 0;
    for (int b = 0; b < (int)blockIdx.x; ++b) s += bsum[b];
    base = s;
  }
  __syncthreads();
  const int i = blockIdx.x * kScanT + threadIdx.x;
  if (i < V) offsets[i] += base;
  if (blockIdx.x == nblk - 1 && threadIdx.x == 0) offsets[V] = base + bsum[nblk - 1];
}

__global__ __launch_bounds__(NT) void place_kernel(const int64_t* __restrict__ idx, int64_t n, int V,
                                                   const int* __restrict__ offsets, int* __restrict__ cursor,
                                                   int* __restrict__ order) {
  for (int64_t i0 = (int64_t)blockIdx.x * NT; i0 < n; i0 += (int64_t)gridDim.x * NT) {
    const int64_t i = i0 + threadIdx.x;
    const int64_t v = i < n ? idx[i] : -1;
    const bool ok = i < n && v >= 0 && v < V;
    const int lead = wave_first_id(ok, (int)v);
    const uint64_t same = __ballot(ok && v == lead);
    if (ok && v == lead) {  // one cursor atomic for the wave's lanes of the first id, ranked by lane
      const int first = __ffsll((unsigned long long)same) - 1;
      int base = 0;
      if (__lane_id() == (unsigned)first) base = atomicAdd(&cursor[v], (int)__popcll(same));
      base = __shfl(base, first, kWave);
      const int rank = (int)__popcll(same & ((1ull << __lane_id()) - 1));
      order[offsets[v] + base + rank] = (int)i;
    } else if (ok) {
      order[offsets[v] + atomicAdd(&cursor[v], 1)] = (int)i;
    }
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

// one wave per 16 sorted slots: sum runs of equal ids, flush each run into acc[offsets[id]].
// The slots' token rows and ids are fetched for all 16 slots at once (one per lane: two
// dependent loads per wave, not per slot), and the dy rows up to four slots at a time, so a wave does
// not wait out three memory latencies per slot (77 µs for GPT-2's 8192 mostly distinct ids, a
// dependent chain per slot).  Only a run that continues into the previous or the next wave's
// slots is added with float atomics; runs inside the wave's slots belong to it alone and are
// plain stores into the zeroed scratch.
constexpr int kSlots = 16;

template <typename T, int NCH>
__global__ __launch_bounds__(NT) void partial_kernel(const T* __restrict__ dy, int C, const int64_t* __restrict__ idx,
                                                     const int* __restrict__ offsets, const int* __restrict__ order,
                                                     int V, float* __restrict__ acc) {
  const int lane = threadIdx.x & 63;
  const int64_t s0 = ((int64_t)blockIdx.x * (NT / kWave) + (threadIdx.x >> 6)) * kSlots;
  const int n_valid = offsets[V];  // placed (in-range) tokens; never read unwritten slots of `order`
  if (s0 >= n_valid) return;
  const int ns = (int)min<int64_t>(kSlots, n_valid - s0);
  int my_row = 0, my_v = 0;
  if (lane < ns) {
    my_row = order[s0 + lane];
    my_v = (int)idx[my_row];
  }
  const int v_first = __builtin_amdgcn_readlane(my_v, 0);
  float run[NCH][4];
  auto zero = [&]() {
#pragma unroll
    for (int k = 0; k < NCH; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) run[k][e] = 0.f;
  };
  // a run's sum over this wave's slots goes to scratch row max(offsets[v], s0): the run's first
  // slot, or this wave's first slot when the run started in an earlier wave — every row written
  // by exactly one wave, plain stores, no zero-fill; rows_kernel adds a run's per-wave rows
  auto flush = [&](int v) {
    float* dst = acc + (int64_t)max(offsets[v], (int)s0) * C;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = 4 * lane + 256 * k;
      if (c < C) *reinterpret_cast<float4*>(dst + c) = make_float4(run[k][0], run[k][1], run[k][2], run[k][3]);
    }
  };
  zero();
  int cur = v_first;
  constexpr int G = NCH <= 4 ? 4 : NCH <= 8 ? 2 : 1;  // dy rows in flight (registers: G·NCH·4)
  for (int j0 = 0; j0 < ns; j0 += G) {
    float x[G][NCH][4];
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int j = j0 + u < ns ? j0 + u : ns - 1;  // (a repeat of the last slot is loaded, not used)
      const int row = __builtin_amdgcn_readlane(my_row, j);
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < C) ld4<T>(dy + (int64_t)row * C + c, x[u][k]);
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      if (j0 + u >= ns) break;
      const int v = __builtin_amdgcn_readlane(my_v, j0 + u);
      if (v != cur) {
        flush(cur);
        cur = v;
        zero();
      }
#pragma unroll
      for (int k = 0; k < NCH; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) run[k][e] += x[u][k][e];
    }
  }
  flush(cur);
}

// one wave per gradient row; a lane owns 4-column chunks c = 4·lane + 256·k, k < NCH.  Rows
// [V, R) (a table padded past the vocabulary) get zeros.  `accumulate`: add into the gradient
// instead (it already holds another contribution — the tied LM head's, ops/embedding.py), and
// touch only the rows some token hit.
template <typename T, int NCH>
__global__ __launch_bounds__(NT) void rows_kernel(const float* __restrict__ acc, int C, const int* __restrict__ offsets,
                                                  int V, int R, T* __restrict__ grad, int accumulate) {
  const int lane = threadIdx.x & 63;
  const int64_t v = (int64_t)blockIdx.x * (NT / kWave) + (threadIdx.x >> 6);
  if (v >= R) return;
  const int b = v < V ? offsets[v] : 0;
  const int e = v < V ? offsets[v + 1] : 0;
  const bool hit = e > b;
  if (accumulate && !hit) return;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < C) {
      float x[4] = {0.f, 0.f, 0.f, 0.f};
      if (hit) {
        const float4 a = *reinterpret_cast<const float4*>(acc + (int64_t)b * C + c);
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
        // a run longer than one wave's slots: one more row per wave it reached (first slots of
        // those waves), four loads in flight at a time
        for (int r = (b / kSlots + 1) * kSlots; r < e; r += 4 * kSlots) {
          float4 y[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            y[u] = r + u * kSlots < e ? *reinterpret_cast<const float4*>(acc + (int64_t)(r + u * kSlots) * C + c)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            x[0] += y[u].x; x[1] += y[u].y; x[2] += y[u].z; x[3] += y[u].w;
          }
        }
      }
      if (accumulate) {
        float o[4];
        ld4<T>(grad + v * C + c, o);
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] += o[e];
      }
      st4<T>(grad + v * C + c, x);
    }
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
// ---- token + position embedding forward: out[r] = wte[idx[r]] + wpe[pos[r % T]] ---------------
// One pass (16 B per lane from each table, fp32 add, one rounding — the same bits as
// F.embedding(idx, wte) + F.embedding(pos, wpe) in the tables' dtype) instead of two gathers and
// an add.  Out-of-range ids (outside [0, V): V = the vocabulary, which may be smaller than the
// table when its rows are padded) read as zero rows and set `err` (F.embedding would raise; the
// host cannot check without a sync — ops/embedding.py reads the flag lazily and raises there).
template <typename T>
__global__ __launch_bounds__(NT) void tokpos_kernel(const int64_t* __restrict__ idx, const int64_t* __restrict__ pos, int T_,
                                                    const T* __restrict__ wte, int V, const T* __restrict__ wpe, int P, int C,
                                                    int64_t n8, T* __restrict__ out, int* __restrict__ err) {
  const int c8 = C / 8;
  for (int64_t i = blockIdx.x * (int64_t)NT + threadIdx.x; i < n8; i += (int64_t)gridDim.x * NT) {
    const int64_t r = i / c8;
    const int c = (int)(i - r * c8) * 8;
    const int64_t v = idx[r], q = pos[r % T_];
    float a[8], b[8];
    if (v >= 0 && v < V) {
      load8<T>(wte + v * C + c, a);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = 0.f;
      if (err != nullptr && c == 0) atomicOr(err, 1);  // (a vector-memory atomic)
    }
    if (q >= 0 && q < P)
      load8<T>(wpe + q * C + c, b);
    else
#pragma unroll
      for (int e = 0; e < 8; ++e) b[e] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] += b[e];
    store8<T>(out + r * C + c, a);
  }
}

at::Tensor embedding_tokpos_hip(const at::Tensor& idx, const at::Tensor& wte, const at::Tensor& pos, const at::Tensor& wpe,
                                int64_t vocab, const c10::optional<at::Tensor>& err) {
  TORCH_CHECK(idx.is_cuda() && wte.is_cuda() && pos.is_cuda() && wpe.is_cuda(), "embedding_tokpos: GPU tensors expected");
  TORCH_CHECK(idx.scalar_type() == at::kLong && pos.scalar_type() == at::kLong && idx.is_contiguous() && pos.is_contiguous() &&
                  pos.dim() == 1 && pos.numel() > 0 && idx.numel() % pos.numel() == 0,
              "embedding_tokpos: int64 ids [..., T] and positions [T]");
  TORCH_CHECK(wte.dim() == 2 && wpe.dim() == 2 && wte.size(1) == wpe.size(1) && wte.is_contiguous() && wpe.is_contiguous() &&
                  wte.scalar_type() == wpe.scalar_type(),
              "embedding_tokpos: contiguous [V, C] / [P, C] tables of one dtype");
  const int64_t C = wte.size(1), N = idx.numel();
  const int64_t V = vocab > 0 ? std::min<int64_t>(vocab, wte.size(0)) : wte.size(0);
  if (err) TORCH_CHECK(err->is_cuda() && err->scalar_type() == at::kInt && err->numel() >= 1, "embedding_tokpos: int32 error flag");
  TORCH_CHECK(C % 8 == 0 && ((uintptr_t)wte.data_ptr() & 15) == 0 && ((uintptr_t)wpe.data_ptr() & 15) == 0,
              "embedding_tokpos: C % 8 == 0 and 16-B aligned tables");
  std::vector<int64_t> shape(idx.sizes().begin(), idx.sizes().end());
  shape.push_back(C);
  at::Tensor out = at::empty(shape, wte.options());
  if (N == 0) return out;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(wte.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int64_t n8 = N * C / 8;
  const int blocks = (int)std::min<int64_t>((n8 + NT - 1) / NT, 4096);
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((tokpos_kernel<T>), dim3(blocks), dim3(NT), 0, st, idx.data_ptr<int64_t>(), pos.data_ptr<int64_t>(),
                       (int)pos.numel(), static_cast<const T*>(wte.data_ptr()), (int)V,
                       static_cast<const T*>(wpe.data_ptr()), (int)wpe.size(0), (int)C, n8, static_cast<T*>(out.data_ptr()),
                       err ? err->data_ptr<int>() : nullptr);
  };
  switch (wte.scalar_type()) {
    case at::kFloat: launch(float{}); break;
    case at::kBFloat16: launch(bf16_t{}); break;
    case at::kHalf: launch(f16_t{}); break;
    default: TORCH_CHECK(false, "embedding_tokpos: unsupported dtype ", wte.scalar_type());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

// grad_out: write (or with `accumulate`, add) the gradient there — [R, C] with R >= V rows
// (a vocabulary-padded table, or the tied LM head's gradient slot, graddst.h)
at::Tensor embedding_bwd_hip(const at::Tensor& dy, const at::Tensor& idx, int64_t V,
                             const c10::optional<at::Tensor>& grad_out, bool accumulate) {
  TORCH_CHECK(dy.is_cuda() && idx.is_cuda(), "embedding_bwd: GPU tensors expected");
  TORCH_CHECK(dy.dim() == 2 && dy.is_contiguous(), "embedding_bwd: dy must be a contiguous [N, C]");
  TORCH_CHECK(idx.dim() == 1 && idx.is_contiguous() && idx.scalar_type() == at::kLong && idx.size(0) == dy.size(0),
              "embedding_bwd: ids must be a contiguous int64 [N]");
  const int64_t N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(C % 4 == 0 && C <= 4096, "embedding_bwd: C must be a multiple of 4 and <= 4096");
  TORCH_CHECK(V > 0 && V < (1LL << 31) && N < (1LL << 31), "embedding_bwd: sizes out of range");
  TORCH_CHECK(((uintptr_t)dy.data_ptr() & 15) == 0, "embedding_bwd: dy must be 16-B aligned");
  at::Tensor grad;
  if (grad_out) {
    grad = *grad_out;
    TORCH_CHECK(grad.dim() == 2 && grad.size(0) >= V && grad.size(1) == C && grad.is_contiguous() &&
                    grad.scalar_type() == dy.scalar_type() && ((uintptr_t)grad.data_ptr() & 15) == 0,
                "embedding_bwd: grad_out must be a contiguous, aligned [R >= V, C] tensor of dy's dtype");
  } else {
    TORCH_CHECK(!accumulate, "embedding_bwd: accumulate needs grad_out");
    grad = at::empty({V, C}, dy.options());
  }
  const int64_t R = grad.size(0);
  auto io = idx.options().dtype(at::kInt);
  at::Tensor cc = at::zeros({2 * V + 1}, io);  // one fill: counts [0, V], flag [V], cursor [V+1, 2V+1)
  at::Tensor counts = cc.narrow(0, 0, V + 1);
  at::Tensor cursor = cc.narrow(0, V + 1, V);
  at::Tensor offsets = at::empty({V + 1}, io);
  const int nsb = (int)((V + kScanT - 1) / kScanT);
  at::Tensor bsum = at::empty({nsb}, io);
  at::Tensor order = at::empty({std::max<int64_t>(N, 1)}, io);
  at::Tensor acc = at::empty({std::max<int64_t>(N, 1), C}, dy.options().dtype(at::kFloat));  // rows read = rows written
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int blocks = (int)std::min<int64_t>((N + NT - 1) / NT + 1, 1024);
  int* cnt = counts.data_ptr<int>();
  hipLaunchKernelGGL(count_kernel, dim3(blocks), dim3(NT), 0, st, idx.data_ptr<int64_t>(), N, (int)V, cnt, cnt + V);
  hipLaunchKernelGGL(scan_local_kernel, dim3(nsb), dim3(kScanT), 0, st, cnt, (int)V, offsets.data_ptr<int>(),
                     bsum.data_ptr<int>());
  hipLaunchKernelGGL(scan_add_kernel, dim3(nsb), dim3(kScanT), 0, st, offsets.data_ptr<int>(), (int)V,
                     bsum.data_ptr<int>(), nsb);
  hipLaunchKernelGGL(place_kernel, dim3(blocks), dim3(NT), 0, st, idx.data_ptr<int64_t>(), N, (int)V,
                     offsets.data_ptr<int>(), cursor.data_ptr<int>(), order.data_ptr<int>());
  // slots [0, offsets[V]) hold every in-range token; out-of-range ids are flagged and never
  // placed, and partial_kernel stops at offsets[V] (read on the device)
  const dim3 pgrid((unsigned)((N + kSlots * 4 - 1) / (kSlots * 4)));
  const dim3 rgrid((unsigned)((R + 3) / 4));
  dispatch_nch(C, [&](auto nch) {
    constexpr int K = decltype(nch)::value;
    auto launch = [&](auto tag) {
      using T = decltype(tag);
      hipLaunchKernelGGL((partial_kernel<T, K>), pgrid, dim3(NT), 0, st, static_cast<const T*>(dy.data_ptr()), (int)C,
                         idx.data_ptr<int64_t>(), offsets.data_ptr<int>(), order.data_ptr<int>(), (int)V,
                         acc.data_ptr<float>());
      hipLaunchKernelGGL((rows_kernel<T, K>), rgrid, dim3(NT), 0, st, acc.data_ptr<float>(), (int)C,
                         offsets.data_ptr<int>(), (int)V, (int)R, static_cast<T*>(grad.data_ptr()), accumulate ? 1 : 0);
    };
    switch (dy.scalar_type()) {
      case at::kFloat: launch(float{}); break;
      case at::kBFloat16: launch(bf16_t{}); break;
      case at::kHalf: launch(f16_t{}); break;
      default: TORCH_CHECK(false, "embedding_bwd: unsupported dtype ", dy.scalar_type());
    }
  });
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return grad;
}

// Position-table gradient of token + position embeddings: out[pos[t]] (+)= Σ_b dy[b·T + t]
// (fp32 sum over the batch in a fixed order, rounded once) — one launch where torch ran a
// batch sum, a zero fill, an index_add and a cast (≈ 25 µs per GPT-2 step).  Positions are
// unique (the caller's contract), so no two threads write one row.  Rows of `out` that no
// position hits are zeroed by the caller (not needed when the T positions cover all P rows).
template <typename T>
__global__ __launch_bounds__(256) void pos_bwd_kernel(const T* __restrict__ dy, const int64_t* __restrict__ pos,
                                                      int B, int Tn, int C, int P, T* __restrict__ out, int accumulate) {
  const int C8 = C / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)Tn * C8) return;
  const int t = (int)(i / C8), c = (int)(i % C8) * 8;
  const int64_t p = pos[t];
  if (p < 0 || p >= P) return;  // (out of range: the forward's id check reports it)
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < B; ++b) {
    float x[8];
    load8<T>(dy + ((int64_t)b * Tn + t) * C + c, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += x[e];
  }
  T* o = out + p * C + c;
  if (accumulate) {
    float x[8];
    load8<T>(o, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += x[e];
  }
  store8<T>(o, acc);
}

// grad [P, C] of the position table from dy [B·T, C]; out given: written (or += with accumulate)
at::Tensor embedding_pos_bwd_hip(const at::Tensor& dy, const at::Tensor& pos, int64_t P,
                                 const c10::optional<at::Tensor>& out_opt, bool accumulate) {
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 2 && dy.is_contiguous() && dy.size(1) % 8 == 0,
              "embedding_pos_bwd: contiguous [rows, C] GPU dy with C % 8 == 0");
  TORCH_CHECK(pos.is_cuda() && pos.scalar_type() == at::kLong && pos.dim() == 1 && pos.is_contiguous() && pos.numel() > 0 &&
                  dy.size(0) % pos.numel() == 0,
              "embedding_pos_bwd: int64 [T] positions dividing dy's rows");
  const int64_t Tn = pos.numel(), C = dy.size(1), B = dy.size(0) / Tn;
  TORCH_CHECK(P >= Tn && P * C < (1LL << 31) && B * Tn * C < (1LL << 40), "embedding_pos_bwd: sizes");
  at::Tensor out;
  if (out_opt.has_value() && out_opt->defined()) {
    out = *out_opt;
    TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.scalar_type() == dy.scalar_type() && out.size(0) == P &&
                    out.size(1) == C,
                "embedding_pos_bwd: out must be a contiguous [P, C] tensor of dy's dtype");
  } else {
    out = at::empty({P, C}, dy.options());
    accumulate = false;
  }
  // positions are unique: T == P means every row is written; otherwise the rest must be zero
  if (!accumulate && Tn < P) out.zero_();
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "embedding_pos_bwd: 16-byte aligned tensors");
  const int64_t work = Tn * (C / 8);
  if (work == 0 || B == 0) return out;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(dy.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const dim3 grid((unsigned)((work + 255) / 256));
  switch (dy.scalar_type()) {
#define NBD_PB(ATY, T)                                                                                                \
  case ATY:                                                                                                           \
    hipLaunchKernelGGL(pos_bwd_kernel<T>, grid, dim3(256), 0, st, static_cast<const T*>(dy.data_ptr()),               \
                       pos.data_ptr<int64_t>(), (int)B, (int)Tn, (int)C, (int)P, static_cast<T*>(out.data_ptr()),     \
                       accumulate ? 1 : 0);                                                                           \
    break;
    NBD_PB(at::kFloat, float)
    NBD_PB(at::kBFloat16, bf16_t)
    NBD_PB(at::kHalf, f16_t)
#undef NBD_PB
    default: TORCH_CHECK(false, "embedding_pos_bwd: unsupported dtype ", dy.scalar_type());
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

}  // namespace embed
}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("embedding_bwd", &nbd::embed::embedding_bwd_hip);
  m.impl("embedding_tokpos", &nbd::embed::embedding_tokpos_hip);
  m.impl("embedding_pos_bwd", &nbd::embed::embedding_pos_bwd_hip);
}
