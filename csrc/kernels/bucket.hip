// bucket.hip — gradient-bucket flatten / unflatten and local pre-reduce for gfx950.
//
// K1 bucket_flatten   : N tensors -> one contiguous communication bucket, fused dtype cast
//                       (fp32 grads -> bf16 wire format) and scale (pre-divide by world size).
// K2 bucket_unflatten : bucket -> N tensors, fused scale (x 1/world), cast back and optional
//                       accumulate (grad += reduced) — one pass instead of copy/div/add kernels.
// K3 local_prereduce  : out = scale * sum_i in_i over k same-shape buffers (fp32 accumulate),
//                       e.g. summing micro-batch gradient buckets once before one all-reduce.
//
// Reference behaviour replaced: DDP's reducer copies every grad into bucket views and then runs
// separate cast / divide / copy-back kernels (torch nn/parallel/distributed.py).
//
// Design (MI355X): pure HBM streaming, so the only levers are bytes and launches.
//  * one launch per <= 256 tensors: the tensor table (7 KiB) travels in the kernel arguments —
//    gfx950/HIP accepts >= 16 KiB of arguments (csrc/kernels/bench/kernarg.hip), so a whole
//    GPT-2 gradient set is one launch with no H2D metadata copy; work is cut in 8 Ki-element
//    chunks (measured best block footprint, csrc/kernels/bench/copy_bw.hip: 16-32 KiB per block
//    5.6-5.7 TB/s vs 64 KiB 5.3) and the chunk->tensor lookup is a block-uniform binary search
//    over the prefix table (scalar ALU);
//  * 16-bit destinations written with non-temporal stores (streamed once; measured +3-6 %;
//    fp32 NT stores were 20 % slower and are not used);
//  * 16 B per lane per access (8 elements), loads for a whole unrolled group issued before the
//    converts/stores so each wave keeps several KiB in flight;
//  * misaligned tensors (storage offsets not multiple of 16 B) fall back to a scalar path inside
//    the same launch — correctness never depends on the bucket planner's padding.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>
#include <vector>

#include "nbd_common.h"

namespace nbd {

constexpr int kMaxT = 256;
constexpr int64_t kChunk = 8192;
constexpr int kThreads = 256;
constexpr int kUnroll = 2;

constexpr int kHint = 2048;  // coarse chunk-group -> tensor table (uint8: kMaxT <= 256)

struct CopyTable {
  const void* src[kMaxT];
  void* dst[kMaxT];
  int64_t numel[kMaxT];
  int32_t chunk_prefix[kMaxT + 1];
  int32_t group_chunks;    // chunks per hint group
  uint8_t hint[kHint];     // tensor owning the first chunk of each group
  uint64_t aligned_mask[kMaxT / 64];  // bit t: both src[t] and dst[t] are 16 B aligned
};

template <typename S, typename D, bool ACC>
__global__ __launch_bounds__(kThreads) void multi_copy_kernel(CopyTable tab, int nt, float scale) {
  const int chunk = blockIdx.x;
  // chunk -> tensor: coarse hint, then a short forward scan (block-uniform, scalar loads).
  // A binary search over the prefix table (8 dependent scalar loads per block) cost 18 % of
  // the kernel on the GPT-2 gradient set (4.5 vs 5.5 TB/s single tensor, ops_bench.py).
  int t = tab.hint[chunk / tab.group_chunks];
  while (t + 1 < nt && tab.chunk_prefix[t + 1] <= chunk) ++t;
  const int64_t begin = (int64_t)(chunk - tab.chunk_prefix[t]) * kChunk;
  const int64_t end = min(begin + kChunk, tab.numel[t]);
  const S* __restrict__ src = static_cast<const S*>(tab.src[t]);
  D* __restrict__ dst = static_cast<D*>(tab.dst[t]);

  if ((tab.aligned_mask[t >> 6] >> (t & 63)) & 1ull) {
    const int64_t stride = (int64_t)kThreads * 8;
    int64_t i = begin + (int64_t)threadIdx.x * 8;
    for (; i + (kUnroll - 1) * stride + 8 <= end; i += kUnroll * stride) {
      float v[kUnroll][8];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) load8<S>(src + i + u * stride, v[u]);
      if (ACC) {
        float w[kUnroll][8];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) load8<D>(dst + i + u * stride, w[u]);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u][j] = fmaf(v[u][j], scale, w[u][j]);
      } else {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u][j] *= scale;
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        // non-temporal only for 16-bit destinations: +3-6 % there, but fp32 NT stores measured
        // 20 % slower (unflatten 3.4 vs 4.2 TB/s); accumulate is read-modify-write: keep cached
        if (!ACC && sizeof(D) == 2) store8_nt<D>(dst + i + u * stride, v[u]);
        else store8<D>(dst + i + u * stride, v[u]);
      }
    }
    for (; i + 8 <= end; i += stride) {
      float v[8];
      load8<S>(src + i, v);
      if (ACC) {
        float w[8];
        load8<D>(dst + i, w);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], scale, w[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= scale;
      }
      store8<D>(dst + i, v);
    }
    // < 8 trailing elements of this chunk (only the last chunk of a tensor can have them)
    if (i < end) {
      for (int64_t k = i; k < end; ++k) {
        float x = Elem<S>::load(src, k) * scale;
        if (ACC) x += Elem<D>::load(dst, k);
        Elem<D>::store(dst, k, x);
      }
    }
  } else {
    for (int64_t k = begin + threadIdx.x; k < end; k += kThreads) {
      float x = Elem<S>::load(src, k) * scale;
      if (ACC) x += Elem<D>::load(dst, k);
      Elem<D>::store(dst, k, x);
    }
  }
}

// ---- host side -------------------------------------------------------------------------------

struct CopyItem {
  const void* src;
  void* dst;
  int64_t numel;
};

template <typename S, typename D>
static void launch_copy(const std::vector<CopyItem>& items, float scale, bool acc, hipStream_t stream) {
  size_t pos = 0;
  while (pos < items.size()) {
    CopyTable tab{};
    int nt = 0;
    int32_t chunks = 0;
    for (; pos < items.size() && nt < kMaxT; ++pos) {
      const CopyItem& it = items[pos];
      if (it.numel == 0) continue;
      tab.src[nt] = it.src;
      tab.dst[nt] = it.dst;
      tab.numel[nt] = it.numel;
      tab.chunk_prefix[nt] = chunks;
      if (((uintptr_t)it.src % 16 == 0) && ((uintptr_t)it.dst % 16 == 0))
        tab.aligned_mask[nt >> 6] |= (1ull << (nt & 63));
      const int64_t c = (it.numel + kChunk - 1) / kChunk;
      TORCH_CHECK(chunks + c < (int64_t)INT32_MAX, "nbd bucket: too many chunks in one launch");
      chunks += (int32_t)c;
      ++nt;
    }
    if (nt == 0) continue;
    tab.chunk_prefix[nt] = chunks;
    tab.group_chunks = (chunks + kHint - 1) / kHint;
    if (tab.group_chunks < 1) tab.group_chunks = 1;
    for (int g = 0, t = 0; g < kHint; ++g) {
      const int32_t first = g * tab.group_chunks;
      while (t + 1 < nt && tab.chunk_prefix[t + 1] <= first) ++t;
      tab.hint[g] = (uint8_t)t;
    }
    if (acc)
      hipLaunchKernelGGL((multi_copy_kernel<S, D, true>), dim3(chunks), dim3(kThreads), 0, stream, tab, nt, scale);
    else
      hipLaunchKernelGGL((multi_copy_kernel<S, D, false>), dim3(chunks), dim3(kThreads), 0, stream, tab, nt, scale);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
}

template <typename S>
static void dispatch_dst(at::ScalarType dt, const std::vector<CopyItem>& items, float scale, bool acc, hipStream_t st) {
  switch (dt) {
    case at::kFloat: launch_copy<S, float>(items, scale, acc, st); break;
    case at::kBFloat16: launch_copy<S, bf16_t>(items, scale, acc, st); break;
    case at::kHalf: launch_copy<S, f16_t>(items, scale, acc, st); break;
    default: TORCH_CHECK(false, "nbd bucket: unsupported destination dtype ", dt);
  }
}

static void dispatch_copy(at::ScalarType st_, at::ScalarType dt, const std::vector<CopyItem>& items, float scale,
                          bool acc, hipStream_t stream) {
  switch (st_) {
    case at::kFloat: dispatch_dst<float>(dt, items, scale, acc, stream); break;
    case at::kBFloat16: dispatch_dst<bf16_t>(dt, items, scale, acc, stream); break;
    case at::kHalf: dispatch_dst<f16_t>(dt, items, scale, acc, stream); break;
    default: TORCH_CHECK(false, "nbd bucket: unsupported source dtype ", st_);
  }
}

static int64_t elem_size(at::ScalarType t) { return (int64_t)c10::elementSize(t); }

// accumulate: bucket[slice] += scale * t (fp32 math) — the local pre-reduce of micro-batch
// gradients into their bucket (DDP no_sync, parallel/ddp.py), instead of overwriting it
void bucket_flatten_hip(at::TensorList tensors, const at::Tensor& bucket, at::IntArrayRef offsets, double scale,
                        bool accumulate) {
  TORCH_CHECK(bucket.is_cuda() && bucket.is_contiguous(), "bucket must be a contiguous GPU tensor");
  TORCH_CHECK((int64_t)tensors.size() == (int64_t)offsets.size(), "tensors/offsets length mismatch");
  if (tensors.empty()) return;
  const at::ScalarType src_t = tensors[0].scalar_type();
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bucket.device());
  std::vector<CopyItem> items;
  items.reserve(tensors.size());
  char* base = static_cast<char*>(bucket.data_ptr());
  const int64_t es = elem_size(bucket.scalar_type());
  for (size_t i = 0; i < tensors.size(); ++i) {
    const at::Tensor& t = tensors[i];
    TORCH_CHECK(t.is_cuda() && t.device() == bucket.device(), "tensor ", i, " is not on the bucket's device");
    TORCH_CHECK(t.is_contiguous(), "tensor ", i, " must be contiguous");
    TORCH_CHECK(t.scalar_type() == src_t, "all tensors must share one dtype");
    TORCH_CHECK(offsets[i] >= 0 && offsets[i] + t.numel() <= bucket.numel(), "tensor ", i, " does not fit the bucket");
    items.push_back({t.data_ptr(), base + offsets[i] * es, t.numel()});
  }
  dispatch_copy(src_t, bucket.scalar_type(), items, (float)scale, accumulate,
                c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
}

void bucket_unflatten_hip(const at::Tensor& bucket, at::TensorList tensors, at::IntArrayRef offsets, double scale,
                          bool accumulate) {
  TORCH_CHECK(bucket.is_cuda() && bucket.is_contiguous(), "bucket must be a contiguous GPU tensor");
  TORCH_CHECK((int64_t)tensors.size() == (int64_t)offsets.size(), "tensors/offsets length mismatch");
  if (tensors.empty()) return;
  const at::ScalarType dst_t = tensors[0].scalar_type();
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(bucket.device());
  std::vector<CopyItem> items;
  items.reserve(tensors.size());
  const char* base = static_cast<const char*>(bucket.data_ptr());
  const int64_t es = elem_size(bucket.scalar_type());
  for (size_t i = 0; i < tensors.size(); ++i) {
    const at::Tensor& t = tensors[i];
    TORCH_CHECK(t.is_cuda() && t.device() == bucket.device(), "tensor ", i, " is not on the bucket's device");
    TORCH_CHECK(t.is_contiguous(), "tensor ", i, " must be contiguous");
    TORCH_CHECK(t.scalar_type() == dst_t, "all tensors must share one dtype");
    TORCH_CHECK(offsets[i] >= 0 && offsets[i] + t.numel() <= bucket.numel(), "tensor ", i, " does not fit the bucket");
    items.push_back({base + offsets[i] * es, t.data_ptr(), t.numel()});
  }
  dispatch_copy(bucket.scalar_type(), dst_t, items, (float)scale, accumulate, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
}

// ---- K3: local pre-reduce --------------------------------------------------------------------
constexpr int kMaxIn = 16;
struct ReduceArgs {
  const void* in[kMaxIn];
};

// One block per kChunk-element chunk (the block footprint the copy kernels measured best at,
// copy_bw.hip) and kUnroll 16-B vectors per input per thread in flight before any add: a
// grid-stride loop over 8-element vectors capped at 2048 blocks reached 4.5 TB/s (4 x bf16 ->
// bf16, docs/FINDINGS.md §3); the inputs are streamed once (non-temporal loads), the output
// written once (non-temporal for 16-bit types).
template <typename S, typename D, int KT>  // KT >= k: the register image of the inputs in flight
__global__ __launch_bounds__(kThreads) void prereduce_kernel(ReduceArgs a, int k, void* out_, int64_t n, float scale,
                                                             int aligned) {
  D* __restrict__ out = static_cast<D*>(out_);
  const int64_t begin = (int64_t)blockIdx.x * kChunk;
  const int64_t end = min(begin + kChunk, n);
  if (aligned) {
    constexpr int64_t stride = (int64_t)kThreads * 8;
    int64_t i = begin + (int64_t)threadIdx.x * 8;
    for (; i + (kUnroll - 1) * stride + 8 <= end; i += kUnroll * stride) {
      float acc[kUnroll][8];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[u][e] = 0.f;
      // every input's loads for both vectors are issued before the adds
      float x[KT][kUnroll][8];
#pragma unroll
      for (int j = 0; j < KT; ++j)
        if (j < k)
#pragma unroll
          for (int u = 0; u < kUnroll; ++u) load8_nt<S>(static_cast<const S*>(a.in[j]) + i + u * stride, x[j][u]);
#pragma unroll
      for (int j = 0; j < KT; ++j)
        if (j < k)
#pragma unroll
          for (int u = 0; u < kUnroll; ++u)
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[u][e] += x[j][u][e];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[u][e] *= scale;
        if (sizeof(D) == 2) store8_nt<D>(out + i + u * stride, acc[u]);
        else store8<D>(out + i + u * stride, acc[u]);
      }
    }
    for (; i + 8 <= end; i += stride) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int j = 0; j < k; ++j) {
        float x[8];
        load8<S>(static_cast<const S*>(a.in[j]) + i, x);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += x[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] *= scale;
      store8<D>(out + i, acc);
    }
    for (int64_t t = i; t < end && t < i + 8; ++t) {  // < 8 trailing elements (last chunk only)
      float v = 0.f;
      for (int j = 0; j < k; ++j) v += Elem<S>::load(static_cast<const S*>(a.in[j]), t);
      Elem<D>::store(out, t, v * scale);
    }
  } else {
    for (int64_t t = begin + threadIdx.x; t < end; t += kThreads) {
      float v = 0.f;
      for (int j = 0; j < k; ++j) v += Elem<S>::load(static_cast<const S*>(a.in[j]), t);
      Elem<D>::store(out, t, v * scale);
    }
  }
}

template <typename S, typename D>
static void launch_prereduce(const ReduceArgs& a, int k, void* out, int64_t n, float scale, int aligned,
                             hipStream_t st) {
  const int64_t blocks = std::max<int64_t>(1, (n + kChunk - 1) / kChunk);
  TORCH_CHECK(blocks < (1LL << 31), "local_prereduce: too many elements");
  const dim3 g((unsigned)blocks), b(kThreads);
  if (k <= 2) hipLaunchKernelGGL((prereduce_kernel<S, D, 2>), g, b, 0, st, a, k, out, n, scale, aligned);
  else if (k <= 4) hipLaunchKernelGGL((prereduce_kernel<S, D, 4>), g, b, 0, st, a, k, out, n, scale, aligned);
  else if (k <= 8) hipLaunchKernelGGL((prereduce_kernel<S, D, 8>), g, b, 0, st, a, k, out, n, scale, aligned);
  else hipLaunchKernelGGL((prereduce_kernel<S, D, kMaxIn>), g, b, 0, st, a, k, out, n, scale, aligned);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

template <typename S>
static void prereduce_dst(at::ScalarType dt, const ReduceArgs& a, int k, void* out, int64_t n, float scale, int al,
                          hipStream_t st) {
  switch (dt) {
    case at::kFloat: launch_prereduce<S, float>(a, k, out, n, scale, al, st); break;
    case at::kBFloat16: launch_prereduce<S, bf16_t>(a, k, out, n, scale, al, st); break;
    case at::kHalf: launch_prereduce<S, f16_t>(a, k, out, n, scale, al, st); break;
    default: TORCH_CHECK(false, "nbd prereduce: unsupported output dtype ", dt);
  }
}

void local_prereduce_hip(at::TensorList inputs, const at::Tensor& out, double scale) {
  // > kMaxIn inputs are grouped by the Python wrapper (nbdistributed_amd.ops.local_prereduce).
  TORCH_CHECK(!inputs.empty() && (int)inputs.size() <= kMaxIn, "local_prereduce: 1..", kMaxIn, " inputs per call");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous(), "out must be a contiguous GPU tensor");
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(out.device());
  const at::ScalarType st_ = inputs[0].scalar_type();
  const int64_t n = out.numel();
  ReduceArgs a{};
  int aligned = ((uintptr_t)out.data_ptr() % 16 == 0) ? 1 : 0;
  const int k = (int)inputs.size();
  for (int j = 0; j < k; ++j) {
    const at::Tensor& t = inputs[j];
    TORCH_CHECK(t.is_cuda() && t.device() == out.device() && t.is_contiguous() && t.numel() == n &&
                    t.scalar_type() == st_,
                "prereduce inputs must be contiguous tensors on out's device, of one dtype and out's numel");
    if ((uintptr_t)t.data_ptr() % 16) aligned = 0;
    a.in[j] = t.data_ptr();
  }
  if (n == 0) return;
  hipStream_t stream = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const float sc = (float)scale;
  switch (st_) {
    case at::kFloat: prereduce_dst<float>(out.scalar_type(), a, k, out.data_ptr(), n, sc, aligned, stream); break;
    case at::kBFloat16: prereduce_dst<bf16_t>(out.scalar_type(), a, k, out.data_ptr(), n, sc, aligned, stream); break;
    case at::kHalf: prereduce_dst<f16_t>(out.scalar_type(), a, k, out.data_ptr(), n, sc, aligned, stream); break;
    default: TORCH_CHECK(false, "nbd prereduce: unsupported input dtype ", st_);
  }
}

}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("bucket_flatten", &nbd::bucket_flatten_hip);
  m.impl("bucket_unflatten", &nbd::bucket_unflatten_hip);
  m.impl("local_prereduce", &nbd::local_prereduce_hip);
}
