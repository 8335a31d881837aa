// mask.hip — padding-mask preparation for the fused sequence-classification path (K15).
//
// HF ``LlamaForSequenceClassification.forward(input_ids, attention_mask)`` masks padded keys in
// every attention layer and pools the rightmost non-pad token.  The fused decoder path runs causal
// flash attention without a key mask, which is exact for RIGHT-padded rows (a real query never
// sees a later pad key).  A left-padded row is made right-padded by rotating it left by its pad
// count: RoPE attention scores depend only on position differences, so every real token's
// attention (and everything after it) is unchanged, and the pooled token is re-indexed into the
// rotated row.  One launch does all of it (the notebook step is
// host-bound: five torch ops would cost five launches; one wave per row):
//
//   off  = first position with mask != 0 (0 for an all-zero row)
//   ids_out[b, j] = ids[b, (j + off) mod T]
//   pool[b] = (last non-pad position of the ORIGINAL row (HF's rule) - off) mod T
//   bad |= 1 if the row's mask is not one contiguous run (holes: no rotation makes it causal-exact),
//          2 if the row is not right-padded (the causal LM, which keeps positions, needs that)
//
// `bad` is read lazily by the caller (models/llama.py _MaskCheck: pinned copy + event, no sync).
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPException.h>
#include <torch/library.h>

#include "nbd_common.h"

namespace nbd {
namespace mask {

constexpr int kThreads = 256;  // 4 waves = 4 rows per workgroup; one wave per row

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// One wave per row: the row's statistics are wave reductions (cross-lane shuffles, no LDS, no
// barrier), so a batch of short rows costs one launch's latency and nothing more.
template <typename M>
__global__ __launch_bounds__(kThreads) void seqcls_prep_kernel(const int64_t* __restrict__ ids,
                                                               const M* __restrict__ mask, int64_t B, int64_t T,
                                                               int64_t pad_id, int has_pad, int64_t* __restrict__ ids_out,
                                                               int64_t* __restrict__ pool, int32_t* __restrict__ bad) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (b >= B) return;  // (wave-uniform)
  const int64_t* row = ids + b * T;
  int first = (int)T, last = -1, cnt = 0, lastnp = -1;
  for (int64_t j = lane; j < T; j += 64) {
    const bool on = mask == nullptr || mask[b * T + j] != M(0);
    if (on) {
      first = min(first, (int)j);
      last = max(last, (int)j);
      ++cnt;
    }
    if (!has_pad || row[j] != pad_id) lastnp = max(lastnp, (int)j);
  }
  first = wave_min(first);
  last = wave_max(last);
  cnt = wave_sum(cnt);
  lastnp = wave_max(lastnp);
  const int64_t off = cnt == 0 ? 0 : first;
  for (int64_t j = lane; j < T; j += 64) {
    int64_t src = j + off;
    if (src >= T) src -= T;
    ids_out[b * T + j] = row[src];
  }
  if (lane == 0) {
    // HF: argmax(arange · non-pad) — the last non-pad position, 0 when the row is all pad
    const int64_t np = lastnp < 0 ? 0 : lastnp;
    pool[b] = (np - off + T) % T;
    int flag = 0;
    if (cnt != 0 && last - first + 1 != cnt) flag |= 1;  // holes
    if (cnt != 0 && first != 0) flag |= 2;               // not right-padded
    if (flag) atomicOr(bad, flag);
  }
}

// (ids_out [B, T] int64, pool [B] int64); ORs 1 into bad[0] for a mask with holes
std::tuple<at::Tensor, at::Tensor> seqcls_prep_hip(const at::Tensor& ids, const c10::optional<at::Tensor>& mask,
                                                   int64_t pad_id, bool has_pad, at::Tensor bad) {
  TORCH_CHECK(ids.is_cuda() && ids.dim() == 2 && ids.scalar_type() == at::kLong && ids.is_contiguous(),
              "seqcls_prep: input_ids must be a contiguous int64 [B, T] GPU tensor");
  TORCH_CHECK(bad.is_cuda() && bad.scalar_type() == at::kInt && bad.numel() >= 1, "seqcls_prep: bad must be int32");
  const int64_t B = ids.size(0), T = ids.size(1);
  auto ids_out = at::empty_like(ids);
  auto pool = at::empty({B}, ids.options());
  if (B == 0 || T == 0) return {ids_out, pool};
  const hipStream_t st = at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const dim3 grid((unsigned)((B + kThreads / 64 - 1) / (kThreads / 64))), block(kThreads);
  auto launch = [&](auto tag, const at::Tensor* m) {
    using M = decltype(tag);
    hipLaunchKernelGGL((seqcls_prep_kernel<M>), grid, block, 0, st, ids.data_ptr<int64_t>(),
                       m ? static_cast<const M*>(m->data_ptr()) : nullptr, B, T, pad_id, has_pad ? 1 : 0,
                       ids_out.data_ptr<int64_t>(), pool.data_ptr<int64_t>(), bad.data_ptr<int32_t>());
  };
  if (!mask || !mask->defined()) {
    launch(int64_t{}, nullptr);
  } else {
    const at::Tensor m = mask->contiguous();
    TORCH_CHECK(m.is_cuda() && m.sizes() == ids.sizes(), "seqcls_prep: attention_mask must match input_ids");
    switch (m.scalar_type()) {
      case at::kLong: launch(int64_t{}, &m); break;
      case at::kInt: launch(int32_t{}, &m); break;
      case at::kBool:
      case at::kByte: launch(uint8_t{}, &m); break;
      default: TORCH_CHECK(false, "seqcls_prep: unsupported attention_mask dtype ", m.scalar_type());
    }
  }
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {ids_out, pool};
}

}  // namespace mask
}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) { m.impl("seqcls_prep", &nbd::mask::seqcls_prep_hip); }
