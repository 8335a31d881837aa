// ring.hip — log-sum-exp merge of flash-attention blocks for ring (context-parallel) attention, gfx950.
//
// parallel/context.py runs one nbd::attn_fwd per (query chunk, key/value chunk) block; each block
// returns o_b (bf16, any [B, H, T, 64] view the attention kernels write) and lse_b (fp32 [B, H, T]).
// Rows are merged exactly:  l = log(e^la + e^lb),  o = o_acc·e^(la−l) + o_b·e^(lb−l).
// As eager PyTorch that is ~8 kernels over fp32 [B, H, T, 64] tensors per block; here it is one
// pass: 8 lanes per row, 8 elements (one 16-B bf16 / two 16-B fp32 vectors) per lane, the row's two
// LSEs read once per lane (L1-broadcast).  With `out` given (the row's last block) the merged row
// is written straight to the bf16 output view and the fp32 accumulator is left untouched.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>

#include "nbd_common.h"

namespace nbd {
namespace ring {

constexpr int NT = 256;
constexpr int D = 64;

struct BView {  // bf16 [B, H, T, 64] view, unit stride in the last dim
  uint16_t* p;
  int64_t sb, sh, st;
};

__global__ __launch_bounds__(NT) void merge_kernel(float* __restrict__ acc, float* __restrict__ lacc, BView ob,
                                                   const float* __restrict__ lb, BView out, int write_out, int H,
                                                   int T, int64_t units) {
  for (int64_t u = (int64_t)blockIdx.x * NT + threadIdx.x; u < units; u += (int64_t)gridDim.x * NT) {
    const int64_t row = u >> 3;
    const int d8 = (int)(u & 7);
    const int t = (int)(row % T), h = (int)(row / T % H), b = (int)(row / T / H);
    const float la = lacc[row], lbb = lb[row];
    const float m = fmaxf(la, lbb);
    const float l = m + __logf(__expf(la - m) + __expf(lbb - m));
    const float wa = __expf(la - l), wb = __expf(lbb - l);
    float a[8], x[8];
    load8<float>(acc + row * D + d8 * 8, a);
    load8<bf16_t>(reinterpret_cast<const bf16_t*>(ob.p + b * ob.sb + h * ob.sh + t * ob.st + d8 * 8), x);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = a[e] * wa + x[e] * wb;
    if (write_out)
      store8<bf16_t>(reinterpret_cast<bf16_t*>(out.p + b * out.sb + h * out.sh + t * out.st + d8 * 8), a);
    else
      store8<float>(acc + row * D + d8 * 8, a);
    if (d8 == 0) lacc[row] = l;
  }
}

static BView bview_of(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 4 && t.size(3) == D && t.stride(3) == 1 && t.scalar_type() == at::kBFloat16,
              "attn_merge_: ", name, " must be a bf16 [B, H, T, 64] GPU view with a contiguous last dim");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0 && ((uintptr_t)t.data_ptr() & 15) == 0,
              "attn_merge_: ", name, " strides must be multiples of 8 elements and its base 16-B aligned");
  return BView{static_cast<uint16_t*>(t.data_ptr()), t.stride(0), t.stride(1), t.stride(2)};
}

void attn_merge_hip(const at::Tensor& acc, const at::Tensor& lacc, const at::Tensor& ob, const at::Tensor& lb,
                    const c10::optional<at::Tensor>& out) {
  TORCH_CHECK(acc.is_cuda() && acc.scalar_type() == at::kFloat && acc.is_contiguous() && acc.dim() == 4 &&
                  acc.size(3) == D,
              "attn_merge_: o_acc must be a contiguous float32 [B, H, T, 64]");
  const int B = acc.size(0), H = acc.size(1), T = acc.size(2);
  const int64_t rows = (int64_t)B * H * T;
  for (const at::Tensor* l : {&lacc, &lb})
    TORCH_CHECK(l->is_cuda() && l->scalar_type() == at::kFloat && l->is_contiguous() && l->numel() == rows,
                "attn_merge_: lse tensors must be contiguous float32 [B, H, T]");
  TORCH_CHECK(ob.sizes() == acc.sizes(), "attn_merge_: o_b shape mismatch");
  const BView obv = bview_of(ob, "o_b");
  BView outv{nullptr, 0, 0, 0};
  if (out.has_value()) {
    TORCH_CHECK(out->sizes() == acc.sizes(), "attn_merge_: out shape mismatch");
    outv = bview_of(*out, "out");
  }
  const int64_t units = rows * (D / 8);
  if (units == 0) return;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(acc.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((units + NT - 1) / NT, 8192));
  hipLaunchKernelGGL(merge_kernel, dim3(grid), dim3(NT), 0, st, acc.data_ptr<float>(), lacc.data_ptr<float>(), obv,
                     lb.data_ptr<float>(), outv, out.has_value() ? 1 : 0, H, T, units);
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

}  // namespace ring
}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) { m.impl("attn_merge_", &nbd::ring::attn_merge_hip); }
