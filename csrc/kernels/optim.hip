// optim.hip — fused AdamW over flat buffers (fp32 master weights, bf16/fp16/fp32 model params).
//
// Flat-buffer data parallelism (nbdistributed_amd.parallel.DistributedDataParallel with
// flat_params=True): every DDP bucket owns contiguous buffers in the same layout — the all-reduced
// gradient bucket (wire dtype), the model parameters (their dtype; the nn.Parameters are views),
// and fp32 master weights / exp_avg / exp_avg_sq.  One launch per bucket then performs the whole
// optimizer step as a single streaming pass:
//
//   g      = grad[i] * grad_scale [* *grad_scale_t]     (bucket is already averaged over ranks;
//                                                        grad_scale_t: on-device clip coefficient)
//   w      = master[i] * (1 - lr * weight_decay)        (decoupled weight decay, as torch AdamW)
//   m      = beta1 * m + (1 - beta1) * g
//   v      = beta2 * v + (1 - beta2) * g * g
//   w     -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
//   master[i] = w ; param[i] = cast(w)
//
// 28 bytes per parameter for bf16 params (read 2 + 12, write 12 + 2) instead of the eager chain
// (bf16->fp32 grad cast, unflatten, multi-tensor AdamW over fp32 params, fp32->bf16 weight cast in
// every autocast forward).  Pure HBM streaming: 16 B per lane per access, 8 elements per thread
// per thread, one thread per 8-element group (no grid-stride loop: measured 8 % faster than a
// 2048-block grid-stride, FINDINGS §31), non-temporal stores for the 16-bit param copy.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "nbd_common.h"

namespace nbd {

struct AdamArgs {
  float lr, beta1, beta2, eps, wd_factor, step_size, inv_sqrt_bc2, grad_scale, weight_decay;
};

// capturable mode (HIP graphs): step and lr come from device memory, so a replayed graph sees the
// current values; the bias corrections are recomputed per thread (two powf per thread)
__device__ __forceinline__ void device_hyper(AdamArgs& a, const float* dstep, const float* dlr) {
  if (dlr != nullptr) {
    a.lr = *dlr;
    a.wd_factor = 1.f - a.lr * a.weight_decay;
  }
  if (dstep != nullptr) {
    const float t = *dstep;
    a.step_size = a.lr / (1.f - powf(a.beta1, t));
    a.inv_sqrt_bc2 = rsqrtf(1.f - powf(a.beta2, t));
  }
}

// U = 8-element groups per thread per iteration (all their loads issued before any math: 112·U
// bytes in flight per lane); NTL = non-temporal loads (every byte is read once per step).
template <typename G, typename P, int U, bool NTL, bool NTS = false>
__global__ __launch_bounds__(256) void adamw_flat_kernel(const G* __restrict__ grad, P* __restrict__ param,
                                                         float* __restrict__ master, float* __restrict__ m,
                                                         float* __restrict__ v, const float* __restrict__ gscale,
                                                         const float* __restrict__ dstep,
                                                         const float* __restrict__ dlr, int64_t n, AdamArgs a) {
  if (gscale != nullptr) a.grad_scale *= *gscale;  // device-side clip coefficient (no host sync)
  device_hyper(a, dstep, dlr);
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * 256;
  const int64_t nv = n / 8;
  auto ld = [](auto* p, float (&x)[8]) {
    using T = std::remove_cv_t<std::remove_pointer_t<decltype(p)>>;
    if constexpr (NTL) load8_nt<T>(p, x);
    else load8<T>(p, x);
  };
  int64_t k = tid;
  for (; k + (U - 1) * nth < nv; k += U * nth) {
    float g[U][8], w[U][8], mm[U][8], vv[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = (k + u * nth) * 8;
      ld(grad + i, g[u]);
      ld(master + i, w[u]);
      ld(m + i, mm[u]);
      ld(v + i, vv[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = (k + u * nth) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gj = g[u][j] * a.grad_scale;
        mm[u][j] = fmaf(a.beta1, mm[u][j], (1.f - a.beta1) * gj);
        vv[u][j] = fmaf(a.beta2, vv[u][j], (1.f - a.beta2) * gj * gj);
        const float denom = sqrtf(vv[u][j]) * a.inv_sqrt_bc2 + a.eps;
        w[u][j] = w[u][j] * a.wd_factor - a.step_size * (mm[u][j] / denom);
      }
      if constexpr (NTS) {  // (variant 4: every stream non-temporal)
        store8_nt<float>(master + i, w[u]);
        store8_nt<float>(m + i, mm[u]);
        store8_nt<float>(v + i, vv[u]);
      } else {
        store8<float>(master + i, w[u]);
        store8<float>(m + i, mm[u]);
        store8<float>(v + i, vv[u]);
      }
      if (sizeof(P) == 2) store8_nt<P>(param + i, w[u]);
      else store8<P>(param + i, w[u]);
    }
  }
  for (; k < nv; k += nth) {  // (U > 1: the groups left over)
    const int64_t i = k * 8;
    float g[8], w[8], mm[8], vv[8];
    ld(grad + i, g);
    ld(master + i, w);
    ld(m + i, mm);
    ld(v + i, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gj = g[j] * a.grad_scale;
      mm[j] = fmaf(a.beta1, mm[j], (1.f - a.beta1) * gj);
      vv[j] = fmaf(a.beta2, vv[j], (1.f - a.beta2) * gj * gj);
      const float denom = sqrtf(vv[j]) * a.inv_sqrt_bc2 + a.eps;
      w[j] = w[j] * a.wd_factor - a.step_size * (mm[j] / denom);
    }
    store8<float>(master + i, w);
    store8<float>(m + i, mm);
    store8<float>(v + i, vv);
    if (sizeof(P) == 2) store8_nt<P>(param + i, w);
    else store8<P>(param + i, w);
  }
  for (int64_t i = nv * 8 + tid; i < n; i += nth) {
    const float gj = Elem<G>::load(grad, i) * a.grad_scale;
    float mm = fmaf(a.beta1, m[i], (1.f - a.beta1) * gj);
    float vv = fmaf(a.beta2, v[i], (1.f - a.beta2) * gj * gj);
    const float denom = sqrtf(vv) * a.inv_sqrt_bc2 + a.eps;
    const float w = master[i] * a.wd_factor - a.step_size * (mm / denom);
    m[i] = mm;
    v[i] = vv;
    master[i] = w;
    Elem<P>::store(param, i, w);
  }
}

// Every bucket of FlatAdamW's step in one launch (adamw_flat_multi): workgroup w updates 256
// 8-element groups of the bucket whose block range holds w (the last workgroup of a bucket also
// its < 8 trailing elements) — the per-element math of adamw_flat_kernel<.., 1, false>, so the
// update is bit-identical; one ramp and one tail instead of one per bucket.
constexpr int kMaxBuckets = 16;
template <typename G, typename P>
struct BucketTable {
  const G* grad[kMaxBuckets];
  P* param[kMaxBuckets];
  float* master[kMaxBuckets];
  float* m[kMaxBuckets];
  float* v[kMaxBuckets];
  int64_t n[kMaxBuckets];
  int block0[kMaxBuckets + 1];
};

template <typename G, typename P>
__global__ __launch_bounds__(256) void adamw_multi_kernel(BucketTable<G, P> t, int nb,
                                                          const float* __restrict__ gscale,
                                                          const float* __restrict__ dstep,
                                                          const float* __restrict__ dlr, AdamArgs a) {
  if (gscale != nullptr) a.grad_scale *= *gscale;
  device_hyper(a, dstep, dlr);
  const int blk = (int)blockIdx.x;
  int d = 0;  // block-uniform scan over <= 16 prefixes
  while (d + 1 < nb && t.block0[d + 1] <= blk) ++d;
  const int64_t n = t.n[d], nv = n / 8;
  const G* grad = t.grad[d];
  P* param = t.param[d];
  float *master = t.master[d], *m = t.m[d], *v = t.v[d];
  const int64_t k = (int64_t)(blk - t.block0[d]) * 256 + threadIdx.x;
  if (k < nv) {
    const int64_t i = k * 8;
    float g[8], w[8], mm[8], vv[8];
    load8<G>(grad + i, g);
    load8<float>(master + i, w);
    load8<float>(m + i, mm);
    load8<float>(v + i, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gj = g[j] * a.grad_scale;
      mm[j] = fmaf(a.beta1, mm[j], (1.f - a.beta1) * gj);
      vv[j] = fmaf(a.beta2, vv[j], (1.f - a.beta2) * gj * gj);
      const float denom = sqrtf(vv[j]) * a.inv_sqrt_bc2 + a.eps;
      w[j] = w[j] * a.wd_factor - a.step_size * (mm[j] / denom);
    }
    store8<float>(master + i, w);
    store8<float>(m + i, mm);
    store8<float>(v + i, vv);
    if (sizeof(P) == 2) store8_nt<P>(param + i, w);
    else store8<P>(param + i, w);
  }
  if (blk == t.block0[d + 1] - 1) {  // the bucket's trailing elements
    for (int64_t i = nv * 8 + threadIdx.x; i < n; i += 256) {
      const float gj = Elem<G>::load(grad, i) * a.grad_scale;
      const float mm = fmaf(a.beta1, m[i], (1.f - a.beta1) * gj);
      const float vv = fmaf(a.beta2, v[i], (1.f - a.beta2) * gj * gj);
      const float denom = sqrtf(vv) * a.inv_sqrt_bc2 + a.eps;
      const float w = master[i] * a.wd_factor - a.step_size * (mm / denom);
      m[i] = mm;
      v[i] = vv;
      master[i] = w;
      Elem<P>::store(param, i, w);
    }
  }
}

// NBD_ADAMW_BLOCKS (A/B): grid cap in workgroups (default none: one thread per 8-element group —
// 0.648 ms against 0.700 for the former 2048-block grid-stride default, 124 M parameters,
// profiles/adamw_grid_r5.txt);
// NBD_ADAMW_VARIANT: 1 = two 8-element groups per thread per iteration, 2 = that with
// non-temporal loads, 3 = one group with non-temporal loads (all measured slower: FINDINGS §31),
// 4 = one group with non-temporal stores
static int adamw_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e == nullptr ? dflt : std::atoi(e);
}

template <typename G, typename P>
static void launch_adamw(const at::Tensor& grad, const at::Tensor& param, const at::Tensor& master,
                         const at::Tensor& m, const at::Tensor& v, const float* gs, const float* dstep,
                         const float* dlr, int64_t n, const AdamArgs& a, hipStream_t st) {
  static const int cap = std::max(1, adamw_env("NBD_ADAMW_BLOCKS", 1 << 30));
  static const int variant = adamw_env("NBD_ADAMW_VARIANT", 0);
  const int64_t work = (n + 7) / 8;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, cap));
#define NBD_ADAMW(U_, NT_, ...)                                                                                   \
  hipLaunchKernelGGL((adamw_flat_kernel<G, P, U_, NT_, ##__VA_ARGS__>), dim3((unsigned)blocks), dim3(256), 0, st,  \
                     static_cast<const G*>(grad.data_ptr()), static_cast<P*>(param.data_ptr()), master.data_ptr<float>(), \
                     m.data_ptr<float>(), v.data_ptr<float>(), gs, dstep, dlr, n, a)
  switch (variant) {
    case 1: NBD_ADAMW(2, false); break;
    case 2: NBD_ADAMW(2, true); break;
    case 3: NBD_ADAMW(1, true); break;
    case 4: NBD_ADAMW(1, false, true); break;
    default: NBD_ADAMW(1, false); break;
  }
#undef NBD_ADAMW
  C10_HIP_KERNEL_LAUNCH_CHECK();
}

template <typename G>
static void dispatch_param(const at::Tensor& grad, const at::Tensor& param, const at::Tensor& master,
                           const at::Tensor& m, const at::Tensor& v, const float* gs, const float* dstep,
                           const float* dlr, int64_t n, const AdamArgs& a, hipStream_t st) {
  switch (param.scalar_type()) {
    case at::kFloat: launch_adamw<G, float>(grad, param, master, m, v, gs, dstep, dlr, n, a, st); break;
    case at::kBFloat16: launch_adamw<G, bf16_t>(grad, param, master, m, v, gs, dstep, dlr, n, a, st); break;
    case at::kHalf: launch_adamw<G, f16_t>(grad, param, master, m, v, gs, dstep, dlr, n, a, st); break;
    default: TORCH_CHECK(false, "adamw_flat: unsupported param dtype ", param.scalar_type());
  }
}

void adamw_flat_hip(const at::Tensor& grad, const at::Tensor& param, const at::Tensor& master, const at::Tensor& exp_avg,
                    const at::Tensor& exp_avg_sq, double lr, double beta1, double beta2, double eps,
                    double weight_decay, int64_t step, double grad_scale,
                    const c10::optional<at::Tensor>& grad_scale_t, const c10::optional<at::Tensor>& step_t,
                    const c10::optional<at::Tensor>& lr_t) {
  TORCH_CHECK(grad.is_cuda() && param.is_cuda() && master.is_cuda() && exp_avg.is_cuda() && exp_avg_sq.is_cuda(),
              "adamw_flat: GPU tensors expected");
  TORCH_CHECK(grad.is_contiguous() && param.is_contiguous() && master.is_contiguous() && exp_avg.is_contiguous() &&
                  exp_avg_sq.is_contiguous(),
              "adamw_flat: contiguous (flat) buffers expected");
  TORCH_CHECK(master.scalar_type() == at::kFloat && exp_avg.scalar_type() == at::kFloat &&
                  exp_avg_sq.scalar_type() == at::kFloat,
              "adamw_flat: master / exp_avg / exp_avg_sq must be float32");
  const int64_t n = param.numel();
  TORCH_CHECK(grad.numel() >= n && master.numel() == n && exp_avg.numel() == n && exp_avg_sq.numel() == n,
              "adamw_flat: buffer sizes disagree");
  TORCH_CHECK(step >= 1, "adamw_flat: step counts from 1");
  for (const at::Tensor* t : {&grad, &param, &master, &exp_avg, &exp_avg_sq})
    TORCH_CHECK((uintptr_t)t->data_ptr() % 16 == 0, "adamw_flat: buffers must be 16-byte aligned");
  const float* gs = nullptr;
  if (grad_scale_t.has_value() && grad_scale_t->defined()) {
    TORCH_CHECK(grad_scale_t->is_cuda() && grad_scale_t->scalar_type() == at::kFloat && grad_scale_t->numel() == 1,
                "adamw_flat: grad_scale_t must be a 1-element float32 GPU tensor");
    gs = grad_scale_t->data_ptr<float>();
  }
  auto dev_scalar = [&](const c10::optional<at::Tensor>& t, const char* name) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() == 1, "adamw_flat: ", name,
                " must be a 1-element float32 GPU tensor");
    return t->data_ptr<float>();
  };
  const float* dstep = dev_scalar(step_t, "step_t");
  const float* dlr = dev_scalar(lr_t, "lr_t");
  TORCH_CHECK((dstep == nullptr) == (dlr == nullptr), "adamw_flat: step_t and lr_t go together (capturable mode)");
  if (n == 0) return;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(param.device());
  AdamArgs a;
  a.weight_decay = (float)weight_decay;
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.wd_factor = (float)(1.0 - lr * weight_decay);
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  a.step_size = (float)(lr / bc1);
  a.inv_sqrt_bc2 = (float)(1.0 / std::sqrt(bc2));
  a.grad_scale = (float)grad_scale;
  hipStream_t stream = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  switch (grad.scalar_type()) {
    case at::kFloat: dispatch_param<float>(grad, param, master, exp_avg, exp_avg_sq, gs, dstep, dlr, n, a, stream); break;
    case at::kBFloat16: dispatch_param<bf16_t>(grad, param, master, exp_avg, exp_avg_sq, gs, dstep, dlr, n, a, stream); break;
    case at::kHalf: dispatch_param<f16_t>(grad, param, master, exp_avg, exp_avg_sq, gs, dstep, dlr, n, a, stream); break;
    default: TORCH_CHECK(false, "adamw_flat: unsupported grad dtype ", grad.scalar_type());
  }
}

// ---- per-parameter AdamW over a tensor list (torch.optim.AdamW's state layout) ----------------
// The one-line HF swap (models.native) keeps HF's fp32 parameters and the notebook's own
// torch.optim.AdamW: its fused implementation runs the update as several chunked launches
// (0.92 ms per SmolLM2 step, profiles/hfnative_prof_r5final.md).  Here: one launch per <= 128
// tensors — the table (pointers, sizes, chunk prefix; ≈7.7 KiB) travels in the kernel arguments
// as bucket.hip's multi_copy does — 8 Ki-element chunks, 16 B per lane per access, each
// tensor's own device-side step count (torch keeps one per parameter) read once per workgroup.
// Math in torch's fused AdamW order: decoupled decay, moments, bias corrections from the step,
// denom = sqrt(v) / sqrt(bc2) + eps.
constexpr int kAT = 128;
constexpr int64_t kAChunk = 8192;
constexpr int kAHint = 1024;

struct AdamTable {
  float* p[kAT];
  const float* g[kAT];
  float* m[kAT];
  float* v[kAT];
  const float* step[kAT];
  int64_t numel[kAT];
  int32_t chunk_prefix[kAT + 1];
  int32_t group_chunks;
  uint8_t hint[kAHint];
  uint64_t aligned_mask[kAT / 64];
};

__device__ __forceinline__ void adamw_elem(float& w, float& mm, float& vv, float g, float lr_wd, float b1, float b2,
                                           float step_size, float sqrt_bc2, float eps) {
  w -= lr_wd * w;
  mm = b1 * mm + (1.f - b1) * g;
  vv = b2 * vv + (1.f - b2) * g * g;
  const float denom = sqrtf(vv) / sqrt_bc2 + eps;
  w -= step_size * mm / denom;
}

__global__ __launch_bounds__(256) void adamw_tensors_kernel(AdamTable tab, int nt, float lr, float b1, float b2,
                                                            float eps, float wd) {
  const int chunk = blockIdx.x;
  int t = tab.hint[chunk / tab.group_chunks];
  while (t + 1 < nt && tab.chunk_prefix[t + 1] <= chunk) ++t;
  const int64_t begin = (int64_t)(chunk - tab.chunk_prefix[t]) * kAChunk;
  const int64_t end = min(begin + kAChunk, tab.numel[t]);
  const float stepv = *tab.step[t];
  const float step_size = lr / (1.f - powf(b1, stepv));
  const float sqrt_bc2 = sqrtf(1.f - powf(b2, stepv));
  const float lr_wd = lr * wd;
  float* __restrict__ P = tab.p[t];
  const float* __restrict__ G = tab.g[t];
  float* __restrict__ M = tab.m[t];
  float* __restrict__ V = tab.v[t];
  if ((tab.aligned_mask[t >> 6] >> (t & 63)) & 1ull) {
    int64_t i = begin + (int64_t)threadIdx.x * 8;
    for (; i + 8 <= end; i += 256 * 8) {
      float g[8], w[8], mm[8], vv[8];
      load8<float>(G + i, g);
      load8<float>(P + i, w);
      load8<float>(M + i, mm);
      load8<float>(V + i, vv);
#pragma unroll
      for (int j = 0; j < 8; ++j) adamw_elem(w[j], mm[j], vv[j], g[j], lr_wd, b1, b2, step_size, sqrt_bc2, eps);
      store8<float>(P + i, w);
      store8<float>(M + i, mm);
      store8<float>(V + i, vv);
    }
    for (int64_t k = i; k < end && k < i + 8; ++k)  // < 8 trailing elements (the tensor's last chunk)
      adamw_elem(P[k], M[k], V[k], G[k], lr_wd, b1, b2, step_size, sqrt_bc2, eps);
  } else {
    for (int64_t k = begin + threadIdx.x; k < end; k += 256)
      adamw_elem(P[k], M[k], V[k], G[k], lr_wd, b1, b2, step_size, sqrt_bc2, eps);
  }
}

void adamw_tensors_hip(at::TensorList params, at::TensorList grads, at::TensorList exp_avgs,
                       at::TensorList exp_avg_sqs, at::TensorList steps, double lr, double beta1, double beta2,
                       double eps, double weight_decay) {
  const size_t n = params.size();
  TORCH_CHECK(grads.size() == n && exp_avgs.size() == n && exp_avg_sqs.size() == n && steps.size() == n,
              "adamw_tensors: one grad, exp_avg, exp_avg_sq and step per parameter");
  if (n == 0) return;
  for (size_t i = 0; i < n; ++i) {
    const int64_t k = params[i].numel();
    for (const at::Tensor* x : {&params[i], &grads[i], &exp_avgs[i], &exp_avg_sqs[i]})
      TORCH_CHECK(x->is_cuda() && x->scalar_type() == at::kFloat && x->is_contiguous() && x->numel() == k &&
                      x->device() == params[0].device(),
                  "adamw_tensors: contiguous float32 GPU parameter / grad / moments of equal size");
    TORCH_CHECK(steps[i].is_cuda() && steps[i].scalar_type() == at::kFloat && steps[i].numel() == 1,
                "adamw_tensors: each step count is a 1-element float32 GPU tensor");
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(params[0].device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  size_t pos = 0;
  while (pos < n) {
    AdamTable tab{};
    int nt = 0;
    int64_t chunks = 0;
    for (; pos < n && nt < kAT; ++pos) {
      const int64_t k = params[pos].numel();
      if (k == 0) continue;
      const int64_t c = (k + kAChunk - 1) / kAChunk;
      if (chunks + c > (int64_t)INT32_MAX / 2 && nt > 0) break;
      tab.p[nt] = params[pos].data_ptr<float>();
      tab.g[nt] = grads[pos].data_ptr<float>();
      tab.m[nt] = exp_avgs[pos].data_ptr<float>();
      tab.v[nt] = exp_avg_sqs[pos].data_ptr<float>();
      tab.step[nt] = steps[pos].data_ptr<float>();
      tab.numel[nt] = k;
      tab.chunk_prefix[nt] = (int32_t)chunks;
      bool al = true;
      for (const void* ptr : {(const void*)tab.p[nt], (const void*)tab.g[nt], (const void*)tab.m[nt],
                              (const void*)tab.v[nt]})
        al = al && ((uintptr_t)ptr % 16 == 0);
      if (al) tab.aligned_mask[nt >> 6] |= 1ull << (nt & 63);
      chunks += c;
      ++nt;
    }
    if (nt == 0) continue;
    tab.chunk_prefix[nt] = (int32_t)chunks;
    tab.group_chunks = (int32_t)std::max<int64_t>(1, (chunks + kAHint - 1) / kAHint);
    for (int h = 0, t = 0; h < kAHint; ++h) {
      const int64_t first = (int64_t)h * tab.group_chunks;
      while (t + 1 < nt && tab.chunk_prefix[t + 1] <= first) ++t;
      tab.hint[h] = (uint8_t)t;
    }
    hipLaunchKernelGGL(adamw_tensors_kernel, dim3((unsigned)chunks), dim3(256), 0, st, tab, nt, (float)lr,
                       (float)beta1, (float)beta2, (float)eps, (float)weight_decay);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
}

// All buckets in one adamw_multi_kernel launch when they allow it (<= 16 buckets, one gradient and
// one parameter dtype, the default kernel variant); false: the caller loops over adamw_flat_hip,
// which also validates every buffer.  NBD_ADAMW_MULTI=0 (A/B).
static bool multi_launch(at::TensorList grads, at::TensorList params, at::TensorList masters, at::TensorList exp_avgs,
                         at::TensorList exp_avg_sqs, double lr, double beta1, double beta2, double eps,
                         double weight_decay, int64_t step, double grad_scale,
                         const c10::optional<at::Tensor>& grad_scale_t, const c10::optional<at::Tensor>& step_t,
                         const c10::optional<at::Tensor>& lr_t) {
  static const bool on = [] {
    const char* e = std::getenv("NBD_ADAMW_MULTI");
    return e == nullptr || e[0] != '0';
  }();
  const size_t nb = params.size();
  if (!on || nb < 2 || nb > (size_t)kMaxBuckets || adamw_env("NBD_ADAMW_VARIANT", 0) != 0 ||
      adamw_env("NBD_ADAMW_BLOCKS", 0) > 0 || step < 1)
    return false;
  const auto gt = grads[0].scalar_type(), pt = params[0].scalar_type();
  for (size_t i = 0; i < nb; ++i) {
    const at::Tensor* ts[5] = {&grads[i], &params[i], &masters[i], &exp_avgs[i], &exp_avg_sqs[i]};
    for (const at::Tensor* t : ts)
      if (!t->is_cuda() || !t->is_contiguous() || (uintptr_t)t->data_ptr() % 16 != 0 ||
          t->device() != params[0].device())
        return false;
    const int64_t n = params[i].numel();
    if (grads[i].scalar_type() != gt || params[i].scalar_type() != pt || masters[i].scalar_type() != at::kFloat ||
        exp_avgs[i].scalar_type() != at::kFloat || exp_avg_sqs[i].scalar_type() != at::kFloat ||
        grads[i].numel() < n || masters[i].numel() != n || exp_avgs[i].numel() != n || exp_avg_sqs[i].numel() != n ||
        n == 0)
      return false;
  }
  auto dev_scalar = [](const c10::optional<at::Tensor>& t) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() == 1,
                "adamw_flat_multi: step_t / lr_t / grad_scale_t must be 1-element float32 GPU tensors");
    return t->data_ptr<float>();
  };
  const float* gs = dev_scalar(grad_scale_t);
  const float* dstep = dev_scalar(step_t);
  const float* dlr = dev_scalar(lr_t);
  TORCH_CHECK((dstep == nullptr) == (dlr == nullptr), "adamw_flat_multi: step_t and lr_t go together (capturable mode)");
  AdamArgs a;
  a.weight_decay = (float)weight_decay;
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.wd_factor = (float)(1.0 - lr * weight_decay);
  a.step_size = (float)(lr / (1.0 - std::pow(beta1, (double)step)));
  a.inv_sqrt_bc2 = (float)(1.0 / std::sqrt(1.0 - std::pow(beta2, (double)step)));
  a.grad_scale = (float)grad_scale;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(params[0].device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  bool done = false;
  auto go = [&](auto gtag, auto ptag) {
    using G = decltype(gtag);
    using P = decltype(ptag);
    BucketTable<G, P> t{};
    int blocks = 0;
    for (size_t i = 0; i < nb; ++i) {
      t.grad[i] = static_cast<const G*>(grads[i].data_ptr());
      t.param[i] = static_cast<P*>(params[i].data_ptr());
      t.master[i] = masters[i].data_ptr<float>();
      t.m[i] = exp_avgs[i].data_ptr<float>();
      t.v[i] = exp_avg_sqs[i].data_ptr<float>();
      t.n[i] = params[i].numel();
      t.block0[i] = blocks;
      const int64_t nbk = std::max<int64_t>(1, (t.n[i] / 8 + 255) / 256);
      TORCH_CHECK(blocks + nbk < (int64_t)INT32_MAX / 2, "adamw_flat_multi: too many workgroups");
      blocks += (int)nbk;
    }
    t.block0[nb] = blocks;
    hipLaunchKernelGGL((adamw_multi_kernel<G, P>), dim3((unsigned)blocks), dim3(256), 0, st, t, (int)nb, gs, dstep,
                       dlr, a);
    C10_HIP_KERNEL_LAUNCH_CHECK();
    done = true;
  };
  auto by_p = [&](auto gtag) {
    switch (pt) {
      case at::kFloat: go(gtag, float{}); break;
      case at::kBFloat16: go(gtag, bf16_t{}); break;
      case at::kHalf: go(gtag, f16_t{}); break;
      default: break;
    }
  };
  switch (gt) {
    case at::kFloat: by_p(float{}); break;
    case at::kBFloat16: by_p(bf16_t{}); break;
    case at::kHalf: by_p(f16_t{}); break;
    default: break;
  }
  return done;
}

// Every bucket's update from one call (FlatAdamW.step's fast path): the same per-bucket kernels
// in bucket order, without a Python round trip and an op dispatch per bucket (an eager small-model
// step is host-bound: docs/FINDINGS.md §27).
void adamw_flat_multi_hip(at::TensorList grads, at::TensorList params, at::TensorList masters, at::TensorList exp_avgs,
                          at::TensorList exp_avg_sqs, double lr, double beta1, double beta2, double eps,
                          double weight_decay, int64_t step, double grad_scale,
                          const c10::optional<at::Tensor>& grad_scale_t, const c10::optional<at::Tensor>& step_t,
                          const c10::optional<at::Tensor>& lr_t) {
  const size_t n = params.size();
  TORCH_CHECK(grads.size() == n && masters.size() == n && exp_avgs.size() == n && exp_avg_sqs.size() == n,
              "adamw_flat_multi: one gradient, master, exp_avg and exp_avg_sq per parameter buffer");
  if (multi_launch(grads, params, masters, exp_avgs, exp_avg_sqs, lr, beta1, beta2, eps, weight_decay, step,
                   grad_scale, grad_scale_t, step_t, lr_t))
    return;
  for (size_t i = 0; i < n; ++i)
    adamw_flat_hip(grads[i], params[i], masters[i], exp_avgs[i], exp_avg_sqs[i], lr, beta1, beta2, eps, weight_decay,
                   step, grad_scale, grad_scale_t, step_t, lr_t);
}

}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("adamw_flat", &nbd::adamw_flat_hip);
  m.impl("adamw_flat_multi", &nbd::adamw_flat_multi_hip);
  m.impl("adamw_tensors", &nbd::adamw_tensors_hip);
}
