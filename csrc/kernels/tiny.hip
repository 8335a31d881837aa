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

// ---- sequence-classification head: pooled row -> score -> mean cross-entropy, fused ----------
// HF's LlamaForSequenceClassification tail (the notebook's model): pooled = h[b, last[b]],
// logits = pooled·Wᵀ (N labels), loss = mean over non-ignored rows of CE(logits.float(), label).
// Torch ran it as gather, the head, a cast, log-softmax, NLL (+ fills) and, backward, NLL′,
// log-softmax′, a cast, the head's backward, a zero fill of dh and a scatter: ≈ 14 launches per
// step.  Here: one forward launch (one workgroup: B ≤ 64 rows) and one backward launch.
constexpr int SQ_NT = 1024;

// the pooled position of row b, clamped into the row (ops.seqcls_prep always yields one inside)
__device__ __forceinline__ int64_t pooled_t(const int64_t* last, int b, int T) {
  const int64_t t = last[b];
  return t < 0 ? 0 : (t >= T ? T - 1 : t);
}

// forward: logits [B, N] (bf16, rounded once as F.linear's output), the loss, and
// dl[b, n] = (softmax − onehot) / #valid (fp32; 0 on ignored rows) for the backward
__global__ __launch_bounds__(SQ_NT) void seqcls_fwd_kernel(const uint16_t* __restrict__ h, const int64_t* __restrict__ last,
                                                           int T, const uint16_t* __restrict__ w,
                                                           const int64_t* __restrict__ labels, int64_t ignore, int B,
                                                           int N, int K, uint16_t* __restrict__ logits,
                                                           float* __restrict__ dl, float* __restrict__ loss) {
  __shared__ float lg[64 * 64];
  __shared__ float rl[64], rv[64], cnt_s;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int o = wave; o < B * N; o += SQ_NT / 64) {  // one wave per (row, label): lanes over K
    const int b = o / N, n = o % N;
    const uint16_t* xr = h + ((int64_t)b * T + pooled_t(last, b, T)) * K;
    const uint16_t* wr = w + (int64_t)n * K;
    float acc = 0.f;
    for (int k = lane * 8; k < K; k += 64 * 8) {
      float a[8], c[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(xr + k), a);
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(wr + k), c);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc = fmaf(a[e], c[e], acc);
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) acc += __shfl_xor(acc, s, 64);
    if (lane == 0) {
      const uint16_t r = f32_to_bf16(acc);
      logits[o] = r;
      lg[o] = bf16_to_f32(r);
    }
  }
  __syncthreads();
  if (threadIdx.x < B) {  // one thread per row: log-softmax over the N labels
    const int b = threadIdx.x;
    float mx = -INFINITY;
    for (int n = 0; n < N; ++n) mx = fmaxf(mx, lg[b * N + n]);
    float se = 0.f;
    for (int n = 0; n < N; ++n) se += expf(lg[b * N + n] - mx);
    const float lse = mx + logf(se);
    const int64_t y = labels[b];
    const bool valid = y != ignore;
    // (an out-of-range label: NaN loss rather than a fault; torch raises a device assert)
    const bool inr = valid && y >= 0 && y < N;
    rl[b] = valid ? (inr ? lse - lg[b * N + y] : NAN) : 0.f;
    rv[b] = valid ? 1.f : 0.f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f, cnt = 0.f;
    for (int b = 0; b < B; ++b) {
      tot += rl[b];
      cnt += rv[b];
    }
    loss[0] = tot / cnt;  // 0 / 0 = nan when every row is ignored (as torch)
    cnt_s = cnt;
  }
  __syncthreads();
  const float cnt = cnt_s;
  if (threadIdx.x < B * N) {
    const int b = threadIdx.x / N, n = threadIdx.x % N;
    float mx = -INFINITY;
    for (int j = 0; j < N; ++j) mx = fmaxf(mx, lg[b * N + j]);
    float se = 0.f;
    for (int j = 0; j < N; ++j) se += expf(lg[b * N + j] - mx);
    const int64_t y = labels[b];
    const float p = expf(lg[b * N + n] - mx) / se;
    dl[b * N + n] = y != ignore ? (p - (n == y ? 1.f : 0.f)) / cnt : 0.f;
  }
}

// backward: d = dl·g (+ glog, a gradient arriving at the logits); blocks [0, bh): dh [B, T, K]
// (zero except row last[b], which gets Σ_n d[b, n]·W[n]), blocks [bh, bh + bw): dW [N, K]
// (= Σ_b d[b, n]·h[b, last[b]]; += into dw with accumulate)
__global__ __launch_bounds__(256) void seqcls_bwd_kernel(const uint16_t* __restrict__ h, const int64_t* __restrict__ last,
                                                         int T, const uint16_t* __restrict__ w,
                                                         const float* __restrict__ dl, const float* __restrict__ g,
                                                         const uint16_t* __restrict__ glog, int B, int N, int K,
                                                         uint16_t* __restrict__ dh, uint16_t* __restrict__ dw,
                                                         int accumulate, int bh) {
  const float gs = g != nullptr ? g[0] : 1.f;
  auto d = [&](int b, int n) {
    float v = dl[b * N + n] * gs;
    if (glog != nullptr) v += bf16_to_f32(glog[b * N + n]);
    return v;
  };
  const int K8 = K / 8;
  if ((int)blockIdx.x < bh) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)B * T * K8) return;
    const int c = (int)(i % K8) * 8;
    const int64_t bt = i / K8;
    const int b = (int)(bt / T), t = (int)(bt % T);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (t == pooled_t(last, b, T)) {
      for (int n = 0; n < N; ++n) {
        const float dv = d(b, n);
        float v[8];
        load8<bf16_t>(reinterpret_cast<const bf16_t*>(w + (int64_t)n * K + c), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(dv, v[e], acc[e]);
      }
    }
    store8<bf16_t>(reinterpret_cast<bf16_t*>(dh + bt * K + c), acc);
  } else {
    const int64_t i = (int64_t)(blockIdx.x - bh) * 256 + threadIdx.x;
    if (i >= (int64_t)N * K8) return;
    const int n = (int)(i / K8), c = (int)(i % K8) * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = 0; b < B; ++b) {
      const float dv = d(b, n);
      float v[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(h + ((int64_t)b * T + pooled_t(last, b, T)) * K + c), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(dv, v[e], acc[e]);
    }
    uint16_t* o = dw + (int64_t)n * K + c;
    if (accumulate) {
      float v[8];
      load8<bf16_t>(reinterpret_cast<const bf16_t*>(o), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
    store8<bf16_t>(reinterpret_cast<bf16_t*>(o), acc);
  }
}

static void check_seqcls(const at::Tensor& h, const at::Tensor& last, const at::Tensor& w) {
  TORCH_CHECK(h.is_cuda() && h.dim() == 3 && h.is_contiguous() && h.scalar_type() == at::kBFloat16,
              "seqcls_head: h must be a contiguous bf16 [B, T, C] GPU tensor");
  TORCH_CHECK(w.is_cuda() && w.dim() == 2 && w.is_contiguous() && w.scalar_type() == at::kBFloat16 && w.size(1) == h.size(2),
              "seqcls_head: w must be a contiguous bf16 [N, C] GPU tensor");
  TORCH_CHECK(h.size(0) >= 1 && h.size(0) <= 64 && w.size(0) >= 1 && w.size(0) <= 64 && h.size(0) * w.size(0) <= SQ_NT &&
                  h.size(2) % 8 == 0,
              "seqcls_head: 1 <= B <= 64 rows, 1 <= N <= 64 labels (B·N <= 1024), C % 8 == 0");
  TORCH_CHECK(last.is_cuda() && last.scalar_type() == at::kLong && last.is_contiguous() && last.numel() == h.size(0),
              "seqcls_head: last must be int64 [B]");
  TORCH_CHECK(h.numel() < (1LL << 40), "seqcls_head: too large");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(h.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "seqcls_head: 16-byte aligned operands");
}

// (loss [], logits [B, N] bf16, dl [B, N] fp32)
std::tuple<at::Tensor, at::Tensor, at::Tensor> seqcls_head_fwd(const at::Tensor& h, const at::Tensor& last,
                                                               const at::Tensor& w, const at::Tensor& labels,
                                                               int64_t ignore_index) {
  check_seqcls(h, last, w);
  const int B = h.size(0), T = h.size(1), K = h.size(2), N = w.size(0);
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == B,
              "seqcls_head: labels must be int64 [B]");
  at::Tensor logits = at::empty({B, N}, h.options());
  at::Tensor dl = at::empty({B, N}, h.options().dtype(at::kFloat));
  at::Tensor loss = at::empty({}, h.options().dtype(at::kFloat));
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(h.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  hipLaunchKernelGGL(seqcls_fwd_kernel, dim3(1), dim3(SQ_NT), 0, st, static_cast<const uint16_t*>(h.data_ptr()),
                     last.data_ptr<int64_t>(), T, static_cast<const uint16_t*>(w.data_ptr()), labels.data_ptr<int64_t>(),
                     ignore_index, B, N, K, static_cast<uint16_t*>(logits.data_ptr()), dl.data_ptr<float>(),
                     loss.data_ptr<float>());
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {loss, logits, dl};
}

// (dh [B, T, C], dw [N, C]); dw_out given: written (or += with accumulate) and returned
std::tuple<at::Tensor, at::Tensor> seqcls_head_bwd(const at::Tensor& h, const at::Tensor& last, const at::Tensor& w,
                                                   const at::Tensor& dl, const c10::optional<at::Tensor>& g,
                                                   const c10::optional<at::Tensor>& glog,
                                                   const c10::optional<at::Tensor>& dw_out, bool accumulate) {
  check_seqcls(h, last, w);
  const int B = h.size(0), T = h.size(1), K = h.size(2), N = w.size(0);
  TORCH_CHECK(dl.is_cuda() && dl.scalar_type() == at::kFloat && dl.is_contiguous() && dl.numel() == (int64_t)B * N,
              "seqcls_head_bwd: dl must be float32 [B, N]");
  if (g) TORCH_CHECK(g->is_cuda() && g->scalar_type() == at::kFloat && g->numel() == 1, "seqcls_head_bwd: g float32 [1]");
  if (glog)
    TORCH_CHECK(glog->is_cuda() && glog->scalar_type() == at::kBFloat16 && glog->is_contiguous() &&
                    glog->numel() == (int64_t)B * N,
                "seqcls_head_bwd: glog must be bf16 [B, N]");
  at::Tensor dw;
  if (dw_out && dw_out->defined()) {
    dw = *dw_out;
    TORCH_CHECK(dw.is_cuda() && dw.is_contiguous() && dw.scalar_type() == at::kBFloat16 && dw.sizes() == w.sizes() &&
                    reinterpret_cast<uintptr_t>(dw.data_ptr()) % 16 == 0,
                "seqcls_head_bwd: dw_out must be a contiguous, aligned bf16 tensor shaped like w");
  } else {
    dw = at::empty_like(w);
    accumulate = false;
  }
  at::Tensor dh = at::empty_like(h);
  const int64_t K8 = K / 8;
  const int bh = (int)(((int64_t)B * T * K8 + 255) / 256), bw = (int)(((int64_t)N * K8 + 255) / 256);
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(h.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  hipLaunchKernelGGL(seqcls_bwd_kernel, dim3((unsigned)(bh + bw)), dim3(256), 0, st,
                     static_cast<const uint16_t*>(h.data_ptr()), last.data_ptr<int64_t>(), T,
                     static_cast<const uint16_t*>(w.data_ptr()), dl.data_ptr<float>(), g ? g->data_ptr<float>() : nullptr,
                     glog ? static_cast<const uint16_t*>(glog->data_ptr()) : nullptr, B, N, K,
                     static_cast<uint16_t*>(dh.data_ptr()), static_cast<uint16_t*>(dw.data_ptr()), accumulate ? 1 : 0, bh);
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return {dh, dw};
}

}  // namespace tiny
}  // namespace nbd

TORCH_LIBRARY_FRAGMENT(nbd, m) {
  m.def("linear_tiny(Tensor x, Tensor w, Tensor? bias) -> Tensor");
  m.def("linear_tiny_bwd(Tensor dy, Tensor x, Tensor w, bool want_dx, bool want_dw, bool want_db) -> "
        "(Tensor, Tensor, Tensor)");
  m.def("seqcls_head(Tensor h, Tensor last, Tensor w, Tensor labels, int ignore_index) -> (Tensor, Tensor, Tensor)");
  m.def("seqcls_head_bwd(Tensor h, Tensor last, Tensor w, Tensor dl, Tensor? g, Tensor? glog, Tensor(a!)? dw_out, "
        "bool accumulate) -> (Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("linear_tiny", &nbd::tiny::linear_tiny_fwd);
  m.impl("linear_tiny_bwd", &nbd::tiny::linear_tiny_bwd);
  m.impl("seqcls_head", &nbd::tiny::seqcls_head_fwd);
  m.impl("seqcls_head_bwd", &nbd::tiny::seqcls_head_bwd);
}
