// smallm.hip — fused "small-M" linear layers for decoding (M ≤ 64 token rows), gfx950.
//
// A decode step multiplies a handful of token rows by every weight matrix of the model.  The
// work is bound by streaming the weights once from HBM, and — inside a replayed HIP graph — by the
// fixed cost of each kernel node (≈5 µs per node on MI355X, measured in profiles/generate_*),
// not by FLOPs.  So this kernel fuses everything around one weight product into one node:
//
//     out[m, n] = epilogue( prologue(x)[m, :] · W[n, :] )
//
//   prologue  none | LayerNorm(γ, β) | RMSNorm(γ) of the input rows, computed per workgroup into
//             LDS (bf16, the same rounding as the standalone norm kernels)
//   epilogue  + bias, then none | GELU(tanh) | SwiGLU (W = [gate; up], out = silu(g)·u), then
//             + residual[m, n]
//
// so a GPT-2 block is ln1+qkv · attention · proj+residual · ln2+fc+GELU · proj+residual, five
// nodes instead of ten.
//
// Mapping: a workgroup (8 waves) owns 16 output columns at a time (one MFMA tile in n) for all
// M rows (MT = ⌈M/16⌉ tiles in m); the K dimension is split over the 8 waves and reduced through
// LDS.  v_mfma_f32_16x16x32_bf16 with A = W (16 weight rows) and B = xᵀ: lane l holds
// D[n = 4·(l/16) + r][m = l%16].  The k order inside an MFMA is free as long as A and B agree, so
// lane group g = l/16 walks its own contiguous quarter of K: each lane streams 16-B pieces of one
// weight row in address order.  Workgroups loop over column tiles (grid capped when the
// prologue is recomputed per workgroup, e.g. the LM head's 3,142 tiles).
#include <mutex>
#include <set>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <algorithm>

#include "nbd_common.h"

namespace nbd {
namespace smallm {

constexpr int NT = 512;
constexpr int NW = NT / kWave;  // 8 waves
constexpr int XPAD = 8;         // bf16 elements of row padding in the LDS x image (bank spread)

enum Norm { NORM_NONE = 0, NORM_LN = 1, NORM_RMS = 2 };
enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_SWIGLU = 2 };

typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));

struct Args {
  const uint16_t* x;  // [M, K] bf16, row stride ldx
  int64_t ldx;
  const uint16_t* w;  // [N_w, K] bf16 contiguous
  const uint16_t* bias;  // [N] or nullptr
  const uint16_t* nw;    // norm γ [K] or nullptr
  const uint16_t* nb;    // LayerNorm β [K] or nullptr
  const uint16_t* res;   // [M, N] or nullptr (row stride N)
  uint16_t* out;         // [M, N]
  int M, N, K, norm, stage, ntiles, up_off;  // stage: x image in LDS; up_off: SwiGLU's first up row
  float eps;
};

__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return x * __fdividef(1.f, 1.f + __expf(-2.f * u));
}
__device__ __forceinline__ float silu(float x) { return x * __fdividef(1.f, 1.f + __expf(-x)); }

__device__ __forceinline__ void unpack8(const u32x4& w, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[2 * j] = __uint_as_float(w[j] << 16);
    v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// the x image xs[MT·16][K + XPAD] in LDS, rows [0, M) only (the MFMA loop substitutes zeros for
// the rest): every thread loads its 16-B pieces of the whole [M, K] block at once (one memory
// round trip); with a norm, wave w then normalises rows w, w+8, … in place — all of its rows
// interleaved, so their LDS reads and cross-lane reductions overlap — with the same bf16
// rounding as the standalone LayerNorm / RMSNorm kernels
template <int MT>
__device__ __forceinline__ void prologue(const Args& a, const uint16_t* x, int M, uint16_t* xs, uint16_t* gb,
                                         int tid) {
  const int ld = a.K + XPAD;
  const int total = M * a.K;
  // γ (and β) travel into LDS in the same memory round trip as x
  if (a.norm != NORM_NONE)
    for (int c = tid * 8; c < a.K; c += NT * 8) {
      *reinterpret_cast<u32x4*>(gb + c) = *reinterpret_cast<const u32x4*>(a.nw + c);
      if (a.norm == NORM_LN) *reinterpret_cast<u32x4*>(gb + a.K + c) = *reinterpret_cast<const u32x4*>(a.nb + c);
    }
#pragma unroll 4
  for (int idx = tid * 8; idx < total; idx += NT * 8) {
    const int r = idx / a.K, c = idx - r * a.K;
    *reinterpret_cast<u32x4*>(xs + r * ld + c) = *reinterpret_cast<const u32x4*>(x + (int64_t)r * a.ldx + c);
  }
  if (a.norm == NORM_NONE) return;
  __syncthreads();
  constexpr int RPW = MT * 16 / NW;  // rows per wave
  const int lane = tid & 63, wave = tid >> 6;
  float s[RPW], q[RPW], mean[RPW], rstd[RPW];
#pragma unroll
  for (int j = 0; j < RPW; ++j) s[j] = q[j] = 0.f;
  if (a.norm == NORM_LN) {
    for (int c = lane * 8; c < a.K; c += kWave * 8) {
#pragma unroll
      for (int j = 0; j < RPW; ++j) {
        const int r = wave + NW * j;
        if (r < M) {
          float f[8];
          unpack8(*reinterpret_cast<const u32x4*>(xs + r * ld + c), f);
#pragma unroll
          for (int e = 0; e < 8; ++e) s[j] += f[e];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RPW; ++j) mean[j] = a.norm == NORM_LN ? wave_sum(s[j]) / (float)a.K : 0.f;
  for (int c = lane * 8; c < a.K; c += kWave * 8) {  // two passes, like the standalone kernels
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int r = wave + NW * j;
      if (r < M) {
        float f[8];
        unpack8(*reinterpret_cast<const u32x4*>(xs + r * ld + c), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = f[e] - mean[j];
          q[j] = fmaf(d, d, q[j]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RPW; ++j) rstd[j] = rsqrtf(wave_sum(q[j]) / (float)a.K + a.eps);
  for (int c = lane * 8; c < a.K; c += kWave * 8) {
    float g[8], b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    unpack8(*reinterpret_cast<const u32x4*>(gb + c), g);
    if (a.norm == NORM_LN) unpack8(*reinterpret_cast<const u32x4*>(gb + a.K + c), b);
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int r = wave + NW * j;
      if (r < M) {
        float f[8], o[8];
        unpack8(*reinterpret_cast<const u32x4*>(xs + r * ld + c), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = fmaf((f[e] - mean[j]) * rstd[j], g[e], b[e]);
        store8<bf16_t>(reinterpret_cast<bf16_t*>(xs + r * ld + c), o);
      }
    }
  }
}

// Latency plan (a decode GEMM is ~1 µs of HBM traffic, so every serial memory round trip shows):
// all of a wave's weight fragments for a tile are loaded before anything else — before the
// prologue, whose x loads and norm then overlap them — and the next tile's fragments are issued
// before this tile's cross-wave reduction.  SMAX = the most k-steps one wave owns (K ≤ 4096, or
// 2048 with SwiGLU's two weight rows per column).
template <int MT, int ACT>
__global__ __launch_bounds__(NT) void linear_small_kernel(Args a) {
  constexpr int NACC = ACT == ACT_SWIGLU ? 2 : 1;
  constexpr int SMAX = ACT == ACT_SWIGLU ? 8 : 16;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool lds_x = a.stage != 0;
  const int ldx_s = a.K + XPAD;
  uint16_t* xs = reinterpret_cast<uint16_t*>(smem);
  uint16_t* gb = xs + (lds_x ? (size_t)MT * 16 * ldx_s : 0);  // γ | β (norm prologue only)
  float* red = reinterpret_cast<float*>(gb + (a.norm != NORM_NONE ? 2 * a.K : 0));

  // this workgroup's rows: m-group blockIdx.y of MT·16 rows
  const int row0 = blockIdx.y * MT * 16;
  const int M = min(MT * 16, a.M - row0);
  const uint16_t* x = a.x + (int64_t)row0 * a.ldx;
  const int g = lane >> 4, li = lane & 15;
  const int steps = a.K >> 5;  // MFMA k-steps (8 k per lane per step)
  const int s0 = wave * steps / NW, ns = (wave + 1) * steps / NW - s0;
  const int kg = g * (a.K >> 2) + s0 * 8;  // lane group g walks its own contiguous quarter of K

  s8v wf[NACC][SMAX];
  auto load_w = [&](int tile) {
    const int nr = min(tile * 16 + li, a.N - 1);  // clamped for a ragged last tile
    const uint16_t* w0 = a.w + (int64_t)nr * a.K + kg;
    const uint16_t* w1 = a.w + (int64_t)(a.up_off + nr) * a.K + kg;
#pragma unroll
    for (int i = 0; i < SMAX; ++i)
      if (i < ns) {
        wf[0][i] = *reinterpret_cast<const s8v*>(w0 + i * 8);
        if (ACT == ACT_SWIGLU) wf[NACC - 1][i] = *reinterpret_cast<const s8v*>(w1 + i * 8);
      }
  };
  load_w(blockIdx.x);
  // the first tile's epilogue operands (bias, residual) are fetched now, not after the reduction
  constexpr int QPT = (MT * 256 + NT - 1) / NT;
  float pre_b[QPT], pre_r[QPT];
#pragma unroll
  for (int u = 0; u < QPT; ++u) {
    const int q = tid + u * NT, t = q >> 8, p = q & 255;
    const int ml = t * 16 + (p >> 4), n = blockIdx.x * 16 + (p & 15);
    const bool ok = q < MT * 256 && ml < M && n < a.N;
    pre_b[u] = ok && a.bias != nullptr ? bf16_to_f32(a.bias[n]) : 0.f;
    pre_r[u] = ok && a.res != nullptr ? bf16_to_f32(a.res[(int64_t)(row0 + ml) * a.N + n]) : 0.f;
  }
  if (lds_x) {
    prologue<MT>(a, x, M, xs, gb, tid);
    __syncthreads();
  }

  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    const int n0 = tile * 16;
    f4 acc[NACC][MT];
#pragma unroll
    for (int j = 0; j < NACC; ++j)
#pragma unroll
      for (int t = 0; t < MT; ++t) acc[j][t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < SMAX; ++i) {
      if (i < ns) {
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int m = t * 16 + li;
          s8v xf;
          if (lds_x)
            xf = m < M ? *reinterpret_cast<const s8v*>(xs + m * ldx_s + kg + i * 8) : s8v{0, 0, 0, 0, 0, 0, 0, 0};
          else
            xf = m < M ? *reinterpret_cast<const s8v*>(x + (int64_t)m * a.ldx + kg + i * 8)
                         : s8v{0, 0, 0, 0, 0, 0, 0, 0};
          acc[0][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[0][i], xf, acc[0][t], 0, 0, 0);
          if (ACT == ACT_SWIGLU)
            acc[NACC - 1][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[NACC - 1][i], xf, acc[NACC - 1][t], 0, 0, 0);
        }
      }
    }
    if (tile + (int)gridDim.x < a.ntiles) load_w(tile + gridDim.x);  // in flight across the reduction
    // partial tiles of the 8 waves -> LDS: red[wave][j][t][m_local][n_local]
#pragma unroll
    for (int j = 0; j < NACC; ++j)
#pragma unroll
      for (int t = 0; t < MT; ++t)
        *reinterpret_cast<f4*>(red + (((wave * NACC + j) * MT + t) * 256) + li * 16 + 4 * g) = acc[j][t];
    __syncthreads();
    const bool first = tile == (int)blockIdx.x;
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
      const int q = tid + u * NT;
      if (q >= MT * 256) break;
      const int t = q >> 8, p = q & 255;
      const int ml = t * 16 + (p >> 4), n = n0 + (p & 15);
      const int64_t m = row0 + ml;
      float v0 = 0.f, v1 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        v0 += red[((w * NACC + 0) * MT + t) * 256 + p];
        if (ACT == ACT_SWIGLU) v1 += red[((w * NACC + 1) * MT + t) * 256 + p];
      }
      if (ml < M && n < a.N) {
        float y = v0;
        if (a.bias != nullptr) y += first ? pre_b[u] : bf16_to_f32(a.bias[n]);
        if (ACT == ACT_GELU) y = gelu_tanh(y);
        if (ACT == ACT_SWIGLU) y = silu(y) * v1;
        if (a.res != nullptr) y += first ? pre_r[u] : bf16_to_f32(a.res[m * a.N + n]);
        a.out[m * a.N + n] = f32_to_bf16(y);
      }
    }
    __syncthreads();  // red is reused by the next tile
  }
}

constexpr size_t kMaxLds = 160 * 1024;

static size_t lds_bytes(int MT, int K, bool stage, int act, int norm) {
  const size_t xs = stage ? (size_t)MT * 16 * (K + XPAD) * 2 : 0;
  const size_t gb = norm != NORM_NONE ? (size_t)2 * K * 2 : 0;
  return xs + gb + (size_t)NW * (act == ACT_SWIGLU ? 2 : 1) * MT * 256 * 4;
}

at::Tensor linear_small_hip(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                            const c10::optional<at::Tensor>& norm_w, const c10::optional<at::Tensor>& norm_b,
                            double eps, int64_t norm, int64_t act, const c10::optional<at::Tensor>& residual) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 &&
                  x.stride(0) % 8 == 0 && ((uintptr_t)x.data_ptr() & 15) == 0,
              "linear_small: x must be a bf16 [M, K] GPU view with unit last stride and 16-B aligned rows");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 2 && w.is_contiguous() &&
                  ((uintptr_t)w.data_ptr() & 15) == 0,
              "linear_small: w must be a contiguous bf16 [N, K] GPU tensor");
  const int64_t M = x.size(0), K = x.size(1);
  TORCH_CHECK(M >= 1 && M <= 64, "linear_small: 1 <= M <= 64 rows");
  TORCH_CHECK(K == w.size(1) && K % 32 == 0 && K <= (act == ACT_SWIGLU ? 2048 : 4096),
              "linear_small: K must match w, K % 32 == 0, K <= 4096 (2048 with SwiGLU)");
  TORCH_CHECK(norm >= 0 && norm <= 2 && act >= 0 && act <= 2, "linear_small: bad norm / act");
  const bool swiglu = act == ACT_SWIGLU;
  TORCH_CHECK(!swiglu || w.size(0) % 2 == 0, "linear_small: SwiGLU needs w = [gate; up]");
  const int64_t N = swiglu ? w.size(0) / 2 : w.size(0);
  TORCH_CHECK(N >= 1 && N < (1LL << 31) / 16, "linear_small: bad N");
  auto opt_bf16 = [&](const c10::optional<at::Tensor>& t, int64_t n, const char* name) -> const uint16_t* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->numel() == n &&
                    ((uintptr_t)t->data_ptr() & 15) == 0,
                "linear_small: ", name, " must be a contiguous 16-B aligned bf16 tensor of ", n, " elements");
    return static_cast<const uint16_t*>(t->data_ptr());
  };
  Args a;
  a.x = static_cast<const uint16_t*>(x.data_ptr());
  a.ldx = x.stride(0);
  a.w = static_cast<const uint16_t*>(w.data_ptr());
  a.bias = opt_bf16(bias, N, "bias");
  a.nw = norm != NORM_NONE ? opt_bf16(norm_w, K, "norm_w") : nullptr;
  a.nb = norm == NORM_LN ? opt_bf16(norm_b, K, "norm_b") : nullptr;
  TORCH_CHECK(norm == NORM_NONE || (a.nw != nullptr && (norm != NORM_LN || a.nb != nullptr)),
              "linear_small: the norm prologue needs its weights");
  a.res = opt_bf16(residual, M * N, "residual");
  at::Tensor out = at::empty({M, N}, x.options().memory_format(at::MemoryFormat::Contiguous));
  a.out = static_cast<uint16_t*>(out.data_ptr());
  a.M = (int)M;
  a.N = (int)N;
  a.K = (int)K;
  a.norm = (int)norm;
  a.ntiles = (int)((N + 15) / 16);
  a.up_off = (int)N;
  a.eps = (float)eps;
  // m-tiles per workgroup: all of them (weights read once) unless the x image would not fit in
  // LDS, or the column tiles alone leave most CUs idle — then one m-tile per workgroup and a
  // second grid dimension over the row groups (the weights are re-read from L2)
  const int MT_all = (int)((M + 15) / 16);
  int MT = MT_all;
  if (MT > 1 && (a.ntiles < 128 || lds_bytes(MT, (int)K, true, (int)act, (int)norm) > kMaxLds)) MT = 1;
  const int mgroups = (MT_all + MT - 1) / MT;
  // the x image goes to LDS whenever it fits (a norm prologue requires it)
  a.stage = norm != NORM_NONE || lds_bytes(MT, (int)K, true, (int)act, (int)norm) <= kMaxLds;
  const size_t lds = lds_bytes(MT, (int)K, a.stage != 0, (int)act, (int)norm);
  TORCH_CHECK(lds <= kMaxLds, "linear_small: needs ", lds, " B of LDS (> 160 KiB); normalise separately");
  // the prologue is recomputed per workgroup: cap the grid there (workgroups loop over tiles)
  const int grid = a.stage ? std::min(a.ntiles, 512) : a.ntiles;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  auto launch = [&](auto kern) {
    // every instantiation has the same pointer type, so the "set once" state is keyed by
    // (device, kernel pointer) — a per-lambda static would cover only the first kernel launched
    static std::mutex mu;
    static std::set<std::pair<int, const void*>> done;
    const void* fp = reinterpret_cast<const void*>(kern);
    {
      std::lock_guard<std::mutex> lk(mu);
      if (done.insert({(int)x.get_device(), fp}).second)
        C10_HIP_CHECK(hipFuncSetAttribute(fp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds));
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)grid, (unsigned)mgroups), dim3(NT), lds, st, a);
  };
#define NBD_SMALLM(mt)                                                    \
  case mt:                                                                \
    if (act == ACT_NONE) launch(linear_small_kernel<mt, ACT_NONE>);       \
    else if (act == ACT_GELU) launch(linear_small_kernel<mt, ACT_GELU>);  \
    else launch(linear_small_kernel<mt, ACT_SWIGLU>);                     \
    break;
  switch (MT) {
    NBD_SMALLM(1)
    NBD_SMALLM(2)
    NBD_SMALLM(3)
    NBD_SMALLM(4)
  }
#undef NBD_SMALLM
  C10_HIP_KERNEL_LAUNCH_CHECK();
  return out;
}

}  // namespace smallm
}  // namespace nbd

TORCH_LIBRARY_IMPL(nbd, CUDA, m) { m.impl("linear_small", &nbd::smallm::linear_small_hip); }
