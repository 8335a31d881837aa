// autograd.hip — the Linear / MLP autograd nodes of the model paths in C++.
//
// An eager training step of a small model is host-bound: SmolLM2-135M at 16x128 tokens spends
// ≈11 ms issuing what the GPU runs in 7 ms (graph replay), and a Python torch.autograd.Function
// costs ≈20-25 µs per call before its kernels (ctx object, saved tensors, Python wrappers around
// every GEMM) — forward and again backward (benchmarks/host_profile.py --cprofile).  These nodes
// run the same kernels (gemm.hip: fused bias / GELU / SwiGLU epilogues, the grouped dgrad + wgrad
// backward launch) with no Python between the dispatcher and the launches.
//
// Which kernel (tile, split-K, or the hipBLASLt library GEMM) runs each product is decided in
// Python once per shape (ops/gemm.py `native_plan`: the tuned table and heuristics of
// `ops.gemm.config` / `prefer_library`) and passed down as an int list, so the two paths pick
// identical kernels.  Plan layout: a sequence of products, 3 ints each (library?, tile, splits),
// then the grouped-launch split counts (-1 = run the backward products one by one):
//   linear_ag     [fwd, dgrad, wgrad]               + [pair]
//   mlp_gelu_ag   [fc, proj, proj dgrad, proj wgrad, fc dgrad, fc wgrad]   + [pair proj, pair fc]
//   mlp_swiglu_ag [gate_up, down, down dgrad, down wgrad, gu dgrad, gu wgrad] + [pair down, pair gu]
// Python reference: ops/gemm.py _Linear / _MLPGelu / _MLPSwiGLU (same math, same kernels).
// Also here: the (add +) RMSNorm / LayerNorm nodes (ops/llama.py _RMSNorm / _AddRMSNorm, ops/norm.py
// _LayerNorm / _AddLayerNorm) and attention from a packed q|k|v projection (ops/attention.py
// _FlashAttentionQKV).
#include <ATen/ATen.h>
#include <ATen/hip/HIPGraph.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/GradMode.h>
#include <torch/csrc/autograd/custom_function.h>
#include <torch/library.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <sstream>
#include <functional>
#include <map>
#include <optional>
#include <memory>
#include <mutex>
#include <tuple>
#include <unordered_map>
#include <unordered_set>

#include "gemm_common.h"
#include "graddst.h"

namespace nbd {
namespace gemm {
void gemm_hip(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c, bool a_km, bool b_kn,
              const c10::optional<at::Tensor>& bias, int64_t epi, const c10::optional<at::Tensor>& aux_in,
              const c10::optional<at::Tensor>& aux_out, int64_t splits, int64_t tile_hint, int64_t accum);
void gemm_pair_hip(const at::Tensor& a1, const at::Tensor& b1, const at::Tensor& c1, int64_t epi1,
                   const c10::optional<at::Tensor>& aux_in1, const at::Tensor& a2, const at::Tensor& b2,
                   const at::Tensor& c2, int64_t epi2, const c10::optional<at::Tensor>& aux_out2, int64_t splits2,
                   int64_t accum2, const c10::optional<at::Tensor>& delta1 = c10::nullopt, int64_t delta_T = 0);
}  // namespace gemm
namespace norm {
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> ln_fwd_hip(const at::Tensor& x,
                                                                      const c10::optional<at::Tensor>& delta,
                                                                      const at::Tensor& weight,
                                                                      const at::Tensor& bias, double eps);
std::tuple<at::Tensor, at::Tensor, at::Tensor> ln_bwd_hip(const at::Tensor& x, const at::Tensor& dy,
                                                          const c10::optional<at::Tensor>& dres,
                                                          const at::Tensor& weight, const at::Tensor& mean,
                                                          const at::Tensor& rstd);
std::tuple<at::Tensor, at::Tensor, at::Tensor> rms_fwd_hip(const at::Tensor& x, const c10::optional<at::Tensor>& delta,
                                                           const at::Tensor& weight, double eps);
std::tuple<at::Tensor, at::Tensor> rms_bwd_hip(const at::Tensor& x, const at::Tensor& dy,
                                               const c10::optional<at::Tensor>& dres, const at::Tensor& weight,
                                               const at::Tensor& rstd);
std::tuple<at::Tensor, at::Tensor, at::Tensor> ln_bwd_into(const at::Tensor& x, const at::Tensor& dy,
                                                           const c10::optional<at::Tensor>& dres,
                                                           const at::Tensor& weight, const at::Tensor& mean,
                                                           const at::Tensor& rstd, const at::Tensor& dw_dst,
                                                           const at::Tensor& db_dst, int accum);
std::tuple<at::Tensor, at::Tensor> rms_bwd_into(const at::Tensor& x, const at::Tensor& dy,
                                                const c10::optional<at::Tensor>& dres, const at::Tensor& weight,
                                                const at::Tensor& rstd, const at::Tensor& dw_dst, int accum);
std::tuple<at::Tensor, at::Tensor, at::Tensor> embed_rms_fwd_hip(const at::Tensor& ids, const at::Tensor& table,
                                                                 const at::Tensor& weight, double eps,
                                                                 const c10::optional<at::Tensor>& err);
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> tokpos_ln_fwd_hip(
    const at::Tensor& idx, const at::Tensor& wte, const at::Tensor& pos, const at::Tensor& wpe, int64_t vocab,
    const at::Tensor& weight, const at::Tensor& bias, double eps, const c10::optional<at::Tensor>& err);
}  // namespace norm
namespace embed {
at::Tensor embedding_bwd_hip(const at::Tensor& dy, const at::Tensor& idx, int64_t V,
                             const c10::optional<at::Tensor>& grad_out, bool accumulate);
at::Tensor embedding_pos_bwd_hip(const at::Tensor& dy, const at::Tensor& pos, int64_t P,
                                 const c10::optional<at::Tensor>& out_opt, bool accumulate);
}  // namespace embed
namespace graddst {
at::Tensor grad_dest_join(const at::Tensor& param);
}  // namespace graddst
namespace gemm {
std::vector<at::Tensor> gemm_warm_take_refs();
}  // namespace gemm
void bucket_flatten_hip(at::TensorList tensors, const at::Tensor& bucket, at::IntArrayRef offsets, double scale,
                        bool accumulate);
namespace attn {
std::tuple<at::Tensor, at::Tensor> attn_fwd_hip(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                                bool causal, double scale, const c10::optional<at::Tensor>& rope_cos,
                                                const c10::optional<at::Tensor>& rope_sin);
void attn_bwd_hip(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                  const at::Tensor& out, const at::Tensor& lse, bool causal, double scale, const at::Tensor& dq,
                  const at::Tensor& dk, const at::Tensor& dv, const c10::optional<at::Tensor>& rope_cos,
                  const c10::optional<at::Tensor>& rope_sin, const c10::optional<at::Tensor>& delta = c10::nullopt);
}  // namespace attn

namespace ag {
using at::Tensor;
using c10::optional;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;
using namespace nbd::gemm;

// ---- host-time breakdown of the block nodes (NBD_HOST_TIMING=1; torch.ops.nbd.host_timing) --
namespace ht {
enum Id { FWD, BWD, UNPACK, RMS_NEXT, SWIGLU, RMS_POST, LIN_O, ATTN, LIN_QKV, GEMM_CALL, PAIR_CALL, ATTN_CALL,
          CLAIM, ALLOC, kN };
const char* const kNames[kN] = {"block fwd (node)", "block bwd (node)", "  bwd: saved unpack", "  bwd: rms next",
                                "  bwd: swiglu", "  bwd: rms post", "  bwd: linear o", "  bwd: attention",
                                "  bwd: linear qkv", "gemm_hip call", "gemm_pair_hip call", "attn_bwd_hip call",
                                "grad_out (claim+alloc)", "unused"};
std::atomic<int64_t> g_ns[kN], g_cnt[kN];
bool on() {
  static const bool e = [] {
    const char* v = std::getenv("NBD_HOST_TIMING");
    return v != nullptr && v[0] == '1';
  }();
  return e;
}
struct Scope {
  int id;
  bool active;
  std::chrono::steady_clock::time_point t0;
  explicit Scope(int i) : id(i), active(on()) {
    if (active) t0 = std::chrono::steady_clock::now();
  }
  ~Scope() {
    if (!active) return;
    g_ns[id] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    ++g_cnt[id];
  }
};
}  // namespace ht

struct Prod {
  bool lib;
  int64_t tile, splits;
};

static Prod prod(at::IntArrayRef plan, int i) {
  TORCH_CHECK((int64_t)plan.size() >= 3 * (i + 1), "nbd autograd: plan too short");
  return {plan[3 * i] != 0, plan[3 * i + 1], plan[3 * i + 2]};
}

static bool aligned(const Tensor& t, int bytes = 16) {
  return reinterpret_cast<uintptr_t>(t.data_ptr()) % bytes == 0;
}

static Tensor bf16c(const Tensor& t) {
  Tensor r = t.scalar_type() == at::kBFloat16 ? t : t.to(at::kBFloat16);
  return r.is_contiguous() ? r : r.contiguous();
}

// c = A·B (layouts as gemm.hip), `epi` with its operands; returns (c, aux_out).  The library path
// (hipBLASLt through at::mm / addmm) serves plain products the plan routes there, and any plain
// product whose operands are not 16-byte aligned (as ops.gemm.matmul does).  `c_out` / `rs_out`:
// write the product / row sums there (gradient destinations, graddst.h), adding to their contents
// when `accum` bit 0 / bit 1 is set.
static std::pair<Tensor, Tensor> run(const Tensor& a, const Tensor& b, bool a_km, bool b_kn, const Prod& p,
                                     int epi = EPI_NONE, const optional<Tensor>& bias = c10::nullopt,
                                     const optional<Tensor>& aux = c10::nullopt, const Tensor& c_out = Tensor(),
                                     const Tensor& rs_out = Tensor(), int accum = 0) {
  const int64_t M = a_km ? a.size(1) : a.size(0), N = b_kn ? b.size(1) : b.size(0);
  const bool bias_ok = !bias || (bias->is_contiguous() && aligned(*bias, 8) && bias->scalar_type() == at::kBFloat16);
  const bool out_ok = !c_out.defined() || aligned(c_out);
  if (epi == EPI_NONE && (p.lib || !aligned(a) || !aligned(b) || !bias_ok || !out_ok)) {
    const Tensor A = a_km ? a.t() : a, B = b_kn ? b : b.t();
    if (c_out.defined()) {
      TORCH_CHECK(!bias, "nbd autograd: bias with a destination");
      if (accum & 1) c_out.view({M, N}).addmm_(A, B);
      else {
        Tensor o = c_out.view({M, N});
        at::mm_out(o, A, B);
      }
      return {c_out, Tensor()};
    }
    return {bias ? at::addmm(*bias, A, B) : at::mm(A, B), Tensor()};
  }
  const int64_t cN = epi == EPI_SWIGLU ? N / 2 : epi == EPI_DSWIGLU ? 2 * N : N;
  // the 256x256 kernel has no accumulating epilogue: product into a temporary, then add
  const bool tmp_acc = accum != 0 && (p.tile / 1000 % 1000) == 256;
  Tensor c = c_out.defined() && !(tmp_acc && (accum & 1)) ? c_out.view({M, cN}) : at::empty({M, cN}, a.options());
  Tensor out;
  if (epi == EPI_GELU) out = at::empty_like(c);
  if (epi == EPI_ROWSUM) out = rs_out.defined() && !(tmp_acc && (accum & 2)) ? rs_out.view({M}) : at::empty({M}, a.options());
  if (epi == EPI_SWIGLU) out = at::empty({M, N}, a.options());
  // a deferred split-K reduce only when it writes the destinations themselves (not a temporary
  // that is read right after)
  const defer::Scope ds(defer::want() && !tmp_acc && c_out.defined() && (epi != EPI_ROWSUM || rs_out.defined()));
  {
    const ht::Scope hs(ht::GEMM_CALL);
    gemm_hip(a, b, c, a_km, b_kn, bias, epi, aux, out.defined() ? optional<Tensor>(out) : c10::nullopt, p.splits,
             p.tile, tmp_acc ? 0 : accum);
  }
  if (tmp_acc) {
    if (accum & 1) { c_out.view({M, cN}).add_(c); c = c_out.view({M, cN}); }
    if (accum & 2) { rs_out.view({M}).add_(out); out = rs_out.view({M}); }
  }
  return {c, out};
}

// A gradient output: the parameter's registered destination (graddst.h) or a fresh tensor.
struct GradOut {
  Tensor t;
  Tensor param;
  bool claimed = false, acc = false;
  int bit(int b) const { return acc ? b : 0; }
  Tensor done() const { return claimed ? graddst::hand_back(param, t, acc) : t; }
};

static GradOut grad_out(const Tensor& param, bool want, at::IntArrayRef shape, const at::TensorOptions& opt) {
  const ht::Scope hs(ht::CLAIM);
  GradOut g;
  if (!want) return g;
  if (param.defined()) {
    g.t = graddst::claim(param, g.acc);
    g.claimed = g.t.defined();
    if (g.claimed) {
      g.param = param;
      if (!aligned(g.t) || g.t.scalar_type() != opt.dtype().toScalarType()) {  // unusable: normal path
        g = GradOut();
      }
    }
  }
  if (!g.claimed) g.t = at::empty(shape, opt);
  return g;
}

// dx = dy·W [· act′(aux)], dW = dyᵀ·x [, db = Σ dy] in one grouped launch (gemm_pair_hip)
static std::tuple<Tensor, Tensor, Tensor> pair(const Tensor& dy, const Tensor& w, const Tensor& x, int epi1,
                                               const optional<Tensor>& aux1, bool bias_grad, int64_t splits,
                                               const Tensor& bparam = Tensor(), const Tensor& delta = Tensor(),
                                               int64_t delta_T = 0) {
  const int64_t M = dy.size(0), N = dy.size(1), K = w.size(1);
  Tensor dx = at::empty({M, epi1 == EPI_DSWIGLU ? 2 * K : K}, dy.options());
  const GradOut dw = grad_out(w, true, {N, K}, dy.options());
  const GradOut db = grad_out(bparam, bias_grad, {N}, dy.options());
  // every output of the split-K reduce is a bucket slice: it may be deferred (graddst.h)
  const defer::Scope ds(dw.claimed && (!bias_grad || db.claimed));
  {
    const ht::Scope hs(ht::PAIR_CALL);
    gemm_pair_hip(dy, w, dx, epi1, aux1, dy, x, dw.t.view({N, K}), bias_grad ? EPI_ROWSUM : EPI_NONE,
                  bias_grad ? optional<Tensor>(db.t.view({N})) : c10::nullopt, splits, dw.bit(1) | db.bit(2),
                  delta.defined() ? optional<Tensor>(delta) : c10::nullopt, delta_T);
  }
  return {dx, dw.done(), bias_grad ? db.done() : Tensor()};
}

// dW = dyᵀ·x [, db = Σ dy] as separate products (plan entry `pi`), into the gradient destinations
static std::pair<Tensor, Tensor> wgrad(const Tensor& dy, const Tensor& x2, const Tensor& w, const Tensor& bparam,
                                       bool nb, at::IntArrayRef plan, int pi) {
  const int64_t N = dy.size(1), K = x2.size(1);
  const GradOut dw = grad_out(w, true, {N, K}, dy.options());
  const GradOut db = grad_out(bparam, nb, {N}, dy.options());
  const defer::Scope ds(dw.claimed && (!nb || db.claimed));
  run(dy, x2, true, true, prod(plan, pi), nb ? EPI_ROWSUM : EPI_NONE, c10::nullopt, c10::nullopt, dw.t,
      nb ? db.t : Tensor(), dw.bit(1) | db.bit(2));
  return {dw.done(), nb ? db.done() : Tensor()};
}

static std::vector<int64_t> out_shape(const Tensor& x, int64_t n) {
  std::vector<int64_t> s(x.sizes().begin(), x.sizes().end());
  s.back() = n;
  return s;
}

// ---- the flash backward's δ from the output projection (GPT-2: attention -> c_proj) ----------
// δ = Σ_d dO·O per (query, head) is the attention backward's pre-pass; dO is the input gradient
// of the Linear that consumes the attention output O, so that Linear's grouped backward launch
// can produce δ in its epilogue (gemm.hip EPI_ADELTA) and the pre-pass launch goes away.  The
// attention node registers its output here at forward time; the Linear's backward, finding its
// input registered, fills δ; the attention's backward takes it only if its dout IS that Linear's
// input gradient (a second consumer of O would have summed gradients into another tensor).
namespace adelta {
struct Req {
  int64_t T = 0, H = 0;
  Tensor delta;             // filled by the Linear's backward
  const void* dx = nullptr;  // ... for this input gradient
};
std::mutex mu;
std::unordered_map<const void*, Req> reqs;

static bool enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NBD_ATTN_DELTA_EPI");  // 0: the pre-pass kernel (A/B)
    return e == nullptr || e[0] != '0';
  }();
  return on;
}
static void want(const Tensor& o, int64_t T, int64_t H) {
  std::lock_guard<std::mutex> lk(mu);
  reqs[o.data_ptr()] = Req{T, H, Tensor(), nullptr};  // (a new forward resets a stale entry)
}
// the δ tensor to fill for the Linear input x2 [B·T, H·64], or undefined
static Tensor request(const Tensor& x2) {
  std::lock_guard<std::mutex> lk(mu);
  auto it = reqs.find(x2.data_ptr());
  if (it == reqs.end()) return Tensor();
  Req& r = it->second;
  if (x2.dim() != 2 || x2.size(1) != r.H * 64 || r.T <= 0 || x2.size(0) % r.T != 0) return Tensor();
  r.delta = at::empty({x2.size(0) / r.T, r.H, r.T}, x2.options().dtype(at::kFloat));
  r.dx = nullptr;
  return r.delta;
}
static void produced(const Tensor& x2, const Tensor& dx) {
  std::lock_guard<std::mutex> lk(mu);
  auto it = reqs.find(x2.data_ptr());
  if (it != reqs.end()) it->second.dx = dx.data_ptr();
}
// δ for the attention output o whose incoming gradient is dout (and forget the entry)
static Tensor take(const Tensor& o, const Tensor& dout) {
  std::lock_guard<std::mutex> lk(mu);
  auto it = reqs.find(o.data_ptr());
  if (it == reqs.end()) return Tensor();
  Tensor d = (it->second.delta.defined() && it->second.dx == dout.data_ptr()) ? it->second.delta : Tensor();
  reqs.erase(it);
  return d;
}
}  // namespace adelta

// ------------------------------------------------------------------------------------- Linear
static Tensor linear_forward(const Tensor& x2, const Tensor& w, const optional<Tensor>& b, at::IntArrayRef plan) {
  return run(x2, w, false, false, prod(plan, 0), EPI_NONE, b).first;
}

// fp32 / fp16 weights (a user's nn.Linear under nbd DDP, parallel/ddp.py): the library GEMMs, with
// the weight / bias gradients written into their DDP bucket slices like the bf16 path
static bool lib_dtype(const Tensor& w) { return w.scalar_type() != at::kBFloat16; }

struct LinearFn : public torch::autograd::Function<LinearFn> {
  static Tensor forward(AutogradContext* ctx, const Tensor& x, const Tensor& w, const optional<Tensor>& b,
                        at::IntArrayRef plan) {
    at::AutoDispatchBelowADInplaceOrView guard;
    const bool lib = lib_dtype(w);
    const Tensor x2 = lib ? x.reshape({-1, x.size(-1)}).contiguous() : bf16c(x).view({-1, x.size(-1)});
    ctx->save_for_backward({x2, w, b ? *b : Tensor()});
    ctx->saved_data["plan"] = plan.vec();
    ctx->saved_data["need"] = std::vector<bool>{x.requires_grad(), w.requires_grad(), b && b->requires_grad()};
    ctx->saved_data["xshape"] = x.sizes().vec();
    if (lib) {
      const Tensor y = b ? at::addmm(*b, x2, w.t()) : at::mm(x2, w.t());
      return y.view(out_shape(x, w.size(0)));
    }
    return linear_forward(x2, w, b, plan).view(out_shape(x, w.size(0)));
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const auto saved = ctx->get_saved_variables();
    const Tensor &x2 = saved[0], &w = saved[1], &b = saved[2];
    const auto plan = ctx->saved_data["plan"].toIntVector();
    const auto need = ctx->saved_data["need"].toBoolList();
    const auto xshape = ctx->saved_data["xshape"].toIntVector();
    const bool nx = need[0], nw = need[1], nb = need[2];
    Tensor dx, dw, db;
    if (lib_dtype(w)) {
      const Tensor dy = grads[0].reshape({-1, w.size(0)}).contiguous();
      if (nx) dx = at::mm(dy, w);
      if (nw) {
        const GradOut g = grad_out(w, true, w.sizes(), dy.options());
        if (g.acc) g.t.addmm_(dy.t(), x2);
        else {
          Tensor o = g.t;
          at::mm_out(o, dy.t(), x2);
        }
        dw = g.done();
      }
      if (nb) {
        const GradOut g = grad_out(b, true, {w.size(0)}, dy.options());
        if (g.acc) g.t.add_(dy.sum(0));
        else {
          Tensor o = g.t;
          at::sum_out(o, dy, {0});
        }
        db = g.done();
      }
      return {dx.defined() ? dx.view(xshape) : dx, dw, db, Tensor()};
    }
    const Tensor dy = bf16c(grads[0]).view({-1, w.size(0)});
    if (nx && nw && plan[9] >= 0) {
      // an attention output as this Linear's input: the flash backward's δ from this launch
      const Tensor delta = adelta::enabled() ? adelta::request(x2) : Tensor();
      if (delta.defined()) {
        std::tie(dx, dw, db) = pair(dy, w, x2, EPI_ADELTA, x2, nb, plan[9], b, delta, delta.size(2));
        adelta::produced(x2, dx);
      } else {
        std::tie(dx, dw, db) = pair(dy, w, x2, EPI_NONE, c10::nullopt, nb, plan[9], b);
      }
    } else {
      if (nx) dx = run(dy, w, false, true, prod(plan, 1)).first;
      if (nw) std::tie(dw, db) = wgrad(dy, x2, w, b, nb, plan, 2);
      else if (nb) db = dy.sum(0, false, at::kFloat).to(dy.scalar_type());
    }
    return {dx.defined() ? dx.view(xshape) : dx, dw, db, Tensor()};
  }
};

Tensor linear_ag(const Tensor& x, const Tensor& w, const optional<Tensor>& b, at::IntArrayRef plan) {
  return LinearFn::apply(x, w, b, plan);
}

Tensor linear_noag(const Tensor& x, const Tensor& w, const optional<Tensor>& b, at::IntArrayRef plan) {
  if (lib_dtype(w)) {
    const Tensor x2 = x.reshape({-1, x.size(-1)});
    return (b ? at::addmm(*b, x2, w.t()) : at::mm(x2, w.t())).view(out_shape(x, w.size(0)));
  }
  return linear_forward(bf16c(x).view({-1, x.size(-1)}), w, b, plan).view(out_shape(x, w.size(0)));
}

// ------------------------------------------------------------------------------ GPT-2 MLP (GELU)
struct MLPGeluFn : public torch::autograd::Function<MLPGeluFn> {
  static Tensor forward(AutogradContext* ctx, const Tensor& x, const Tensor& w1, const optional<Tensor>& b1,
                        const Tensor& w2, const optional<Tensor>& b2, at::IntArrayRef plan) {
    at::AutoDispatchBelowADInplaceOrView guard;
    const Tensor x2 = bf16c(x).view({-1, x.size(-1)});
    auto [g, pre] = run(x2, w1, false, false, prod(plan, 0), EPI_GELU, b1);
    const Tensor y = run(g, w2, false, false, prod(plan, 1), EPI_NONE, b2).first;
    ctx->save_for_backward({x2, w1, w2, pre, g, b1 ? *b1 : Tensor(), b2 ? *b2 : Tensor()});
    ctx->saved_data["plan"] = plan.vec();
    ctx->saved_data["need"] = std::vector<bool>{x.requires_grad(), b1.has_value(), b2.has_value()};
    ctx->saved_data["xshape"] = x.sizes().vec();
    return y.view(out_shape(x, w2.size(0)));
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const auto s = ctx->get_saved_variables();
    const Tensor &x2 = s[0], &w1 = s[1], &w2 = s[2], &pre = s[3], &g = s[4], &b1 = s[5], &b2 = s[6];
    const auto plan = ctx->saved_data["plan"].toIntVector();
    const auto need = ctx->saved_data["need"].toBoolList();
    const auto xshape = ctx->saved_data["xshape"].toIntVector();
    const bool nx = need[0], hb1 = need[1], hb2 = need[2];
    const Tensor dy = bf16c(grads[0]).view({-1, w2.size(0)});
    Tensor dpre, dw2, db2, dx, dw1, db1;
    if (plan[18] >= 0) {
      std::tie(dpre, dw2, db2) = pair(dy, w2, g, EPI_DGELU, pre, hb2, plan[18], b2);
    } else {
      dpre = run(dy, w2, false, true, prod(plan, 2), EPI_DGELU, c10::nullopt, pre).first;
      std::tie(dw2, db2) = wgrad(dy, g, w2, b2, hb2, plan, 3);
    }
    if (nx && plan[19] >= 0) {
      std::tie(dx, dw1, db1) = pair(dpre, w1, x2, EPI_NONE, c10::nullopt, hb1, plan[19], b1);
    } else {
      if (nx) dx = run(dpre, w1, false, true, prod(plan, 4)).first;
      std::tie(dw1, db1) = wgrad(dpre, x2, w1, b1, hb1, plan, 5);
    }
    return {dx.defined() ? dx.view(xshape) : dx, dw1, db1, dw2, db2, Tensor()};
  }
};

Tensor mlp_gelu_ag(const Tensor& x, const Tensor& w1, const optional<Tensor>& b1, const Tensor& w2,
                   const optional<Tensor>& b2, at::IntArrayRef plan) {
  return MLPGeluFn::apply(x, w1, b1, w2, b2, plan);
}

Tensor mlp_gelu_noag(const Tensor& x, const Tensor& w1, const optional<Tensor>& b1, const Tensor& w2,
                     const optional<Tensor>& b2, at::IntArrayRef plan) {
  const Tensor x2 = bf16c(x).view({-1, x.size(-1)});
  const Tensor g = run(x2, w1, false, false, prod(plan, 0), EPI_GELU, b1).first;
  return run(g, w2, false, false, prod(plan, 1), EPI_NONE, b2).first.view(out_shape(x, w2.size(0)));
}

// ----------------------------------------------------------------------------- Llama MLP (SwiGLU)
struct MLPSwiGLUFn : public torch::autograd::Function<MLPSwiGLUFn> {
  static Tensor forward(AutogradContext* ctx, const Tensor& x, const Tensor& w_gu, const Tensor& w_down,
                        at::IntArrayRef plan) {
    at::AutoDispatchBelowADInplaceOrView guard;
    const Tensor x2 = bf16c(x).view({-1, x.size(-1)});
    auto [act, pre] = run(x2, w_gu, false, false, prod(plan, 0), EPI_SWIGLU);
    const Tensor y = run(act, w_down, false, false, prod(plan, 1)).first;
    ctx->save_for_backward({x2, w_gu, w_down, pre, act});
    ctx->saved_data["plan"] = plan.vec();
    ctx->saved_data["nx"] = x.requires_grad();
    ctx->saved_data["xshape"] = x.sizes().vec();
    return y.view(out_shape(x, w_down.size(0)));
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const auto s = ctx->get_saved_variables();
    const Tensor &x2 = s[0], &w_gu = s[1], &w_down = s[2], &pre = s[3], &act = s[4];
    const auto plan = ctx->saved_data["plan"].toIntVector();
    const bool nx = ctx->saved_data["nx"].toBool();
    const auto xshape = ctx->saved_data["xshape"].toIntVector();
    const Tensor dy = bf16c(grads[0]).view({-1, w_down.size(0)});
    Tensor dgu, dw_down, dx, dw_gu, unused;
    if (plan[18] >= 0) {
      std::tie(dgu, dw_down, unused) = pair(dy, w_down, act, EPI_DSWIGLU, pre, false, plan[18]);
    } else {
      dgu = run(dy, w_down, false, true, prod(plan, 2), EPI_DSWIGLU, c10::nullopt, pre).first;
      dw_down = wgrad(dy, act, w_down, Tensor(), false, plan, 3).first;
    }
    if (nx && plan[19] >= 0) {
      std::tie(dx, dw_gu, unused) = pair(dgu, w_gu, x2, EPI_NONE, c10::nullopt, false, plan[19]);
    } else {
      if (nx) dx = run(dgu, w_gu, false, true, prod(plan, 4)).first;
      dw_gu = wgrad(dgu, x2, w_gu, Tensor(), false, plan, 5).first;
    }
    return {dx.defined() ? dx.view(xshape) : dx, dw_gu, dw_down, Tensor()};
  }
};

Tensor mlp_swiglu_ag(const Tensor& x, const Tensor& w_gu, const Tensor& w_down, at::IntArrayRef plan) {
  return MLPSwiGLUFn::apply(x, w_gu, w_down, plan);
}

Tensor mlp_swiglu_noag(const Tensor& x, const Tensor& w_gu, const Tensor& w_down, at::IntArrayRef plan) {
  const Tensor x2 = bf16c(x).view({-1, x.size(-1)});
  const Tensor act = run(x2, w_gu, false, false, prod(plan, 0), EPI_SWIGLU).first;
  return run(act, w_down, false, false, prod(plan, 1)).first.view(out_shape(x, w_down.size(0)));
}

// ------------------------------------------------------------ (add +) RMSNorm / LayerNorm nodes
// The residual add and the norm in one pass forward (s = x + delta, y = norm(s)), their
// backward in one pass too (dx = ds + norm′(dy)).  ``delta`` absent: the plain norm (one output).
static c10::optional<Tensor> opt(const Tensor& t) { return t.defined() ? c10::optional<Tensor>(t.contiguous()) : c10::nullopt; }

struct RMSFn : public torch::autograd::Function<RMSFn> {
  static variable_list forward(AutogradContext* ctx, const Tensor& x, const optional<Tensor>& delta, const Tensor& w,
                               double eps) {
    at::AutoDispatchBelowADInplaceOrView guard;
    ctx->set_materialize_grads(false);
    auto [y, sum, rstd] = norm::rms_fwd_hip(x, delta, w, eps);
    const bool add = delta.has_value();
    ctx->save_for_backward({add ? sum : x, w, rstd});
    ctx->saved_data["add"] = add;
    if (add) return {sum, y};
    return {y};
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const auto sv = ctx->get_saved_variables();
    const bool add = ctx->saved_data["add"].toBool();
    const Tensor ds = add ? grads[0] : Tensor(), dy = add ? grads[1] : grads[0];
    if (!dy.defined()) return {ds, ds, Tensor(), Tensor()};
    // dγ into its bucket slice when DDP registered one (graddst.h); the column sum may be deferred
    const Tensor& w = sv[1];
    const GradOut gw = grad_out(w, w.requires_grad(), w.sizes(), w.options());
    const defer::Scope dsc(gw.claimed);
    auto [dx, dw] = norm::rms_bwd_into(sv[0], dy.contiguous(), opt(ds), w, sv[2], gw.t, gw.bit(1));
    return {dx, add ? dx : Tensor(), gw.t.defined() ? gw.done() : dw, Tensor()};
  }
};

struct LNFn : public torch::autograd::Function<LNFn> {
  static variable_list forward(AutogradContext* ctx, const Tensor& x, const optional<Tensor>& delta, const Tensor& w,
                               const Tensor& b, double eps) {
    at::AutoDispatchBelowADInplaceOrView guard;
    ctx->set_materialize_grads(false);
    auto [y, sum, mean, rstd] = norm::ln_fwd_hip(x, delta, w, b, eps);
    const bool add = delta.has_value();
    ctx->save_for_backward({add ? sum : x, w, mean, rstd});
    ctx->saved_data["add"] = add;
    if (b.requires_grad()) ctx->saved_data["b"] = b;  // (identity only: its gradient's bucket slice)
    if (add) return {sum, y};
    return {y};
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const auto sv = ctx->get_saved_variables();
    const bool add = ctx->saved_data["add"].toBool();
    const Tensor ds = add ? grads[0] : Tensor(), dy = add ? grads[1] : grads[0];
    if (!dy.defined()) return {ds, ds, Tensor(), Tensor(), Tensor()};
    const Tensor& w = sv[1];
    const GradOut gw = grad_out(w, w.requires_grad(), w.sizes(), w.options());
    // the bias is not saved: its slice is looked up through the weight's node input (below)
    const GradOut gb = grad_out(ctx->saved_data.count("b") ? ctx->saved_data["b"].toTensor() : Tensor(), true,
                                w.sizes(), w.options());
    const defer::Scope dsc(gw.claimed && gb.claimed);
    auto [dx, dw, db] = norm::ln_bwd_into(sv[0], dy.contiguous(), opt(ds), w, sv[2], sv[3], gw.t, gb.t,
                                          gw.bit(1) | gb.bit(2));
    return {dx, add ? dx : Tensor(), gw.t.defined() ? gw.done() : dw, gb.t.defined() ? gb.done() : db, Tensor()};
  }
};

// The gradient of an embedding table from the gradient at its gathered rows (ids < V; rows of the
// table past V are padding and get zeros): into the table's DDP bucket slice when it has one — or,
// when a tied LM head already wrote this pass's gradient there, added into it (nothing returned)
static Tensor table_grad(const Tensor& table, const Tensor& dx, const Tensor& ids, int64_t V) {
  const int64_t C = table.size(1);
  const Tensor d2 = dx.reshape({-1, C}).contiguous(), id1 = ids.reshape({-1});
  const Tensor j = graddst::grad_dest_join(table);
  if (j.numel() > 0 && j.scalar_type() == d2.scalar_type()) {
    embed::embedding_bwd_hip(d2, id1, V, j.view(table.sizes()), true);
    return Tensor();
  }
  const GradOut gt = grad_out(table, true, table.sizes(), table.options());
  embed::embedding_bwd_hip(d2, id1, V, gt.t, gt.acc);
  return gt.done();
}

// Token embedding + the first RMSNorm (Llama): one forward launch (norm.hip embed_rms_kernel)
// returning the residual stream x0 and h0 = RMSNorm(x0); in backward the two incoming gradients
// meet here, so the norm's backward adds the residual stream's gradient in its own pass (no
// separate add), and the table's gradient goes straight into its DDP bucket slice (graddst.h).
struct EmbedRMSFn : public torch::autograd::Function<EmbedRMSFn> {
  static variable_list forward(AutogradContext* ctx, const Tensor& ids, const Tensor& table, const Tensor& w,
                               double eps, const optional<Tensor>& err) {
    at::AutoDispatchBelowADInplaceOrView guard;
    ctx->set_materialize_grads(false);
    auto [x0, y, rstd] = norm::embed_rms_fwd_hip(ids, table, w, eps, err);
    ctx->save_for_backward({ids, x0, w, rstd});
    ctx->saved_data["table"] = table;  // (its bucket slice; the values are not read)
    return {x0, y};
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const auto sv = ctx->get_saved_variables();
    const Tensor& ids = sv[0];
    const Tensor& x0 = sv[1];
    const Tensor& w = sv[2];
    const Tensor table = ctx->saved_data["table"].toTensor();
    const Tensor ds = grads[0], dy = grads[1];
    Tensor dx = ds, dw_ret;
    if (dy.defined()) {
      const GradOut gw = grad_out(w, w.requires_grad(), w.sizes(), w.options());
      const defer::Scope dsc(gw.claimed);
      auto [dxx, dw] = norm::rms_bwd_into(x0, dy.contiguous(), opt(ds), w, sv[3], gw.t, gw.bit(1));
      dx = dxx;
      dw_ret = gw.t.defined() ? gw.done() : dw;
    }
    const Tensor dtable = dx.defined() && table.requires_grad() ? table_grad(table, dx, ids, table.size(0)) : Tensor();
    return {Tensor(), dtable, dw_ret, Tensor(), Tensor()};
  }
};

// GPT-2's token + position embedding + the first LayerNorm: one forward launch (norm.hip
// tokpos_ln_kernel); in backward the norm's pass adds the residual stream's gradient, then the
// token table's gradient (bucket slice / tied head: table_grad) and the position table's
// (the batch summed per position, into its slice: embedding_pos_bwd).
struct TokPosLNFn : public torch::autograd::Function<TokPosLNFn> {
  static variable_list forward(AutogradContext* ctx, const Tensor& idx, const Tensor& wte, const Tensor& pos,
                               const Tensor& wpe, const Tensor& w, const Tensor& b, int64_t vocab, double eps,
                               const optional<Tensor>& err) {
    at::AutoDispatchBelowADInplaceOrView guard;
    ctx->set_materialize_grads(false);
    auto [x0, y, mean, rstd] = norm::tokpos_ln_fwd_hip(idx, wte, pos, wpe, vocab, w, b, eps, err);
    ctx->save_for_backward({idx, pos, x0, w, mean, rstd});
    ctx->saved_data["wte"] = wte;  // (identities only: their gradients' bucket slices)
    ctx->saved_data["wpe"] = wpe;
    if (b.requires_grad()) ctx->saved_data["b"] = b;
    ctx->saved_data["V"] = vocab > 0 ? std::min<int64_t>(vocab, wte.size(0)) : wte.size(0);
    return {x0, y};
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const auto sv = ctx->get_saved_variables();
    const Tensor &idx = sv[0], &pos = sv[1], &x0 = sv[2], &w = sv[3];
    const Tensor wte = ctx->saved_data["wte"].toTensor(), wpe = ctx->saved_data["wpe"].toTensor();
    const Tensor ds = grads[0], dy = grads[1];
    Tensor dx = ds, dw_ret, db_ret;
    if (dy.defined()) {
      const GradOut gw = grad_out(w, w.requires_grad(), w.sizes(), w.options());
      const GradOut gb = grad_out(ctx->saved_data.count("b") ? ctx->saved_data["b"].toTensor() : Tensor(), true,
                                  w.sizes(), w.options());
      const defer::Scope dsc(gw.claimed && gb.claimed);
      auto [dxx, dw, db] = norm::ln_bwd_into(x0, dy.contiguous(), opt(ds), w, sv[4], sv[5], gw.t, gb.t,
                                             gw.bit(1) | gb.bit(2));
      dx = dxx;
      dw_ret = gw.t.defined() ? gw.done() : dw;
      db_ret = gb.t.defined() ? gb.done() : db;
    }
    Tensor dwte, dwpe;
    if (dx.defined()) {
      if (wte.requires_grad()) dwte = table_grad(wte, dx, idx, ctx->saved_data["V"].toInt());
      if (wpe.requires_grad()) {
        const int64_t C = wpe.size(1), P = wpe.size(0);
        const Tensor d2 = dx.reshape({-1, C}).contiguous();
        const GradOut gp = grad_out(wpe, true, wpe.sizes(), wpe.options());
        embed::embedding_pos_bwd_hip(d2, pos, P, gp.t, gp.acc);
        dwpe = gp.done();
      }
    }
    return {Tensor(), dwte, Tensor(), dwpe, dw_ret, db_ret, Tensor(), Tensor(), Tensor()};
  }
};

std::tuple<Tensor, Tensor> tokpos_layer_norm_ag(const Tensor& idx, const Tensor& wte, const Tensor& pos,
                                                const Tensor& wpe, const Tensor& w, const Tensor& b, int64_t vocab,
                                                double eps, const optional<Tensor>& err) {
  auto r = TokPosLNFn::apply(idx, wte, pos, wpe, w, b, vocab, eps, err);
  return {r[0], r[1]};
}
std::tuple<Tensor, Tensor> tokpos_layer_norm_noag(const Tensor& idx, const Tensor& wte, const Tensor& pos,
                                                  const Tensor& wpe, const Tensor& w, const Tensor& b, int64_t vocab,
                                                  double eps, const optional<Tensor>& err) {
  auto r = norm::tokpos_ln_fwd_hip(idx, wte, pos, wpe, vocab, w, b, eps, err);
  return {std::get<0>(r), std::get<1>(r)};
}

std::tuple<Tensor, Tensor> embed_rms_norm_ag(const Tensor& ids, const Tensor& table, const Tensor& w, double eps,
                                             const optional<Tensor>& err) {
  auto r = EmbedRMSFn::apply(ids, table, w, eps, err);
  return {r[0], r[1]};
}
std::tuple<Tensor, Tensor> embed_rms_norm_noag(const Tensor& ids, const Tensor& table, const Tensor& w, double eps,
                                               const optional<Tensor>& err) {
  auto r = norm::embed_rms_fwd_hip(ids, table, w, eps, err);
  return {std::get<0>(r), std::get<1>(r)};
}

Tensor rms_norm_ag(const Tensor& x, const Tensor& w, double eps) { return RMSFn::apply(x, c10::nullopt, w, eps)[0]; }
std::tuple<Tensor, Tensor> add_rms_norm_ag(const Tensor& x, const Tensor& delta, const Tensor& w, double eps) {
  auto r = RMSFn::apply(x, optional<Tensor>(delta), w, eps);
  return {r[0], r[1]};
}
Tensor layer_norm_ag(const Tensor& x, const Tensor& w, const Tensor& b, double eps) {
  return LNFn::apply(x, c10::nullopt, w, b, eps)[0];
}
std::tuple<Tensor, Tensor> add_layer_norm_ag(const Tensor& x, const Tensor& delta, const Tensor& w, const Tensor& b,
                                             double eps) {
  auto r = LNFn::apply(x, optional<Tensor>(delta), w, b, eps);
  return {r[0], r[1]};
}
Tensor rms_norm_noag(const Tensor& x, const Tensor& w, double eps) {
  return std::get<0>(norm::rms_fwd_hip(x, c10::nullopt, w, eps));
}
std::tuple<Tensor, Tensor> add_rms_norm_noag(const Tensor& x, const Tensor& delta, const Tensor& w, double eps) {
  auto r = norm::rms_fwd_hip(x, delta, w, eps);
  return {std::get<1>(r), std::get<0>(r)};
}
Tensor layer_norm_noag(const Tensor& x, const Tensor& w, const Tensor& b, double eps) {
  return std::get<0>(norm::ln_fwd_hip(x, c10::nullopt, w, b, eps));
}
std::tuple<Tensor, Tensor> add_layer_norm_noag(const Tensor& x, const Tensor& delta, const Tensor& w, const Tensor& b,
                                               double eps) {
  auto r = norm::ln_fwd_hip(x, delta, w, b, eps);
  return {std::get<1>(r), std::get<0>(r)};
}

// ------------------------------------------------------------------ attention from packed q|k|v
// [B, T, (H + 2·Hkv)·D] in, [B, T, H·D] out; the backward writes the packed gradient directly.
// Python reference: ops/attention.py _FlashAttentionQKV.
static std::tuple<Tensor, Tensor, Tensor> split_qkv(const Tensor& qkv, int64_t H, int64_t Hkv) {
  const int64_t B = qkv.size(0), T = qkv.size(1), D = qkv.size(2) / (H + 2 * Hkv);
  return {qkv.narrow(2, 0, H * D).view({B, T, H, D}).transpose(1, 2),
          qkv.narrow(2, H * D, Hkv * D).view({B, T, Hkv, D}).transpose(1, 2),
          qkv.narrow(2, (H + Hkv) * D, Hkv * D).view({B, T, Hkv, D}).transpose(1, 2)};
}

struct AttnQKVFn : public torch::autograd::Function<AttnQKVFn> {
  static Tensor forward(AutogradContext* ctx, const Tensor& qkv, int64_t H, int64_t Hkv, bool causal, double scale,
                        const optional<Tensor>& cos, const optional<Tensor>& sin) {
    at::AutoDispatchBelowADInplaceOrView guard;
    auto [q, k, v] = split_qkv(qkv, H, Hkv);
    auto [o, lse] = attn::attn_fwd_hip(q, k, v, causal, scale, cos, sin);
    const bool rope = cos.has_value();
    // sequences past two 128-query blocks get the pre-pass (attn.hip: fd off): offer δ to the
    // consumer of the output (adelta above)
    if (adelta::enabled() && q.size(3) == 64 && qkv.size(1) / 128 > 2 && qkv.size(1) % 128 == 0)
      adelta::want(o, qkv.size(1), H);
    if (rope) ctx->save_for_backward({qkv, o, lse, *cos, *sin});
    else ctx->save_for_backward({qkv, o, lse});
    ctx->saved_data["H"] = H;
    ctx->saved_data["Hkv"] = Hkv;
    ctx->saved_data["causal"] = causal;
    ctx->saved_data["scale"] = scale;
    return o.transpose(1, 2).reshape({qkv.size(0), qkv.size(1), -1});  // o is stored [B, T, H, D]: a view
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const auto sv = ctx->get_saved_variables();
    const Tensor &qkv = sv[0], &o = sv[1], &lse = sv[2];
    const bool rope = sv.size() > 3;
    const int64_t H = ctx->saved_data["H"].toInt(), Hkv = ctx->saved_data["Hkv"].toInt();
    const int64_t B = qkv.size(0), T = qkv.size(1), D = qkv.size(2) / (H + 2 * Hkv);
    auto [q, k, v] = split_qkv(qkv, H, Hkv);
    Tensor dqkv = at::empty_like(qkv, at::MemoryFormat::Contiguous);
    auto [dq, dk, dv] = split_qkv(dqkv, H, Hkv);
    const Tensor delta = adelta::enabled() ? adelta::take(o, grads[0]) : Tensor();
    const Tensor dout = grads[0].contiguous().view({B, T, H, D}).transpose(1, 2);
    attn::attn_bwd_hip(dout, q, k, v, o, lse, ctx->saved_data["causal"].toBool(), ctx->saved_data["scale"].toDouble(),
                       dq, dk, dv, rope ? optional<Tensor>(sv[3]) : c10::nullopt,
                       rope ? optional<Tensor>(sv[4]) : c10::nullopt,
                       delta.defined() ? optional<Tensor>(delta) : c10::nullopt);
    return {dqkv, Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

Tensor attn_qkv_ag(const Tensor& qkv, int64_t H, int64_t Hkv, bool causal, double scale, const optional<Tensor>& cos,
                   const optional<Tensor>& sin) {
  return AttnQKVFn::apply(qkv, H, Hkv, causal, scale, cos, sin);
}

Tensor attn_qkv_noag(const Tensor& qkv, int64_t H, int64_t Hkv, bool causal, double scale, const optional<Tensor>& cos,
                     const optional<Tensor>& sin) {
  auto [q, k, v] = split_qkv(qkv, H, Hkv);
  auto [o, lse] = attn::attn_fwd_hip(q, k, v, causal, scale, cos, sin);
  return o.transpose(1, 2).reshape({qkv.size(0), qkv.size(1), -1});
}

// ------------------------------------------------------------ fused Llama decoder block
// One autograd node for a whole pre-norm decoder block of the Llama family:
//   qkv = h·W_qkvᵀ (+b) → causal GQA attention with RoPE → y = a·W_oᵀ (+b)
//   x1 = x + y, h1 = rms(x1)·γ_post → m = down(silu(g)·u), [g|u] = h1·W_guᵀ
//   x2 = x1 + m, h2 = rms(x2)·γ_next                                  → returns (x2, h2)
// The same kernels, in the same order, as the per-op nodes above (Linear, attention, add+RMSNorm,
// SwiGLU MLP: bit-identical results), but one Python call and one autograd node per block instead
// of six and five — an eager SmolLM2 step is host-bound (docs/FINDINGS.md §15, §27).  Weight
// gradients go to their bucket slices (graddst) exactly as in the per-op nodes.
static std::tuple<Tensor, Tensor, Tensor> linear_bwd_core(const Tensor& dy, const Tensor& x2, const Tensor& w,
                                                          const Tensor& b, at::IntArrayRef plan, bool nx, bool nw,
                                                          bool nb) {
  Tensor dx, dw, db;
  if (nx && nw && plan[9] >= 0) {
    std::tie(dx, dw, db) = pair(dy, w, x2, EPI_NONE, c10::nullopt, nb, plan[9], b);
  } else {
    if (nx) dx = run(dy, w, false, true, prod(plan, 1)).first;
    if (nw) std::tie(dw, db) = wgrad(dy, x2, w, b, nb, plan, 2);
    else if (nb) db = dy.sum(0, false, at::kFloat).to(dy.scalar_type());
  }
  return {dx, dw, db};
}

// (dh, dW_gu, dW_down) of m = down(silu(g)·u), [g|u] = h·W_guᵀ, for dm [M, C]
static std::tuple<Tensor, Tensor, Tensor> swiglu_bwd_core(const Tensor& dm, const Tensor& x2, const Tensor& w_gu,
                                                          const Tensor& w_down, const Tensor& pre, const Tensor& act,
                                                          at::IntArrayRef plan, bool nx) {
  Tensor dgu, dw_down, dx, dw_gu, unused;
  if (plan[18] >= 0) {
    std::tie(dgu, dw_down, unused) = pair(dm, w_down, act, EPI_DSWIGLU, pre, false, plan[18]);
  } else {
    dgu = run(dm, w_down, false, true, prod(plan, 2), EPI_DSWIGLU, c10::nullopt, pre).first;
    dw_down = wgrad(dm, act, w_down, Tensor(), false, plan, 3).first;
  }
  if (nx && plan[19] >= 0) {
    std::tie(dx, dw_gu, unused) = pair(dgu, w_gu, x2, EPI_NONE, c10::nullopt, false, plan[19]);
  } else {
    if (nx) dx = run(dgu, w_gu, false, true, prod(plan, 4)).first;
    dw_gu = wgrad(dgu, x2, w_gu, Tensor(), false, plan, 5).first;
  }
  return {dx, dw_gu, dw_down};
}

// (d sum, dγ) of (s = x + δ, y = rms(s)·γ) for dy and the sum's own gradient ds (may be undefined)
static std::pair<Tensor, Tensor> rms_bwd_core(const Tensor& s, const Tensor& dy, const Tensor& ds, const Tensor& w,
                                              const Tensor& rstd) {
  const GradOut gw = grad_out(w, w.requires_grad(), w.sizes(), w.options());
  const defer::Scope dsc(gw.claimed);
  auto [dx, dw] = norm::rms_bwd_into(s, dy.contiguous(), opt(ds), w, rstd, gw.t, gw.bit(1));
  return {dx, gw.t.defined() ? gw.done() : dw};
}

static Tensor attn_bwd_core(const Tensor& da, const Tensor& qkv, const Tensor& o, const Tensor& lse, int64_t H,
                            int64_t Hkv, double scale, const optional<Tensor>& cos, const optional<Tensor>& sin) {
  const int64_t B = qkv.size(0), T = qkv.size(1), D = qkv.size(2) / (H + 2 * Hkv);
  auto [q, k, v] = split_qkv(qkv, H, Hkv);
  Tensor dqkv = at::empty_like(qkv, at::MemoryFormat::Contiguous);
  auto [dq, dk, dv] = split_qkv(dqkv, H, Hkv);
  const Tensor dout = da.contiguous().view({B, T, H, D}).transpose(1, 2);
  {
    const ht::Scope hs(ht::ATTN_CALL);
    attn::attn_bwd_hip(dout, q, k, v, o, lse, true, scale, dq, dk, dv, cos, sin);
  }
  return dqkv;
}

// forward of the block; `save` (autograd) receives what the backward needs
static std::tuple<Tensor, Tensor> llama_block_fwd(const Tensor& x, const Tensor& h, const Tensor& w_qkv,
                                                  const optional<Tensor>& b_qkv, const Tensor& w_o,
                                                  const optional<Tensor>& b_o, const Tensor& w_post,
                                                  const Tensor& w_gu, const Tensor& w_down, const Tensor& w_next,
                                                  at::IntArrayRef plan_qkv, at::IntArrayRef plan_o,
                                                  at::IntArrayRef plan_mlp, int64_t H, int64_t Hkv, double scale,
                                                  double eps, const optional<Tensor>& cos, const optional<Tensor>& sin,
                                                  std::vector<Tensor>* save) {
  const int64_t B = h.size(0), T = h.size(1), C = h.size(2);
  const Tensor h2 = bf16c(h).view({-1, C});
  const Tensor qkv = linear_forward(h2, w_qkv, b_qkv, plan_qkv).view({B, T, -1});
  auto [q, k, v] = split_qkv(qkv, H, Hkv);
  auto [o, lse] = attn::attn_fwd_hip(q, k, v, true, scale, cos, sin);
  const Tensor a2 = o.transpose(1, 2).reshape({B * T, -1});  // o is stored [B, T, H, D]: a view
  const Tensor y = linear_forward(a2, w_o, b_o, plan_o).view({B, T, C});
  auto [h1, x1, rstd1] = norm::rms_fwd_hip(bf16c(x), y, w_post, eps);
  const Tensor h1f = h1.view({-1, C});
  auto [act, pre] = run(h1f, w_gu, false, false, prod(plan_mlp, 0), EPI_SWIGLU);
  const Tensor m = run(act, w_down, false, false, prod(plan_mlp, 1)).first.view({B, T, C});
  auto [h_out, x_out, rstd2] = norm::rms_fwd_hip(x1, m, w_next, eps);
  if (save != nullptr) {
    *save = {h2, w_qkv, b_qkv ? *b_qkv : Tensor(), qkv, o, lse, w_o, b_o ? *b_o : Tensor(), x1, w_post,
             rstd1, h1f, w_gu, w_down, pre, act, x_out, w_next, rstd2, cos ? *cos : Tensor(), sin ? *sin : Tensor()};
  }
  return {x_out, h_out};
}

// ---- one HIP graph per decoder block for the EAGER step (opt-in: NBD_BLOCK_GRAPHS=1 or
// torch.ops.nbd.llama_block_graphs(1)).  The block's forward — seven kernels plus allocations,
// ≈70 µs of issuing-thread time on SmolLM2 (docs/FINDINGS.md §27) — is captured once per
// (block, shape) after two eager calls and then replayed: one graph launch instead of seven
// kernel launches.  The graph writes its activations into static memory (its private pool), so:
//  * the block's inputs are copied into static buffers, except when they ARE another block
//    graph's outputs (the residual stream between consecutive graphed blocks needs no copy);
//  * the static memory may be replayed into only once the previous pass's autograd node has let
//    go of it: a token among the node's saved tensors clears `armed` when backward releases the
//    saved tensors (or the node dies).  A forward while the block is armed (a second forward
//    before backward, retain_graph) runs eagerly, as does any call whose weights, RoPE tables or
//    aliased input moved, or that comes inside another capture (graphs.GraphedStep);
//  * the returned tensors alias that memory: they hold this pass's values until the block's next
//    replay (a caller keeping block outputs across steps must clone them);
//  * each (block, shape) keeps its activations allocated between steps: at most 4 shapes per block
//    are graphed, further sequence lengths run eagerly.
// The backward of a graph-forwarded block is captured too (its first graphed backward) when every
// weight gradient goes to a DDP bucket slice (graddst.h): the claims made during the capture are
// recorded, and a replay first checks that each parameter's destination (and whether it
// accumulates, no_sync) is still the captured one — peek(), no side effects — then claims them
// (the pass bookkeeping) and hands the slices back as the weight gradients.  One backward graph per
// accumulate pattern; the deferred reductions of the capture are recorded and queued after each
// replay, so they join the backward's single flush.  Without bucket slices
// (plain training) the backward stays eager: a graph's weight gradients would be static memory
// that AccumulateGrad keeps as .grad.
// Same kernels, same order: bit-identical to the eager block (tests/test_gpu_block_graphs.py).
namespace bg {
using Key = std::tuple<const void*, int64_t, int64_t, int64_t>;  // (W_qkv, B, T, device)

struct Bwd {
  std::unique_ptr<at::cuda::CUDAGraph> g;
  Tensor dx_in, dh_in;                    // static inputs (the incoming gradients)
  bool dx_alias = false, dh_alias = false;  // ...that are another block graph's outputs
  Tensor g1, dh;                          // static outputs: the gradients of x and h
  std::vector<graddst::ClaimRecord> claims;  // in capture order
  std::vector<int> pidx;                  // the saved parameter each claim was made for (by position:
                                          // native()'s cast weights are new tensors every step)
  std::vector<int> slot;                  // the node output each claim's slice is returned as
  std::vector<Tensor> warm_refs;
  std::shared_ptr<void> deferred;          // its deferred reductions (defer::record_begin)
};
struct Graph {
  std::unique_ptr<at::cuda::CUDAGraph> g;
  Tensor x_in, h_in;                   // static inputs
  bool x_alias = false, h_alias = false;  // ...that are another block graph's outputs
  std::vector<const void*> ptrs;       // weights, RoPE tables at capture
  std::vector<int64_t> sig;            // their shapes and the block's scalars
  std::vector<Tensor> saved;           // llama_block_fwd's saved list (static; weight slots empty)
  Tensor x_out, h_out;
  std::vector<Tensor> warm_refs;       // storages the captured GEMM warm-ups read
  std::atomic<bool> armed{false};
  int64_t id = 0;
  Key key{};
  std::map<int, std::shared_ptr<Bwd>> bwd;  // key: accumulate mask | need bits
  int bwd_captures = 0;
  bool bwd_off = false;
  // the static output at `p` (forward or backward), or nullptr
  const Tensor* output_at(const void* p) const {
    if (x_out.defined() && x_out.data_ptr() == p) return &x_out;
    if (h_out.defined() && h_out.data_ptr() == p) return &h_out;
    for (const auto& kv : bwd) {
      if (kv.second->g1.defined() && kv.second->g1.data_ptr() == p) return &kv.second->g1;
      if (kv.second->dh.defined() && kv.second->dh.data_ptr() == p) return &kv.second->dh;
    }
    return nullptr;
  }
};
// A block call's arguments, kept (strong references) so that a stack capture can re-run it.
struct Args {
  Tensor w_qkv, w_o, w_post, w_gu, w_down, w_next;
  optional<Tensor> b_qkv, b_o, cos, sin;
  std::vector<int64_t> plan_qkv, plan_o, plan_mlp;
  int64_t H = 0, Hkv = 0;
  double scale = 0, eps = 0;
};

// Stack graphs (mode 1): every graph launch costs the GPU ≈8.5 µs of its own
// (benchmarks/graph_chunks.py), so once a run of consecutive graphed blocks has replayed
// steadily — each block's input the previous block's static output — the whole run is captured
// as ONE graph, replayed at its first block's call; the following blocks' calls, arriving in the
// recorded order with the recorded weights and the stack's outputs as inputs, are served from it
// without a launch.  Any deviation drops the stack (back to per-block graphs).
struct StackMember {
  Key key;
  std::vector<const void*> ptrs;
  std::vector<int64_t> sig;
  std::vector<Tensor> saved;  // weight slots empty
  Tensor x_out, h_out;
};
// Casts of fp32 master weights into kept compute-dtype buffers (CastGroupFn) since process start.
// A stack replays every member at the head's call, so a cast between two member calls would be
// read one step late: serving checks that none ran since the head's replay.
std::atomic<uint64_t> g_cast_epoch{0};

struct Stack {
  std::unique_ptr<at::cuda::CUDAGraph> g;
  Tensor x_in, h_in;
  uint64_t cast_epoch = 0;     // g_cast_epoch at the head's replay
  std::vector<StackMember> m;
  std::vector<Tensor> warm_refs;
  size_t next = 0;             // members served in the current pass
  std::atomic<int> held{0};    // served members whose autograd nodes still hold the memory
  Key head{};
  int64_t owner = 0;           // the head slot's owner (per-model reset)
};

struct Slot {
  int64_t owner = 0;  // the model that made the calls (LlamaModel's id; per-model reset)
  int eager = 0, captures = 0, misses = 0;
  bool off = false;
  std::shared_ptr<Graph> g;
  std::shared_ptr<Args> args;  // (stack capture)
  Key next_key{};              // the block that consumed this block's outputs last pass
  bool has_next = false;
  int steady = 0;              // consecutive per-block replays
  std::shared_ptr<Stack> stack;  // a stack headed by this block
  int stack_fail = 0;
};
std::mutex g_mu;
std::map<Key, Slot> g_slots;
std::unordered_map<const void*, std::weak_ptr<Graph>> g_outs;  // a graph's output address -> graph
std::unordered_map<int64_t, std::weak_ptr<Graph>> g_by_id;      // for the backward
int64_t g_next_id = 1;
std::atomic<int> g_mode{-1};                                    // -1: not read from the env yet
std::atomic<bool> g_suspended{false};                           // overrides per-model modes too
// forward captures, replays, eager calls; backward captures, replays, eager calls
std::atomic<int64_t> g_stat[10];  // + stack captures, stack replays, stack-served blocks, stacks dropped
std::weak_ptr<Stack> g_active;    // the stack serving the current pass
std::atomic<int> g_fail_bwd{0};   // fault injection (tests): fail this many backward captures

// 0 off, 1 forward graphs, 2 forward and backward graphs (NBD_BLOCK_GRAPHS)
int mode() {
  int m = g_mode.load(std::memory_order_relaxed);
  if (m < 0) {
    const char* e = std::getenv("NBD_BLOCK_GRAPHS");
    m = e != nullptr && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
    g_mode.store(m, std::memory_order_relaxed);
  }
  return m;
}
bool enabled() { return mode() >= 1; }
bool stacks_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NBD_BLOCK_STACKS");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}
bool bwd_enabled() { return mode() >= 2; }

bool stream_capturing() {
  hipStreamCaptureStatus s = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(), &s) != hipSuccess) return true;
  return s != hipStreamCaptureStatusNone;
}

// x is an output of a live block graph (so it stays put while that graph lives); under g_mu
bool is_graph_output(const Tensor& x) {
  if (!x.is_contiguous()) return false;
  auto it = g_outs.find(x.data_ptr());
  if (it == g_outs.end()) return false;
  auto gr = it->second.lock();
  if (!gr) return false;
  const Tensor* o = gr->output_at(x.data_ptr());
  return o != nullptr && o->numel() == x.numel() && o->scalar_type() == x.scalar_type();
}

// Capture `body` into `g` on a side stream ordered after the caller's stream, which then waits
// for it.  Returns the error ("" = captured).
// A stream of our own per device for the captures: a pool stream could be the one a process
// group's collectives run on (ProcessGroupNCCL takes its streams from the same pool).
c10::hip::HIPStreamMasqueradingAsCUDA capture_stream(c10::DeviceIndex dev) {
  static std::mutex mu;
  static std::unordered_map<int, hipStream_t> streams;
  std::lock_guard<std::mutex> lk(mu);
  hipStream_t& st = streams[dev];
  if (st == nullptr) {
    const c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, dev));
    C10_HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  }
  return c10::hip::getStreamFromExternalMasqueradingAsCUDA(st, dev);
}

std::string capture(at::cuda::CUDAGraph& g, const std::function<void()>& body) {
  auto cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA();
  auto side = capture_stream(cur.device_index());
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  C10_HIP_CHECK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
  C10_HIP_CHECK(hipEventCreateWithFlags(&ev_out, hipEventDisableTiming));
  C10_HIP_CHECK(hipEventRecord(ev_in, cur.stream()));
  C10_HIP_CHECK(hipStreamWaitEvent(side.stream(), ev_in, 0));
  std::string err;
  {
    const c10::hip::HIPStreamGuardMasqueradingAsCUDA sg(side);
    g.capture_begin(at::cuda::graph_pool_handle(), hipStreamCaptureModeThreadLocal);
    try {
      body();
    } catch (const std::exception& e) {
      err = e.what();
    }
    try {
      g.capture_end();
    } catch (const std::exception& e) {
      if (err.empty()) err = e.what();
    }
  }
  C10_HIP_CHECK(hipEventRecord(ev_out, side.stream()));
  C10_HIP_CHECK(hipStreamWaitEvent(cur.stream(), ev_out, 0));
  C10_HIP_CHECK(hipEventDestroy(ev_in));
  C10_HIP_CHECK(hipEventDestroy(ev_out));
  return err;
}

// a CPU scalar whose release (backward done with the saved tensors, or the node gone) disarms
Tensor token(const std::shared_ptr<Graph>& gr) {
  static int64_t dummy = 0;
  std::weak_ptr<Graph> w = gr;
  return at::from_blob(
      &dummy, {1},
      [w](void*) {
        if (auto g = w.lock()) g->armed.store(false, std::memory_order_release);
      },
      at::TensorOptions().dtype(at::kLong));
}
std::vector<std::shared_ptr<Stack>> g_dropped;  // dropped stacks: a replay may still be in flight

// under g_mu: the block whose static output `x` is now feeds block `key`
void link_pred(const Tensor& x, const Key& key) {
  auto it = g_outs.find(x.data_ptr());
  if (it == g_outs.end()) return;
  auto pg = it->second.lock();
  if (!pg) return;
  auto ps = g_slots.find(pg->key);
  if (ps == g_slots.end()) return;
  ps->second.next_key = key;
  ps->second.has_next = true;
}

// under g_mu: stop serving `st` (its head slot captures no new stack after two failures)
void drop_stack(const std::shared_ptr<Stack>& st, const Key& head) {
  auto it = g_slots.find(head);
  if (it != g_slots.end() && it->second.stack == st) {
    it->second.stack.reset();
    ++it->second.stack_fail;
  }
  if (g_active.lock() == st) g_active.reset();
  g_dropped.push_back(st);
  if (g_dropped.size() > 8) g_dropped.erase(g_dropped.begin());
  ++g_stat[9];
}

Tensor stack_token(const std::shared_ptr<Stack>& st) {
  static int64_t dummy = 0;
  std::weak_ptr<Stack> w = st;
  return at::from_blob(
      &dummy, {1},
      [w](void*) {
        if (auto s = w.lock()) s->held.fetch_sub(1, std::memory_order_acq_rel);
      },
      at::TensorOptions().dtype(at::kLong));
}
}  // namespace bg

namespace castbuf {  // (below, with the cast node)
bool kept(const Tensor& t);
// the warm-up references minus kept cast buffers: the cache keeps those alive, and a graph
// holding them would make them look in use forever
std::vector<Tensor> drop_kept(std::vector<Tensor> refs);
}  // namespace castbuf

// saved-list slots holding the call's weights / RoPE tables (the node's gradient targets)
constexpr int kBlockWeightSlots[] = {1, 2, 6, 7, 9, 12, 13, 17, 19, 20};

// Replay (or capture, then replay) the block's graph for this call; nullptr = run it eagerly.
static std::shared_ptr<bg::Graph> block_graph(const Tensor& x, const Tensor& h, const Tensor& w_qkv,
                                              const optional<Tensor>& b_qkv, const Tensor& w_o,
                                              const optional<Tensor>& b_o, const Tensor& w_post, const Tensor& w_gu,
                                              const Tensor& w_down, const Tensor& w_next, at::IntArrayRef plan_qkv,
                                              at::IntArrayRef plan_o, at::IntArrayRef plan_mlp, int64_t H,
                                              int64_t Hkv, double scale, double eps, const optional<Tensor>& cos,
                                              const optional<Tensor>& sin, int64_t owner) {
  using namespace bg;
  if (stream_capturing()) return nullptr;  // inside a whole-step capture: the outer graph takes it
  const Tensor* ts[] = {&w_qkv, b_qkv ? &*b_qkv : nullptr, &w_o, b_o ? &*b_o : nullptr, &w_post, &w_gu,
                        &w_down, &w_next, cos ? &*cos : nullptr, sin ? &*sin : nullptr};
  std::vector<const void*> ptrs;
  std::vector<int64_t> sig{H, Hkv, (int64_t)(scale * 1e9), (int64_t)(eps * 1e12), (int64_t)x.scalar_type()};
  for (const Tensor* t : ts) {
    ptrs.push_back(t != nullptr ? t->data_ptr() : nullptr);
    if (t != nullptr) sig.insert(sig.end(), t->sizes().begin(), t->sizes().end());
    sig.push_back(-1);
  }
  for (at::IntArrayRef p : {plan_qkv, plan_o, plan_mlp}) sig.insert(sig.end(), p.begin(), p.end());
  const Key key{w_qkv.data_ptr(), h.size(0), h.size(1), h.get_device()};
  auto make_args = [&] {
    // variable_data(): the data only — a registry holding a cast weight's autograd history would
    // keep that pass's AccumulateGrad nodes alive (the stream hazard of x_in below)
    auto vd = [](const optional<Tensor>& t) { return t ? optional<Tensor>(t->variable_data()) : c10::nullopt; };
    auto a = std::make_shared<Args>();
    a->w_qkv = w_qkv.variable_data(), a->w_o = w_o.variable_data(), a->w_post = w_post.variable_data();
    a->w_gu = w_gu.variable_data(), a->w_down = w_down.variable_data(), a->w_next = w_next.variable_data();
    a->b_qkv = vd(b_qkv), a->b_o = vd(b_o), a->cos = vd(cos), a->sin = vd(sin);
    a->plan_qkv = plan_qkv.vec(), a->plan_o = plan_o.vec(), a->plan_mlp = plan_mlp.vec();
    a->H = H, a->Hkv = Hkv, a->scale = scale, a->eps = eps;
    return a;
  };
  std::shared_ptr<Graph> gr;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    Slot& s = g_slots[key];
    s.owner = owner;
    if (s.off) return nullptr;
    if (s.g && (s.g->ptrs != ptrs || s.g->sig != sig)) s.g.reset(), s.eager = 0, s.args.reset(), s.steady = 0;
    if (s.g) {
      Graph& G = *s.g;
      const bool inputs_ok = (!G.x_alias || x.data_ptr() == G.x_in.data_ptr()) &&
                             (!G.h_alias || h.data_ptr() == G.h_in.data_ptr());
      if (!inputs_ok) {  // the block before ran eagerly this time; twice in a row: capture anew
        if (++s.misses >= 2) s.g.reset(), s.eager = 0, s.misses = 0;
        ++g_stat[2];
        return nullptr;
      }
      if (G.armed.exchange(true, std::memory_order_acq_rel)) {  // last pass still holds the memory
        ++g_stat[2];
        return nullptr;
      }
      s.misses = 0;
      ++s.steady;
      if (!s.args) s.args = make_args();
      if (G.x_alias) link_pred(x, key);
      gr = s.g;
    } else if (++s.eager < 3) {
      ++g_stat[2];
      return nullptr;
    } else if (++s.captures > 4) {
      s.off = true;
      return nullptr;
    } else {
      // each (block, shape) keeps its activations: a model fed many sequence lengths (dynamic
      // padding) would grow without bound — at most kMaxShapes graphs per block, the rest eager
      // (and at most kMaxLive graphs in all: weights that move every step — per-forward casts
      // landing at new addresses — must not capture without bound either)
      constexpr int kMaxShapes = 4, kMaxLive = 512;
      int shapes = 0, live = 0;
      for (const auto& kv : g_slots) {
        live += kv.second.g != nullptr;
        shapes += std::get<0>(kv.first) == std::get<0>(key) && std::get<3>(kv.first) == std::get<3>(key) &&
                  kv.second.g != nullptr;
      }
      if (shapes >= kMaxShapes || live >= kMaxLive) {
        s.off = true;
        ++g_stat[2];
        return nullptr;
      }
    }
  }
  if (gr) {
    if (!gr->x_alias && x.data_ptr() != gr->x_in.data_ptr()) gr->x_in.copy_(x);
    if (!gr->h_alias && h.data_ptr() != gr->h_in.data_ptr()) gr->h_in.copy_(h);
    gr->g->replay();
    ++g_stat[1];
    return gr;
  }
  // capture on a side stream, then replay once on the caller's stream (capturing runs nothing)
  auto G = std::make_shared<Graph>();
  G->ptrs = std::move(ptrs);
  G->sig = std::move(sig);
  {
    std::lock_guard<std::mutex> lk(g_mu);
    G->x_alias = is_graph_output(x);
    G->h_alias = is_graph_output(h);
  }
  // (variable_data: the graph must not hold the caller's autograd history — an aliased input is
  // the previous block's output, whose node would keep this pass's AccumulateGrad nodes alive)
  G->x_in = G->x_alias ? x.variable_data() : at::empty_like(x, at::MemoryFormat::Contiguous).copy_(x);
  G->h_in = G->h_alias ? h.variable_data() : at::empty_like(h, at::MemoryFormat::Contiguous).copy_(h);
  std::vector<Tensor> save;
  G->g = std::make_unique<at::cuda::CUDAGraph>();
  const std::string err = capture(*G->g, [&] {
    std::tie(G->x_out, G->h_out) = llama_block_fwd(G->x_in, G->h_in, w_qkv, b_qkv, w_o, b_o, w_post, w_gu, w_down,
                                                   w_next, plan_qkv, plan_o, plan_mlp, H, Hkv, scale, eps, cos, sin,
                                                   &save);
  });
  G->warm_refs = castbuf::drop_kept(gemm::gemm_warm_take_refs());
  if (!err.empty()) {
    TORCH_WARN_ONCE("nbd: a decoder block's HIP graph capture failed (", err, "); the block runs eagerly");
    std::lock_guard<std::mutex> lk(g_mu);
    g_slots[key].off = true;
    return nullptr;
  }
  for (int i : kBlockWeightSlots) save[i] = Tensor();
  G->saved = std::move(save);
  G->armed.store(true, std::memory_order_release);
  G->g->replay();
  ++g_stat[0];
  ++g_stat[1];
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto it = g_outs.begin(); it != g_outs.end();) it = it->second.expired() ? g_outs.erase(it) : std::next(it);
  for (auto it = g_by_id.begin(); it != g_by_id.end();) it = it->second.expired() ? g_by_id.erase(it) : std::next(it);
  g_outs[G->x_out.data_ptr()] = G;
  g_outs[G->h_out.data_ptr()] = G;
  G->id = g_next_id++;
  G->key = key;
  g_by_id[G->id] = G;
  Slot& s = g_slots[key];
  s.g = G;
  s.misses = 0;
  s.steady = 0;
  s.args = make_args();
  if (G->x_alias) link_pred(x, key);
  return G;
}

// A stack graph for this call (see bg::Stack): the head's call replays it, the following blocks'
// calls are served from it.  {nullptr, 0} = not served (per-block path).
static std::pair<std::shared_ptr<bg::Stack>, size_t> stack_serve(
    const Tensor& x, const Tensor& h, const Tensor& w_qkv, const optional<Tensor>& b_qkv, const Tensor& w_o,
    const optional<Tensor>& b_o, const Tensor& w_post, const Tensor& w_gu, const Tensor& w_down, const Tensor& w_next,
    at::IntArrayRef plan_qkv, at::IntArrayRef plan_o, at::IntArrayRef plan_mlp, int64_t H, int64_t Hkv, double scale,
    double eps, const optional<Tensor>& cos, const optional<Tensor>& sin) {
  using namespace bg;
  if (stream_capturing()) return {nullptr, 0};
  const Tensor* ts[] = {&w_qkv, b_qkv ? &*b_qkv : nullptr, &w_o, b_o ? &*b_o : nullptr, &w_post, &w_gu,
                        &w_down, &w_next, cos ? &*cos : nullptr, sin ? &*sin : nullptr};
  std::vector<const void*> ptrs;
  std::vector<int64_t> sig{H, Hkv, (int64_t)(scale * 1e9), (int64_t)(eps * 1e12), (int64_t)x.scalar_type()};
  for (const Tensor* t : ts) {
    ptrs.push_back(t != nullptr ? t->data_ptr() : nullptr);
    if (t != nullptr) sig.insert(sig.end(), t->sizes().begin(), t->sizes().end());
    sig.push_back(-1);
  }
  for (at::IntArrayRef p : {plan_qkv, plan_o, plan_mlp}) sig.insert(sig.end(), p.begin(), p.end());
  const Key key{w_qkv.data_ptr(), h.size(0), h.size(1), h.get_device()};
  std::lock_guard<std::mutex> lk(g_mu);
  // 1. the next member of the stack serving this pass
  if (auto st = g_active.lock()) {
    if (st->next > 0 && st->next < st->m.size()) {
      StackMember& mb = st->m[st->next];
      const StackMember& prev = st->m[st->next - 1];
      if (mb.key == key && mb.ptrs == ptrs && mb.sig == sig && x.data_ptr() == prev.x_out.data_ptr() &&
          h.data_ptr() == prev.h_out.data_ptr()) {
        // the replay already ran this member on the weights as they were at the head's call
        TORCH_CHECK(g_cast_epoch.load(std::memory_order_acquire) == st->cast_epoch,
                    "nbd: a decoder block's weights were cast after its stack graph had replayed (the block would "
                    "read the previous values): cast every layer before the first block (models/llama.py "
                    "_forward_cast), or turn block graphs off (NBD_BLOCK_GRAPHS=0)");
        st->held.fetch_add(1, std::memory_order_acq_rel);
        ++g_stat[8];
        return {st, st->next++};
      }
      drop_stack(st, st->head);  // the pass left the recorded order
    }
  }
  // 2. the head of a stack
  auto it = g_slots.find(key);
  if (it == g_slots.end()) return {nullptr, 0};
  Slot& s = it->second;
  if (!s.stack) {
    // 3. capture one: a steadily replaying chain of >= 2 graphed blocks starting here
    if (!s.g || s.g->x_alias || s.g->ptrs != ptrs || s.g->sig != sig) return {nullptr, 0};
    if (s.stack_fail >= 2 || s.steady < 3 || !s.args) return {nullptr, 0};
    std::vector<Key> chain{key};
    for (Key k = key; chain.size() < 256;) {
      const Slot& cs = g_slots[k];
      if (!cs.has_next) break;
      auto nit = g_slots.find(cs.next_key);
      if (nit == g_slots.end() || !nit->second.g || !nit->second.args || nit->second.steady < 3 ||
          !nit->second.g->x_alias || std::find(chain.begin(), chain.end(), cs.next_key) != chain.end())
        break;
      chain.push_back(cs.next_key);
      k = cs.next_key;
    }
    if (chain.size() < 2) return {nullptr, 0};
    auto st = std::make_shared<Stack>();
    st->head = key;
    st->owner = s.owner;
    st->x_in = at::empty_like(x, at::MemoryFormat::Contiguous);
    st->h_in = at::empty_like(h, at::MemoryFormat::Contiguous);
    st->m.resize(chain.size());
    std::vector<std::shared_ptr<Args>> args;
    for (size_t i = 0; i < chain.size(); ++i) {
      const Slot& cs = g_slots[chain[i]];
      st->m[i].key = chain[i];
      st->m[i].ptrs = cs.g->ptrs;
      st->m[i].sig = cs.g->sig;
      args.push_back(cs.args);
    }
    st->g = std::make_unique<at::cuda::CUDAGraph>();
    const std::string err = capture(*st->g, [&] {
      Tensor cx = st->x_in, ch = st->h_in;
      for (size_t i = 0; i < args.size(); ++i) {
        const Args& a = *args[i];
        std::vector<Tensor> save;
        std::tie(st->m[i].x_out, st->m[i].h_out) =
            llama_block_fwd(cx, ch, a.w_qkv, a.b_qkv, a.w_o, a.b_o, a.w_post, a.w_gu, a.w_down, a.w_next, a.plan_qkv,
                            a.plan_o, a.plan_mlp, a.H, a.Hkv, a.scale, a.eps, a.cos, a.sin, &save);
        for (int j : kBlockWeightSlots) save[j] = Tensor();
        st->m[i].saved = std::move(save);
        cx = st->m[i].x_out;
        ch = st->m[i].h_out;
      }
    });
    st->warm_refs = castbuf::drop_kept(gemm::gemm_warm_take_refs());
    if (!err.empty()) {
      ++s.stack_fail;
      TORCH_WARN_ONCE("nbd: a stack of decoder-block graphs failed to capture (", err, "); per-block graphs stay");
      return {nullptr, 0};
    }
    ++g_stat[6];
    s.stack = st;
    // the members' own graphs are not replayed while the stack serves: free their static memory
    // (a block the stack stops serving captures its own graph again after two eager calls)
    for (const Key& k : chain) {
      Slot& ms = g_slots[k];
      ms.g.reset();
      ms.eager = 0;
      ms.steady = 0;
    }
  }
  Stack& st = *s.stack;
  if (st.m[0].ptrs != ptrs || st.m[0].sig != sig) {
    drop_stack(s.stack, key);
    return {nullptr, 0};
  }
  if (st.held.load(std::memory_order_acquire) != 0) return {nullptr, 0};  // the last pass still holds it
  if (st.x_in.data_ptr() != x.data_ptr()) st.x_in.copy_(x);
  if (st.h_in.data_ptr() != h.data_ptr()) st.h_in.copy_(h);
  st.g->replay();
  st.next = 1;
  st.cast_epoch = g_cast_epoch.load(std::memory_order_acquire);
  st.held.store(1, std::memory_order_release);
  g_active = s.stack;
  ++g_stat[7];
  return {s.stack, 0};
}

// The block's backward into `out` (the node's 20 outputs).
static void block_bwd(const std::vector<Tensor>& sv, const std::array<at::IntArrayRef, 3>& plans, int64_t H,
                      int64_t Hkv, double scale, const std::vector<int64_t>& shape, bool need_x, bool need_h,
                      const Tensor& dx_out, const Tensor& dh_out, variable_list& out) {
  const Tensor &h2 = sv[0], &w_qkv = sv[1], &b_qkv = sv[2], &qkv = sv[3], &o = sv[4], &lse = sv[5], &w_o = sv[6],
               &b_o = sv[7], &x1 = sv[8], &w_post = sv[9], &rstd1 = sv[10], &h1f = sv[11], &w_gu = sv[12],
               &w_down = sv[13], &pre = sv[14], &act = sv[15], &x_out = sv[16], &w_next = sv[17], &rstd2 = sv[18];
  const optional<Tensor> cos = sv[19].defined() ? optional<Tensor>(sv[19]) : c10::nullopt;
  const optional<Tensor> sin = sv[20].defined() ? optional<Tensor>(sv[20]) : c10::nullopt;
  const int64_t C = shape[2];
  // x2 = x1 + m, h2 = rms(x2)·γ_next
  Tensor g2, dw_next;
  {
    const ht::Scope hs(ht::RMS_NEXT);
    if (dh_out.defined()) std::tie(g2, dw_next) = rms_bwd_core(x_out, dh_out, dx_out, w_next, rstd2);
    else g2 = dx_out;
  }
  if (!g2.defined()) return;  // neither output reached the loss
  // m = down(swiglu(h1·W_guᵀ))
  Tensor dh1, dw_gu, dw_down;
  {
    const ht::Scope hs(ht::SWIGLU);
    std::tie(dh1, dw_gu, dw_down) = swiglu_bwd_core(bf16c(g2).view({-1, C}), h1f, w_gu, w_down, pre, act, plans[2], true);
  }
  // x1 = x + y, h1 = rms(x1)·γ_post
  Tensor g1, dw_post;
  {
    const ht::Scope hs(ht::RMS_POST);
    std::tie(g1, dw_post) = rms_bwd_core(x1, dh1.view(shape), g2, w_post, rstd1);
  }
  // y = a·W_oᵀ (+b)
  Tensor da, dw_o, db_o;
  {
    const ht::Scope hs(ht::LIN_O);
    const Tensor a2 = o.transpose(1, 2).reshape({h2.size(0), -1});
    std::tie(da, dw_o, db_o) = linear_bwd_core(bf16c(g1).view({-1, C}), a2, w_o, b_o, plans[1], true,
                                               w_o.requires_grad(), b_o.defined() && b_o.requires_grad());
  }
  Tensor dqkv;
  {
    const ht::Scope hs(ht::ATTN);
    dqkv = attn_bwd_core(da, qkv, o, lse, H, Hkv, scale, cos, sin);
  }
  Tensor dh, dw_qkv, db_qkv;
  {
    const ht::Scope hs(ht::LIN_QKV);
    std::tie(dh, dw_qkv, db_qkv) = linear_bwd_core(dqkv.view({h2.size(0), -1}), h2, w_qkv, b_qkv, plans[0], need_h,
                                                   w_qkv.requires_grad(), b_qkv.defined() && b_qkv.requires_grad());
  }
  out[0] = need_x ? g1 : Tensor();
  out[1] = dh.defined() ? dh.view(shape) : dh;
  out[2] = dw_qkv;
  out[3] = db_qkv;
  out[4] = dw_o;
  out[5] = db_o;
  out[6] = dw_post;
  out[7] = dw_gu;
  out[8] = dw_down;
  out[9] = dw_next;
}

// The block's backward as a HIP graph (see namespace bg); false = run it eagerly.
static bool block_bwd_graph(bg::Graph& G, const std::vector<Tensor>& sv,
                            const std::array<at::IntArrayRef, 3>& plans, int64_t H, int64_t Hkv, double scale,
                            const std::vector<int64_t>& shape, bool need_x, bool need_h, const Tensor& dx_out,
                            const Tensor& dh_out, variable_list& out) {
  using namespace bg;
  if (G.bwd_off || !dh_out.defined() || bg::stream_capturing()) return false;
  for (const Tensor* t : {&dx_out, &dh_out})
    if (t->defined() && (!t->is_contiguous() || t->scalar_type() != at::kBFloat16 ||
                         t->numel() != shape[0] * shape[1] * shape[2]))
      return false;
  const bool has_dx = dx_out.defined();  // (the last block's residual output reaches no loss)
  // the parameters whose gradients this node returns: every one needs a bucket slice
  constexpr int kSlot[] = {2, 3, 4, 5, 6, 7, 8, 9};  // node outputs of sv[1, 2, 6, 7, 9, 12, 13, 17]
  const Tensor* ps[] = {&sv[1], &sv[2], &sv[6], &sv[7], &sv[9], &sv[12], &sv[13], &sv[17]};
  Tensor dst[8];
  bool acc[8] = {};
  int mask = 0, wants = 0;
  for (int i = 0; i < 8; ++i) {
    if (!ps[i]->defined() || !ps[i]->requires_grad()) continue;
    dst[i] = graddst::peek(*ps[i], acc[i]);
    if (!dst[i].defined()) return false;
    mask |= (int)acc[i] << i;
    wants |= 1 << i;
  }
  // one graph per (accumulate pattern, which parameters want gradients, which inputs do)
  const int key = mask | (int)need_x << 8 | (int)need_h << 9 | (int)has_dx << 10 | wants << 11;
  auto param_index = [&](const c10::TensorImpl* impl) {
    for (int i = 0; i < 8; ++i)
      if (ps[i]->defined() && ps[i]->unsafeGetTensorImpl() == impl) return i;
    return -1;
  };
  std::shared_ptr<Bwd> found;  // (G.bwd under g_mu: is_graph_output reads it from the forward)
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = G.bwd.find(key);
    if (it != G.bwd.end()) found = it->second;
  }
  if (found) {
    Bwd& B = *found;
    bool ok = (!has_dx || !B.dx_alias || dx_out.data_ptr() == B.dx_in.data_ptr()) &&
              (!B.dh_alias || dh_out.data_ptr() == B.dh_in.data_ptr());
    for (size_t k = 0; k < B.claims.size(); ++k) {
      const auto& c = B.claims[k];
      const int i = B.pidx[k];
      ok = ok && i >= 0 && dst[i].defined() && dst[i].data_ptr() == c.dst && acc[i] == c.acc;
    }
    if (!ok) {
      std::lock_guard<std::mutex> lk(g_mu);
      G.bwd.erase(key);  // destinations moved: capture anew next time
      return false;
    }
    if (has_dx && !B.dx_alias && dx_out.data_ptr() != B.dx_in.data_ptr()) B.dx_in.copy_(dx_out);
    if (!B.dh_alias && dh_out.data_ptr() != B.dh_in.data_ptr()) B.dh_in.copy_(dh_out);
    for (size_t k = 0; k < B.claims.size(); ++k) {  // the pass bookkeeping of the captured claims
      const auto& c = B.claims[k];
      const int i = B.pidx[k];
      bool a = false;
      const Tensor d = graddst::claim(*ps[i], a);
      TORCH_CHECK(d.defined() && d.data_ptr() == c.dst && a == c.acc, "nbd: block graph claim changed");
    }
    B.g->replay();
    defer::replay(B.deferred, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
    out[0] = need_x ? at::alias(B.g1) : Tensor();
    out[1] = need_h ? at::alias(B.dh) : Tensor();
    for (size_t k = 0; k < B.claims.size(); ++k) {
      const int i = B.pidx[k];
      if (B.slot[k] >= 0) out[B.slot[k]] = graddst::hand_back(*ps[i], dst[i], B.claims[k].acc);
    }
    return true;
  }
  if (G.bwd_captures >= 4) {
    G.bwd_off = true;
    return false;
  }
  ++G.bwd_captures;
  defer::flush();  // reductions queued by eager nodes before this one stay out of the graph
  auto B = std::make_shared<Bwd>();
  {
    std::lock_guard<std::mutex> lk(g_mu);
    B->dx_alias = has_dx && is_graph_output(dx_out);
    B->dh_alias = is_graph_output(dh_out);
  }
  if (has_dx)
    B->dx_in = B->dx_alias ? dx_out.variable_data() : at::empty_like(dx_out, at::MemoryFormat::Contiguous).copy_(dx_out);
  B->dh_in = B->dh_alias ? dh_out.variable_data() : at::empty_like(dh_out, at::MemoryFormat::Contiguous).copy_(dh_out);
  B->g = std::make_unique<at::cuda::CUDAGraph>();
  variable_list o(20);
  std::string err;
  {
    // (RAII: an exception must not leave this thread recording claims or deferred reductions)
    struct Recording {
      explicit Recording(std::vector<graddst::ClaimRecord>* log) {
        graddst::record_claims(log);
        defer::record_begin();  // this node's deferred reductions: queued after each replay
      }
      ~Recording() {
        if (!ended) defer::record_end();
        graddst::record_claims(nullptr);
      }
      std::shared_ptr<void> end() {
        ended = true;
        return defer::record_end();
      }
      bool ended = false;
    } rec(&B->claims);
    err = capture(*B->g, [&] {
      block_bwd(sv, plans, H, Hkv, scale, shape, need_x, need_h, B->dx_in, B->dh_in, o);
      int f = g_fail_bwd.load();
      while (f > 0 && !g_fail_bwd.compare_exchange_weak(f, f - 1)) {
      }
      if (f > 0) throw std::runtime_error("injected backward capture failure");
    });
    B->deferred = rec.end();
  }
  B->warm_refs = castbuf::drop_kept(gemm::gemm_warm_take_refs());
  if (!err.empty()) {
    // nothing captured ran: undo the pass bookkeeping of the claims made while capturing, so the
    // eager backward the caller runs next claims the same bucket slices (a training step must not
    // be lost to a performance feature)
    G.bwd_off = true;
    graddst::release(B->claims);
    TORCH_WARN_ONCE("nbd: a decoder block's backward graph capture failed (", err, "); the block's backward runs eagerly");
    return false;
  }
  // every weight gradient must be its claimed slice (else it would be static graph memory)
  B->pidx.resize(B->claims.size());
  for (size_t k = 0; k < B->claims.size(); ++k) B->pidx[k] = param_index(B->claims[k].param);
  B->slot.assign(B->claims.size(), -1);
  bool valid = true;
  for (int i = 0; i < 8; ++i) {
    const Tensor& g = o[kSlot[i]];
    if (!g.defined()) continue;
    int found = -1;
    for (size_t k = 0; k < B->claims.size(); ++k)
      if (B->claims[k].dst == g.data_ptr() && B->claims[k].param == ps[i]->unsafeGetTensorImpl()) found = (int)k;
    if (found < 0) valid = false;
    else B->slot[found] = kSlot[i];
  }
  B->g->replay();
  defer::replay(B->deferred, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  ++g_stat[3];
  if (!valid) {  // this call: private copies of the non-slice gradients; later calls: eager
    G.bwd_off = true;
    for (int i = 0; i < 8; ++i) {
      Tensor& g = o[kSlot[i]];
      bool claimed = false;
      for (const auto& c : B->claims) claimed = claimed || (g.defined() && c.dst == g.data_ptr());
      if (g.defined() && !claimed) g = g.clone();
    }
    out = o;
    for (int k : {0, 1})
      if (out[k].defined()) out[k] = out[k].clone();
    return true;
  }
  B->g1 = o[0].defined() ? o[0].view(shape) : Tensor();
  B->dh = o[1].defined() ? o[1].view(shape) : Tensor();
  out = o;
  out[0] = B->g1.defined() ? at::alias(B->g1) : Tensor();
  out[1] = B->dh.defined() ? at::alias(B->dh) : Tensor();
  std::lock_guard<std::mutex> lk(g_mu);
  G.bwd[key] = B;
  auto self = g_by_id.count(G.id) ? g_by_id[G.id] : std::weak_ptr<Graph>();
  if (B->g1.defined()) g_outs[B->g1.data_ptr()] = self;
  if (B->dh.defined()) g_outs[B->dh.data_ptr()] = self;
  return true;
}

struct LlamaBlockFn : public torch::autograd::Function<LlamaBlockFn> {
  static variable_list forward(AutogradContext* ctx, const Tensor& x, const Tensor& h, const Tensor& w_qkv,
                               const optional<Tensor>& b_qkv, const Tensor& w_o, const optional<Tensor>& b_o,
                               const Tensor& w_post, const Tensor& w_gu, const Tensor& w_down, const Tensor& w_next,
                               at::IntArrayRef plan_qkv, at::IntArrayRef plan_o, at::IntArrayRef plan_mlp, int64_t H,
                               int64_t Hkv, double scale, double eps, const optional<Tensor>& cos,
                               const optional<Tensor>& sin, int64_t graph_mode) {
    const ht::Scope hs(ht::FWD);
    at::AutoDispatchBelowADInplaceOrView guard;
    ctx->set_materialize_grads(false);
    const int64_t owner = graph_mode >> 8;  // (llama_block_ag packs the model id above the mode)
    graph_mode &= 0xff;
    std::vector<Tensor> save;
    Tensor x_out, h_out;
    std::shared_ptr<bg::Graph> gr;
    std::pair<std::shared_ptr<bg::Stack>, size_t> sh{nullptr, 0};
    if (graph_mode == 1 && bg::stacks_enabled())
      sh = stack_serve(x, h, w_qkv, b_qkv, w_o, b_o, w_post, w_gu, w_down, w_next, plan_qkv, plan_o, plan_mlp, H, Hkv,
                       scale, eps, cos, sin);
    if (!sh.first && graph_mode >= 1)
      gr = block_graph(x, h, w_qkv, b_qkv, w_o, b_o, w_post, w_gu, w_down, w_next, plan_qkv, plan_o, plan_mlp, H, Hkv,
                       scale, eps, cos, sin, owner);
    if (sh.first) {
      const bg::StackMember& mb = sh.first->m[sh.second];
      save = mb.saved;
      const Tensor none;
      const Tensor* ts[] = {&w_qkv, b_qkv ? &*b_qkv : &none, &w_o, b_o ? &*b_o : &none, &w_post, &w_gu,
                            &w_down, &w_next, cos ? &*cos : &none, sin ? &*sin : &none};
      for (size_t i = 0; i < std::size(kBlockWeightSlots); ++i) save[kBlockWeightSlots[i]] = *ts[i];
      save.push_back(bg::stack_token(sh.first));
      x_out = at::alias(mb.x_out);
      h_out = at::alias(mb.h_out);
    } else if (gr) {
      save = gr->saved;
      const Tensor none;
      const Tensor* ts[] = {&w_qkv, b_qkv ? &*b_qkv : &none, &w_o, b_o ? &*b_o : &none, &w_post, &w_gu,
                            &w_down, &w_next, cos ? &*cos : &none, sin ? &*sin : &none};
      for (size_t i = 0; i < std::size(kBlockWeightSlots); ++i) save[kBlockWeightSlots[i]] = *ts[i];
      save.push_back(bg::token(gr));
      x_out = at::alias(gr->x_out);
      h_out = at::alias(gr->h_out);
      if (graph_mode >= 2) ctx->saved_data["bg"] = gr->id;
    } else {
      std::tie(x_out, h_out) = llama_block_fwd(x, h, w_qkv, b_qkv, w_o, b_o, w_post, w_gu, w_down, w_next, plan_qkv,
                                               plan_o, plan_mlp, H, Hkv, scale, eps, cos, sin, &save);
    }
    ctx->save_for_backward(save);
    std::vector<int64_t> meta{H, Hkv, x.requires_grad(), h.requires_grad(), h.size(0), h.size(1), h.size(2),
                              (int64_t)plan_qkv.size(), (int64_t)plan_o.size(), (int64_t)plan_mlp.size()};
    meta.reserve(meta.size() + plan_qkv.size() + plan_o.size() + plan_mlp.size());
    for (at::IntArrayRef p : {plan_qkv, plan_o, plan_mlp}) meta.insert(meta.end(), p.begin(), p.end());
    ctx->saved_data["m"] = std::move(meta);
    ctx->saved_data["s"] = scale;
    return {x_out, h_out};
  }

  static variable_list backward(AutogradContext* ctx, variable_list grads) {
    const ht::Scope hs_total(ht::BWD);
    std::optional<ht::Scope> hs_unpack(std::in_place, ht::UNPACK);
    const auto sv = ctx->get_saved_variables();
    // [H, Hkv, need x, need h, B, T, C, |plan_qkv|, |plan_o|, |plan_mlp|, plans...] (one IValue)
    const std::vector<int64_t> m = ctx->saved_data["m"].toIntVector();
    const double scale = ctx->saved_data["s"].toDouble();
    const int64_t H = m[0], Hkv = m[1];
    const bool need[2] = {m[2] != 0, m[3] != 0};
    const std::vector<int64_t> shape{m[4], m[5], m[6]};
    const int64_t* pp = m.data() + 10;
    const std::array<at::IntArrayRef, 3> plans{at::IntArrayRef(pp, (size_t)m[7]),
                                               at::IntArrayRef(pp + m[7], (size_t)m[8]),
                                               at::IntArrayRef(pp + m[7] + m[8], (size_t)m[9])};
    hs_unpack.reset();
    variable_list out(20);
    if (ctx->saved_data.count("bg")) {  // graph-forwarded: the backward may be a graph too
      std::shared_ptr<bg::Graph> gr;
      {
        std::lock_guard<std::mutex> lk(bg::g_mu);
        auto it = bg::g_by_id.find(ctx->saved_data["bg"].toInt());
        if (it != bg::g_by_id.end()) gr = it->second.lock();
      }
      if (gr && block_bwd_graph(*gr, sv, plans, H, Hkv, scale, shape, need[0], need[1], grads[0], grads[1], out)) {
        ++bg::g_stat[4];
        return out;
      }
      ++bg::g_stat[5];
    }
    block_bwd(sv, plans, H, Hkv, scale, shape, need[0], need[1], grads[0], grads[1], out);
    return out;
  }
};


std::tuple<Tensor, Tensor> llama_block_ag(const Tensor& x, const Tensor& h, const Tensor& w_qkv,
                                          const optional<Tensor>& b_qkv, const Tensor& w_o, const optional<Tensor>& b_o,
                                          const Tensor& w_post, const Tensor& w_gu, const Tensor& w_down,
                                          const Tensor& w_next, at::IntArrayRef plan_qkv, at::IntArrayRef plan_o,
                                          at::IntArrayRef plan_mlp, int64_t H, int64_t Hkv, double scale, double eps,
                                          const optional<Tensor>& cos, const optional<Tensor>& sin, int64_t graphs,
                                          int64_t owner) {
  // graphs: the caller's per-model mode (LlamaModel.block_graphs), -1 = the process setting;
  // only parameters, or weights cast into a kept buffer (models.native(): stable addresses)
  int64_t mode = graphs < 0 ? bg::mode() : std::min<int64_t>(graphs, 2);
  if (bg::g_suspended.load(std::memory_order_relaxed)) mode = 0;  // (graphs.GraphedStep)
  if (!(c10::GradMode::is_enabled() && x.is_cuda() && (w_qkv.is_leaf() || castbuf::kept(w_qkv)))) mode = 0;
  // owner: the model's id (LlamaModel), recorded with its block graphs for a per-model reset
  auto r = LlamaBlockFn::apply(x, h, w_qkv, b_qkv, w_o, b_o, w_post, w_gu, w_down, w_next, plan_qkv, plan_o, plan_mlp,
                               H, Hkv, scale, eps, cos, sin, mode | (std::max<int64_t>(owner, 0) << 8));
  return {r[0], r[1]};
}

std::tuple<Tensor, Tensor> llama_block_noag(const Tensor& x, const Tensor& h, const Tensor& w_qkv,
                                            const optional<Tensor>& b_qkv, const Tensor& w_o,
                                            const optional<Tensor>& b_o, const Tensor& w_post, const Tensor& w_gu,
                                            const Tensor& w_down, const Tensor& w_next, at::IntArrayRef plan_qkv,
                                            at::IntArrayRef plan_o, at::IntArrayRef plan_mlp, int64_t H, int64_t Hkv,
                                            double scale, double eps, const optional<Tensor>& cos,
                                            const optional<Tensor>& sin, int64_t /*graphs*/, int64_t /*owner*/) {
  return llama_block_fwd(x, h, w_qkv, b_qkv, w_o, b_o, w_post, w_gu, w_down, w_next, plan_qkv, plan_o, plan_mlp, H, Hkv,
                         scale, eps, cos, sin, nullptr);
}

// The NBD_HOST_TIMING breakdown: per section calls and mean µs; `reset` clears the counters.
std::string host_timing(bool reset) {
  std::ostringstream os;
  for (int i = 0; i < ht::kN - 1; ++i) {
    const int64_t n = ht::g_cnt[i].load(), ns = ht::g_ns[i].load();
    if (n == 0) continue;
    os << ht::kNames[i] << ": " << n << " calls, " << (double)ns / n / 1e3 << " us/call\n";
  }
  if (reset)
    for (int i = 0; i < ht::kN; ++i) ht::g_ns[i] = 0, ht::g_cnt[i] = 0;
  return os.str();
}

// Per-block graphs: mode 0 off, 1 forward, 2 forward and backward, -1 query; returns the previous mode.
int64_t llama_block_graphs(int64_t mode) {
  const int64_t prev = bg::mode();
  if (mode >= 0) bg::g_mode.store((int)std::min<int64_t>(mode, 2), std::memory_order_relaxed);
  return prev;
}

// Suspend every block graph, per-model modes included (graphs.GraphedStep's warm-up and
// capture); returns the previous state.
bool llama_block_graphs_suspend(bool on) { return bg::g_suspended.exchange(on); }

// Drop every captured block graph (their static memory goes once no autograd node holds it).
void llama_block_graphs_reset() {
  std::map<bg::Key, bg::Slot> slots;
  std::vector<std::shared_ptr<bg::Stack>> dropped;
  std::lock_guard<std::mutex> lk(bg::g_mu);
  slots.swap(bg::g_slots);
  dropped.swap(bg::g_dropped);
  bg::g_active.reset();
  bg::g_outs.clear();
}

// Drop the block graphs made by one model (LlamaModel's finalizer): the other models' graphs stay.
void llama_block_graphs_reset_owner(int64_t owner) {
  std::vector<bg::Slot> drop;  // (destroyed after the lock is released)
  std::vector<std::shared_ptr<bg::Stack>> stacks;  // dropped stacks of this model go too
  std::lock_guard<std::mutex> lk(bg::g_mu);
  auto active = bg::g_active.lock();
  for (auto it = bg::g_slots.begin(); it != bg::g_slots.end();) {
    if (it->second.owner != owner) {
      ++it;
      continue;
    }
    if (active && it->second.stack == active) bg::g_active.reset();
    drop.push_back(std::move(it->second));
    it = bg::g_slots.erase(it);
  }
  for (auto it = bg::g_dropped.begin(); it != bg::g_dropped.end();) {
    if ((*it)->owner == owner) {
      stacks.push_back(*it);
      it = bg::g_dropped.erase(it);
    } else {
      ++it;
    }
  }
  std::unordered_set<const bg::Graph*> gone;
  for (const auto& s : drop)
    if (s.g) gone.insert(s.g.get());
  for (auto it = bg::g_outs.begin(); it != bg::g_outs.end();) {
    auto g = it->second.lock();
    it = (!g || gone.count(g.get())) ? bg::g_outs.erase(it) : std::next(it);
  }
}

// The private memory pools of every live block / stack graph, as [id0, id1, ...] pairs: the
// caching allocator's segments in those pools are the memory block graphs hold (%dist_status).
std::vector<int64_t> llama_block_graphs_pools() {
  std::vector<int64_t> out;
  auto add = [&](const std::unique_ptr<at::cuda::CUDAGraph>& g) {
    if (!g) return;
    const auto id = g->pool();
    out.push_back((int64_t)id.first);
    out.push_back((int64_t)id.second);
  };
  std::lock_guard<std::mutex> lk(bg::g_mu);
  for (const auto& kv : bg::g_slots) {
    if (kv.second.g) {
      add(kv.second.g->g);
      for (const auto& b : kv.second.g->bwd) add(b.second->g);
    }
    if (kv.second.stack) add(kv.second.stack->g);
  }
  for (const auto& st : bg::g_dropped) add(st->g);
  return out;
}

// Tests: make the next `n` backward block-graph captures fail (the eager fallback must run).
void llama_block_graphs_fault(int64_t n) { bg::g_fail_bwd.store((int)n); }

// [captures, replays, eager calls, live graphs, backward captures, replays, eager calls]
std::vector<int64_t> llama_block_graphs_stats() {
  std::lock_guard<std::mutex> lk(bg::g_mu);
  int64_t live = 0;
  for (const auto& kv : bg::g_slots) live += kv.second.g != nullptr;
  return {bg::g_stat[0].load(), bg::g_stat[1].load(), bg::g_stat[2].load(), live,
          bg::g_stat[3].load(), bg::g_stat[4].load(), bg::g_stat[5].load(),
          bg::g_stat[6].load(), bg::g_stat[7].load(), bg::g_stat[8].load(), bg::g_stat[9].load()};
}

// ------------------------------------------------------- fp32 master weights, bf16 compute
// One decoder layer's parameters cast into one flat compute-dtype buffer by one bucket_flatten
// pass, and their gradients cast back into one flat fp32 buffer by another (models/llama.py
// _CastGroup, the Python form of the same node): `models.native()` runs one per layer per
// forward, and the Python autograd.Function around it was ≈20-30 µs of host time per call and
// direction on a host-bound loop (docs/FINDINGS.md §30).
static std::pair<std::vector<int64_t>, int64_t> flat_offsets(const std::vector<Tensor>& ts) {
  std::vector<int64_t> offs;
  offs.reserve(ts.size());
  int64_t pos = 0;
  for (const Tensor& t : ts) {
    offs.push_back(pos);
    pos += (t.numel() + 63) / 64 * 64;  // 64-element starts: every slice on the 16-B vector path
  }
  return {offs, pos};
}

static std::vector<Tensor> slices(const Tensor& buf, const std::vector<int64_t>& offs,
                                  const std::vector<std::vector<int64_t>>& shapes) {
  std::vector<Tensor> out;
  out.reserve(offs.size());
  for (size_t i = 0; i < offs.size(); ++i) {
    int64_t n = 1;
    for (int64_t d : shapes[i]) n *= d;
    out.push_back(buf.narrow(0, offs[i], n).view(shapes[i]));
  }
  return out;
}

// The cast buffer of a parameter group is kept and rewritten by the next forward when nothing
// else holds it any more (the previous pass's autograd graph has released its saved weights):
// the compute-dtype weights then stay at the same addresses from step to step, which is what lets
// the per-block graphs (namespace bg) run on the fp32-master path too.  Still held (a second
// forward before backward): a fresh buffer, as before.
namespace castbuf {
struct Entry {
  c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl> first;  // the group's first parameter (validates the key)
  Tensor buf;
  std::shared_ptr<std::atomic<bool>> busy;  // a cast node of an earlier pass still owns it
  Tensor gbuf;  // the kept cast's gradient buffer (same layout): its slices are the cast weights'
                // registered gradient destinations (graddst::set), allocated on first use
};
std::mutex g_mu;
std::unordered_map<const c10::TensorImpl*, Entry> g_bufs;
std::unordered_map<const void*, int> g_addrs;  // data pointers of the kept buffers
std::vector<Tensor> g_old;                      // replaced buffers (see get)

// The buffer for this group's cast and, when it is the kept one, the flag its node releases
// (a token among the node's saved tensors: freed by that node's backward — which runs after every
// node that saved the cast weights — or with the node).  Storage use counts cannot tell: the
// block graphs keep references to the weights they were captured with.
std::pair<Tensor, std::shared_ptr<std::atomic<bool>>> get(const Tensor& first, int64_t total,
                                                          const at::TensorOptions& opt) {
  std::lock_guard<std::mutex> lk(g_mu);
  // forget the groups of dead parameters (a re-run `model = native(...)` cell must not keep the
  // old model's cast and gradient buffers); the map holds a few groups per live model
  for (auto it = g_bufs.begin(); it != g_bufs.end();) {
    if (it->second.first.expired()) {
      g_addrs.erase(it->second.buf.data_ptr());
      it = g_bufs.erase(it);
    } else {
      ++it;
    }
  }
  auto it = g_bufs.find(first.unsafeGetTensorImpl());
  if (it != g_bufs.end() && !it->second.first.expired() && it->second.buf.numel() == total &&
      it->second.buf.scalar_type() == opt.dtype().toScalarType() && it->second.buf.device() == opt.device()) {
    if (!it->second.busy->exchange(true)) return {it->second.buf, it->second.busy};
    return {at::empty({total}, opt), nullptr};  // still owned (a second forward before backward): a temporary
  }
  Tensor buf = at::empty({total}, opt);
  auto busy = std::make_shared<std::atomic<bool>>(true);
  if (it != g_bufs.end()) {  // (the group changed shape: the old buffer may still be read by a
    g_old.push_back(it->second.buf);  // captured warm-up — keep it, bounded)
    if (g_old.size() > 64) g_old.erase(g_old.begin());
    g_addrs.erase(it->second.buf.data_ptr());
  }
  g_bufs.insert_or_assign(first.unsafeGetTensorImpl(),
                          Entry{c10::weak_intrusive_ptr<c10::TensorImpl, c10::UndefinedTensorImpl>(
                                    first.getIntrusivePtr()),
                                buf, busy});
  g_addrs[buf.data_ptr()] = 1;
  return {buf, busy};
}

// The gradient buffer of the group whose kept cast buffer is `buf` (allocated on first use).
Tensor grad_buf(const Tensor& first, const Tensor& buf) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_bufs.find(first.unsafeGetTensorImpl());
  if (it == g_bufs.end() || !it->second.buf.is_same(buf)) return Tensor();
  if (!it->second.gbuf.defined()) it->second.gbuf = at::empty_like(buf);
  return it->second.gbuf;
}

// [live groups, cast-buffer bytes, gradient-buffer bytes] held for models.native()'s kept casts
// (bytes of every held group: a dead model's stay until the next cast purges them; %dist_status)
std::vector<int64_t> memory() {
  std::lock_guard<std::mutex> lk(g_mu);
  int64_t n = 0, cb = 0, gb = 0;
  for (const auto& kv : g_bufs) {
    n += !kv.second.first.expired();
    cb += kv.second.buf.nbytes();
    if (kv.second.gbuf.defined()) gb += kv.second.gbuf.nbytes();
  }
  return {n, cb, gb};
}

Tensor release_token(std::shared_ptr<std::atomic<bool>> busy) {
  static int64_t dummy = 0;
  return at::from_blob(
      &dummy, {1}, [busy](void*) { busy->store(false, std::memory_order_release); },
      at::TensorOptions().dtype(at::kLong));
}

// t lives in a kept cast buffer (its address is stable across steps)
bool kept(const Tensor& t) {
  if (!t.has_storage()) return false;
  std::lock_guard<std::mutex> lk(g_mu);
  return g_addrs.count(t.storage().data()) != 0;
}

std::vector<Tensor> drop_kept(std::vector<Tensor> refs) {
  std::lock_guard<std::mutex> lk(g_mu);
  refs.erase(std::remove_if(refs.begin(), refs.end(),
                            [](const Tensor& t) { return t.has_storage() && g_addrs.count(t.storage().data()) != 0; }),
             refs.end());
  return refs;
}
}  // namespace castbuf

// Gradient destinations for the cast weights (NBD_CAST_GRAD_DEST=0: off).  A kept cast (stable
// addresses) gets a kept gradient buffer of the same layout; cast_group_ag registers each returned
// weight's slice of it (graddst::set), so the decoder block's backward writes the weight gradients
// there — static addresses, which is what lets the block's backward run as a HIP graph (bg, mode 2)
// on the fp32-master path — and the cast node's backward reads them from one place.
static bool cast_grad_dest_on() {
  static const bool on = [] {
    const char* e = std::getenv("NBD_CAST_GRAD_DEST");
    return e == nullptr || std::atoi(e) != 0;
  }();
  return on;
}
thread_local Tensor t_cast_gbuf;  // forward -> cast_group_ag: the gradient buffer to register

struct CastGroupFn : public torch::autograd::Function<CastGroupFn> {
  // (ps as a TensorList: only that form counts its elements as the node's inputs)
  static variable_list forward(AutogradContext* ctx, at::TensorList ps, int64_t dtype) {
    at::AutoDispatchBelowADInplaceOrView guard;
    TORCH_CHECK(!ps.empty(), "cast_group: no tensors");
    auto [offs, total] = flat_offsets(ps.vec());
    std::vector<std::vector<int64_t>> shapes;
    for (const Tensor& p : ps) {
      TORCH_CHECK(p.is_cuda() && p.device() == ps[0].device() && p.scalar_type() == ps[0].scalar_type(),
                  "cast_group: one device and dtype");
      shapes.push_back(p.sizes().vec());
    }
    auto [buf, busy] = castbuf::get(ps[0], total, ps[0].options().dtype((at::ScalarType)dtype));
    bg::g_cast_epoch.fetch_add(1, std::memory_order_acq_rel);
    if (busy) ctx->save_for_backward({castbuf::release_token(busy)});
    t_cast_gbuf = busy && cast_grad_dest_on() ? castbuf::grad_buf(ps[0], buf) : Tensor();
    std::vector<Tensor> src;
    src.reserve(ps.size());
    for (const Tensor& p : ps) src.push_back(p.contiguous());
    bucket_flatten_hip(src, buf, offs, 1.0, false);
    std::vector<int64_t> flat_shapes;
    for (const auto& sh : shapes) {
      flat_shapes.push_back((int64_t)sh.size());
      flat_shapes.insert(flat_shapes.end(), sh.begin(), sh.end());
    }
    ctx->saved_data["offs"] = offs;
    ctx->saved_data["shapes"] = flat_shapes;
    ctx->saved_data["meta"] = std::vector<int64_t>{total, (int64_t)ps[0].scalar_type()};
    return slices(buf, offs, shapes);
  }

  static variable_list backward(AutogradContext* ctx, variable_list gs) {
    const auto offs = ctx->saved_data["offs"].toIntVector();
    const auto flat = ctx->saved_data["shapes"].toIntVector();
    const auto meta = ctx->saved_data["meta"].toIntVector();
    std::vector<std::vector<int64_t>> shapes;
    for (size_t i = 0; i < flat.size();) {
      const int64_t r = flat[i];
      shapes.emplace_back(flat.begin() + (int64_t)i + 1, flat.begin() + (int64_t)i + 1 + r);
      i += (size_t)r + 1;
    }
    variable_list out(gs.size() + 1);  // (the dtype argument: none)
    // weight gradients written into the registered slices may still have reductions queued
    // (defer.hip: nothing else flushes them on this path)
    if (defer::pending() > 0) defer::flush();
    std::vector<Tensor> have;
    std::vector<int64_t> have_offs;
    for (size_t i = 0; i < gs.size(); ++i)
      if (gs[i].defined()) {
        have.push_back(gs[i].contiguous());
        have_offs.push_back(offs[i]);
      }
    if (have.empty()) return out;
    const Tensor buf = at::empty({meta[0]}, have[0].options().dtype((at::ScalarType)meta[1]));
    bucket_flatten_hip(have, buf, have_offs, 1.0, false);
    const auto views = slices(buf, offs, shapes);
    for (size_t i = 0; i < gs.size(); ++i)
      if (gs[i].defined()) out[i] = views[i];
    return out;
  }
};

std::vector<Tensor> cast_group_ag(at::TensorList ps, int64_t dtype) {
  t_cast_gbuf = Tensor();
  std::vector<Tensor> out = CastGroupFn::apply(ps, dtype);
  const Tensor gbuf = std::move(t_cast_gbuf);
  t_cast_gbuf = Tensor();
  if (gbuf.defined() && c10::GradMode::is_enabled()) {
    auto [offs, total] = flat_offsets(ps.vec());
    for (size_t i = 0; i < out.size(); ++i)
      if (out[i].requires_grad()) graddst::set(out[i], gbuf.narrow(0, offs[i], out[i].numel()).view(out[i].sizes()));
  }
  return out;
}

std::vector<Tensor> cast_group_noag(at::TensorList ps, int64_t dtype) {
  const std::vector<Tensor> v = ps.vec();
  auto [offs, total] = flat_offsets(v);
  std::vector<std::vector<int64_t>> shapes;
  std::vector<Tensor> src;
  for (const Tensor& p : v) {
    shapes.push_back(p.sizes().vec());
    src.push_back(p.contiguous());
  }
  const Tensor buf = at::empty({total}, v[0].options().dtype((at::ScalarType)dtype));
  bucket_flatten_hip(src, buf, offs, 1.0, false);
  return slices(buf, offs, shapes);
}

}  // namespace ag
}  // namespace nbd

// Autograd key: the nodes above.  CUDA key (reached under torch.inference_mode / no autograd):
// the forward alone.
TORCH_LIBRARY_IMPL(nbd, Autograd, m) {
  m.impl("linear_ag", &nbd::ag::linear_ag);
  m.impl("mlp_gelu_ag", &nbd::ag::mlp_gelu_ag);
  m.impl("mlp_swiglu_ag", &nbd::ag::mlp_swiglu_ag);
  m.impl("rms_norm_ag", &nbd::ag::rms_norm_ag);
  m.impl("add_rms_norm_ag", &nbd::ag::add_rms_norm_ag);
  m.impl("layer_norm_ag", &nbd::ag::layer_norm_ag);
  m.impl("add_layer_norm_ag", &nbd::ag::add_layer_norm_ag);
  m.impl("embed_rms_norm_ag", &nbd::ag::embed_rms_norm_ag);
  m.impl("tokpos_layer_norm_ag", &nbd::ag::tokpos_layer_norm_ag);
  m.impl("attn_qkv_ag", &nbd::ag::attn_qkv_ag);
  m.impl("llama_block_ag", &nbd::ag::llama_block_ag);
  m.impl("cast_group_ag", &nbd::ag::cast_group_ag);
}

TORCH_LIBRARY_IMPL(nbd, CUDA, m) {
  m.impl("rms_norm_ag", &nbd::ag::rms_norm_noag);
  m.impl("add_rms_norm_ag", &nbd::ag::add_rms_norm_noag);
  m.impl("layer_norm_ag", &nbd::ag::layer_norm_noag);
  m.impl("add_layer_norm_ag", &nbd::ag::add_layer_norm_noag);
  m.impl("embed_rms_norm_ag", &nbd::ag::embed_rms_norm_noag);
  m.impl("tokpos_layer_norm_ag", &nbd::ag::tokpos_layer_norm_noag);
  m.impl("attn_qkv_ag", &nbd::ag::attn_qkv_noag);
  m.impl("linear_ag", &nbd::ag::linear_noag);
  m.impl("mlp_gelu_ag", &nbd::ag::mlp_gelu_noag);
  m.impl("mlp_swiglu_ag", &nbd::ag::mlp_swiglu_noag);
  m.impl("llama_block_ag", &nbd::ag::llama_block_noag);
  m.impl("cast_group_ag", &nbd::ag::cast_group_noag);
}

// bookkeeping only (no device work): catch-all kernels
TORCH_LIBRARY_FRAGMENT(nbd, m) {
  m.def("llama_block_graphs(int mode) -> int", &nbd::ag::llama_block_graphs);
  m.def("llama_block_graphs_reset() -> ()", &nbd::ag::llama_block_graphs_reset);
  m.def("llama_block_graphs_reset_owner(int owner) -> ()", &nbd::ag::llama_block_graphs_reset_owner);
  m.def("llama_block_graphs_pools() -> int[]", &nbd::ag::llama_block_graphs_pools);
  m.def("llama_block_graphs_fault(int n) -> ()", &nbd::ag::llama_block_graphs_fault);
  m.def("llama_block_graphs_stats() -> int[]", &nbd::ag::llama_block_graphs_stats);
  m.def("host_timing(bool reset) -> str", &nbd::ag::host_timing);
  m.def("llama_block_graphs_suspend(bool on) -> bool", &nbd::ag::llama_block_graphs_suspend);
  m.def("cast_buffers_memory() -> int[]", &nbd::ag::castbuf::memory);
}
