// graddst.cpp — the gradient-destination registry (graddst.h) and its torch.ops.nbd.* entry points.
#include "graddst.h"

#include <c10/util/intrusive_ptr.h>
#include <torch/library.h>

#include <algorithm>
#include <mutex>
#include <unordered_map>

namespace nbd {
namespace graddst {

namespace {
struct Entry {
  Entry(const c10::intrusive_ptr<c10::TensorImpl>& p, at::Tensor d) : param(p), dst(std::move(d)) {}
  c10::weak_intrusive_ptr<c10::TensorImpl> param;  // validates the key (a freed parameter's
                                                   // address can be reused by a new tensor)
  at::Tensor dst;                                  // bucket view shaped like the parameter
  uint64_t gen = 0;                                // backward pass that last handed it out
};
std::mutex g_mu;
std::unordered_map<const c10::TensorImpl*, Entry> g_map;
uint64_t g_gen = 1;
}  // namespace

thread_local std::vector<ClaimRecord>* t_log = nullptr;

void record_claims(std::vector<ClaimRecord>* log) { t_log = log; }

// claim() with `take` = hand it out (pass bookkeeping, flush on a second use); peek() without
static at::Tensor lookup(const at::Tensor& param, bool& acc, bool take) {
  acc = false;
  if (!param.defined() || !param.requires_grad()) return at::Tensor();
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_map.empty()) return at::Tensor();
  auto it = g_map.find(param.unsafeGetTensorImpl());
  if (it == g_map.end()) return at::Tensor();
  Entry& e = it->second;
  if (e.param.expired()) return at::Tensor();
  if (e.gen == g_gen) {
    // a second use in this pass: the engine adds the contributions before AccumulateGrad, so the
    // first writer's deferred reduce into the slice must have been issued
    if (take) defer::flush();
    return at::Tensor();
  }
  const at::Tensor g = param.is_leaf() ? param.grad() : at::Tensor();  // (a registered cast: no .grad)
  if (g.defined()) {
    // accumulate only onto our own slice; any other .grad (set by the user) keeps the normal path
    if (g.data_ptr() != e.dst.data_ptr() || !g.sizes().equals(e.dst.sizes()) || g.scalar_type() != e.dst.scalar_type())
      return at::Tensor();
    acc = true;
  }
  if (take) e.gen = g_gen;
  return e.dst;
}

at::Tensor claim(const at::Tensor& param, bool& acc) {
  at::Tensor d = lookup(param, acc, true);
  if (t_log != nullptr && param.defined())
    t_log->push_back({param.unsafeGetTensorImpl(), d.defined() ? d.data_ptr() : nullptr, acc});
  return d;
}

at::Tensor peek(const at::Tensor& param, bool& acc) { return lookup(param, acc, false); }

void release(const std::vector<ClaimRecord>& claims) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (const ClaimRecord& c : claims) {
    if (c.dst == nullptr) continue;  // that claim handed nothing out
    auto it = g_map.find(c.param);
    if (it != g_map.end() && it->second.gen == g_gen && it->second.dst.data_ptr() == c.dst) it->second.gen = 0;
  }
}

at::Tensor hand_back(const at::Tensor& param, const at::Tensor& dst, bool acc) {
  // AccumulateGrad steals a gradient only while .grad is unset; the slice already holds the sum
  if (acc) param.mutable_grad().reset();
  return dst.view(dst.sizes());  // a fresh TensorImpl (use_count 1) aliasing the slice
}

// ---- ops -----------------------------------------------------------------------------------------
namespace {
// entries whose parameter died still pin their bucket view (and so the whole bucket buffer):
// drop them whenever the registry changes
void purge_expired_locked() {
  for (auto it = g_map.begin(); it != g_map.end();) {
    if (it->second.param.expired()) it = g_map.erase(it);
    else ++it;
  }
}
}  // namespace

void set(const at::Tensor& param, const at::Tensor& dst) {
  std::lock_guard<std::mutex> lk(g_mu);
  // (amortised: the cast weights of models.native() register afresh at every forward)
  static size_t purge_at = 64;
  if (g_map.size() >= purge_at) {
    purge_expired_locked();
    purge_at = std::max<size_t>(64, 2 * g_map.size());
  }
  const c10::TensorImpl* key = param.unsafeGetTensorImpl();
  if (!dst.defined()) {
    g_map.erase(key);
    return;
  }
  TORCH_CHECK(dst.sizes().equals(param.sizes()) && dst.scalar_type() == param.scalar_type() &&
                  dst.device() == param.device() && dst.is_contiguous(),
              "set_grad_dest: the destination must be a contiguous tensor of the parameter's shape, dtype and device");
  g_map.erase(key);
  g_map.emplace(key, Entry(param.getIntrusivePtr(), dst));
}

void set_grad_dest(const at::Tensor& param, const c10::optional<at::Tensor>& dst) {
  graddst::set(param, dst ? *dst : at::Tensor());
}

void grad_dest_new_pass() {
  defer::flush();  // nothing should be pending here (DDP flushes at the end of backward)
  std::lock_guard<std::mutex> lk(g_mu);
  ++g_gen;
}

int64_t grad_dest_count() {
  std::lock_guard<std::mutex> lk(g_mu);
  purge_expired_locked();
  return (int64_t)g_map.size();
}

// The destination if it was handed out earlier in the current pass (its gradient is still in flight
// to AccumulateGrad): a later contribution may add itself into it and return no gradient — the
// tied embedding after the LM head (ops/embedding.py).  Empty tensor otherwise.
at::Tensor grad_dest_join(const at::Tensor& param) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_map.find(param.unsafeGetTensorImpl());
  if (it == g_map.end() || it->second.param.expired() || it->second.gen != g_gen) return at::empty({0}, param.options());
  defer::flush();  // the caller adds into the slice: the first writer's reduce goes first
  return it->second.dst;
}

// Python-side users (ops/loss.py LM head): (destination or an empty tensor, accumulate)
std::tuple<at::Tensor, bool> grad_dest_claim(const at::Tensor& param) {
  bool acc = false;
  at::Tensor d = claim(param, acc);
  return {d.defined() ? d : at::empty({0}, param.options()), acc};
}

void grad_defer_enable(bool on) { defer::set_enabled(on); }
void grad_defer_flush() { defer::flush(); }
void grad_defer_force(bool on) { defer::set_force(on); }
int64_t grad_defer_pending() { return defer::pending(); }

}  // namespace graddst
}  // namespace nbd

// catch-all kernels: bookkeeping only, nothing to differentiate
TORCH_LIBRARY_FRAGMENT(nbd, m) {
  m.def("set_grad_dest(Tensor param, Tensor? dst) -> ()", &nbd::graddst::set_grad_dest);
  m.def("grad_dest_new_pass() -> ()", &nbd::graddst::grad_dest_new_pass);
  m.def("grad_dest_count() -> int", &nbd::graddst::grad_dest_count);
  m.def("grad_dest_claim(Tensor param) -> (Tensor, bool)", &nbd::graddst::grad_dest_claim);
  m.def("grad_dest_join(Tensor param) -> Tensor", &nbd::graddst::grad_dest_join);
  m.def("grad_defer_enable(bool on) -> ()", &nbd::graddst::grad_defer_enable);
  m.def("grad_defer_flush() -> ()", &nbd::graddst::grad_defer_flush);
  m.def("grad_defer_force(bool on) -> ()", &nbd::graddst::grad_defer_force);
  m.def("grad_defer_pending() -> int", &nbd::graddst::grad_defer_pending);
}
