// ddp_hooks.cpp — DDP bucket readiness counted in C++ (parallel/ddp.py).
//
// DistributedDataParallel launches a bucket's collective when the last of its parameters has had
// its gradient accumulated.  With one Python post-accumulate hook per parameter that is one
// interpreter entry per parameter per backward (SmolLM2-135M: 183 per step, ≈3 µs each on the
// eager step's critical host path — the eager notebook step is host-bound).  Here every
// parameter gets a C++ PostAccumulateGradHook that decrements its bucket's counter; Python is
// entered only twice per backward plus once per bucket: callback(-1) at the first gradient of a
// pass (DDP registers its end-of-backward callback then) and callback(b) when bucket b is
// complete.  ``ddp_hooks_rearm`` resets the counters (DDP's forward and end of backward).
//
// The callback is a Python callable passed by address (``id(fn)``; a strong reference is taken
// here, dropped when the last hook goes).  A hook already present on a parameter (a user's
// ``register_post_accumulate_grad_hook``) is kept and called first; one registered later
// replaces ours — ``ddp_hooks_intact`` lets DDP notice and re-install.
#include <Python.h>

#include <ATen/ATen.h>
#include <torch/csrc/autograd/function_hook.h>
#include <torch/csrc/autograd/variable.h>
#include <torch/library.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace nbd {
namespace ddp_hooks {

namespace {

struct State {
  PyObject* cb = nullptr;                      // strong reference
  std::vector<int> total;                      // parameters per bucket
  std::unique_ptr<std::atomic<int>[]> pending;  // per bucket
  std::atomic<bool> started{false};

  State(PyObject* f, std::vector<int> tot) : cb(f), total(std::move(tot)), pending(new std::atomic<int>[total.size()]) {
    rearm();
  }
  ~State() {
    if (cb != nullptr && Py_IsInitialized()) {
      PyGILState_STATE g = PyGILState_Ensure();
      Py_DECREF(cb);
      PyGILState_Release(g);
    }
  }
  void rearm() {
    for (size_t i = 0; i < total.size(); ++i) pending[i].store(total[i], std::memory_order_relaxed);
    started.store(false, std::memory_order_release);
  }
  // Call the Python callback; a Python exception becomes a C++ one, which the autograd engine
  // re-raises from backward().
  void call(int bucket) {
    PyGILState_STATE g = PyGILState_Ensure();
    PyObject* r = PyObject_CallFunction(cb, "i", bucket);
    std::string err;
    if (r == nullptr) {
      PyObject *type = nullptr, *value = nullptr, *tb = nullptr;
      PyErr_Fetch(&type, &value, &tb);
      PyErr_NormalizeException(&type, &value, &tb);
      PyObject* s = value != nullptr ? PyObject_Str(value) : nullptr;
      const char* msg = s != nullptr ? PyUnicode_AsUTF8(s) : nullptr;
      const char* tname = type != nullptr ? reinterpret_cast<PyTypeObject*>(type)->tp_name : "error";
      err = std::string(tname) + ": " + (msg != nullptr ? msg : "");
      Py_XDECREF(s);
      Py_XDECREF(type);
      Py_XDECREF(value);
      Py_XDECREF(tb);
      PyErr_Clear();
    } else {
      Py_DECREF(r);
    }
    PyGILState_Release(g);
    TORCH_CHECK(err.empty(), "DistributedDataParallel bucket callback failed: ", err);
  }
};

struct BucketHook : torch::autograd::PostAccumulateGradHook {
  BucketHook(std::shared_ptr<State> s, int b, std::unique_ptr<torch::autograd::PostAccumulateGradHook> prev)
      : st(std::move(s)), bucket(b), prev(std::move(prev)) {}
  void operator()(const torch::autograd::Variable& t) override {
    if (prev) (*prev)(t);
    State& s = *st;
    if (!s.started.exchange(true, std::memory_order_acq_rel)) s.call(-1);
    if (s.pending[bucket].fetch_sub(1, std::memory_order_acq_rel) == 1) s.call(bucket);
  }
  std::shared_ptr<State> st;
  int bucket;
  std::unique_ptr<torch::autograd::PostAccumulateGradHook> prev;
};

std::mutex g_mu;
std::unordered_map<int64_t, std::shared_ptr<State>> g_states;
int64_t g_next = 1;

std::shared_ptr<State> find(int64_t handle) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_states.find(handle);
  return it == g_states.end() ? nullptr : it->second;
}

void attach(const std::shared_ptr<State>& s, const at::Tensor& p, int b) {
  auto& slot = torch::autograd::impl::post_acc_grad_hooks(p);
  if (auto* mine = dynamic_cast<BucketHook*>(slot.get()); mine != nullptr && mine->st == s) return;
  std::unique_ptr<torch::autograd::PostAccumulateGradHook> prev = std::move(slot);
  torch::autograd::impl::set_post_acc_grad_hooks(p, std::make_unique<BucketHook>(s, b, std::move(prev)));
}

}  // namespace

// params[i] belongs to bucket bucket_of[i]; callback = id() of a Python callable taking one int.
int64_t ddp_hooks_install(const std::vector<at::Tensor>& params, const std::vector<int64_t>& bucket_of,
                          int64_t callback) {
  TORCH_CHECK(params.size() == bucket_of.size() && !params.empty(), "ddp_hooks_install: one bucket index per parameter");
  TORCH_CHECK(callback != 0, "ddp_hooks_install: no callback");
  int64_t nb = 0;
  for (int64_t b : bucket_of) {
    TORCH_CHECK(b >= 0, "ddp_hooks_install: bucket index");
    nb = std::max(nb, b + 1);
  }
  std::vector<int> total((size_t)nb, 0);
  for (int64_t b : bucket_of) ++total[(size_t)b];
  for (const at::Tensor& p : params)
    TORCH_CHECK(p.defined() && p.is_leaf() && p.requires_grad(), "ddp_hooks_install: trainable leaf parameters only");
  PyObject* cb = reinterpret_cast<PyObject*>(callback);
  {
    // torch.ops calls run without the GIL
    PyGILState_STATE g = PyGILState_Ensure();
    const bool ok = PyCallable_Check(cb) != 0;
    if (ok) Py_INCREF(cb);
    PyGILState_Release(g);
    TORCH_CHECK(ok, "ddp_hooks_install: the callback is not callable");
  }
  auto s = std::make_shared<State>(cb, std::move(total));
  for (size_t i = 0; i < params.size(); ++i) attach(s, params[i], (int)bucket_of[i]);
  std::lock_guard<std::mutex> lk(g_mu);
  const int64_t h = g_next++;
  g_states.emplace(h, std::move(s));
  return h;
}

// Start a new pass: every bucket waits for all its parameters again.
void ddp_hooks_rearm(int64_t handle) {
  if (auto s = find(handle)) s->rearm();
}

// Parameters each bucket still waits for in the current pass.
std::vector<int64_t> ddp_hooks_pending(int64_t handle) {
  std::vector<int64_t> out;
  if (auto s = find(handle))
    for (size_t i = 0; i < s->total.size(); ++i) out.push_back(s->pending[i].load(std::memory_order_acquire));
  return out;
}

// How many of `params` still carry this handle's hook (a later user hook replaces it).
int64_t ddp_hooks_intact(int64_t handle, const std::vector<at::Tensor>& params) {
  auto s = find(handle);
  if (!s) return 0;
  int64_t n = 0;
  for (const at::Tensor& p : params) {
    auto* h = dynamic_cast<BucketHook*>(torch::autograd::impl::post_acc_grad_hooks(p).get());
    n += h != nullptr && h->st == s;
  }
  return n;
}

// Re-attach this handle's hooks where they were replaced (keeping the replacement, called first).
void ddp_hooks_reattach(int64_t handle, const std::vector<at::Tensor>& params, const std::vector<int64_t>& bucket_of) {
  auto s = find(handle);
  TORCH_CHECK(s != nullptr, "ddp_hooks_reattach: unknown handle");
  TORCH_CHECK(params.size() == bucket_of.size(), "ddp_hooks_reattach: one bucket index per parameter");
  for (size_t i = 0; i < params.size(); ++i) attach(s, params[i], (int)bucket_of[i]);
}

// Remove this handle's hooks (restoring any hook they wrapped) and forget the handle.  Our hook may
// sit anywhere in a parameter's chain: a DDP built over the same module before this one was
// collected (a re-run notebook cell) wraps this handle's hook as its `prev` — splice it out there.
void ddp_hooks_remove(int64_t handle, const std::vector<at::Tensor>& params) {
  std::shared_ptr<State> s;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_states.find(handle);
    if (it == g_states.end()) return;
    s = it->second;
    g_states.erase(it);
  }
  for (const at::Tensor& p : params) {
    if (!p.defined()) continue;
    auto& slot = torch::autograd::impl::post_acc_grad_hooks(p);
    auto* h = dynamic_cast<BucketHook*>(slot.get());
    if (h == nullptr) continue;
    if (h->st == s) {  // outermost
      std::unique_ptr<torch::autograd::PostAccumulateGradHook> prev = std::move(h->prev);
      torch::autograd::impl::set_post_acc_grad_hooks(p, std::move(prev));
      continue;
    }
    for (BucketHook* outer = h; outer != nullptr;) {  // inner: unlink from the hook wrapping it
      auto* inner = dynamic_cast<BucketHook*>(outer->prev.get());
      if (inner == nullptr) break;
      if (inner->st == s) {
        std::unique_ptr<torch::autograd::PostAccumulateGradHook> rest = std::move(inner->prev);
        outer->prev = std::move(rest);  // destroys `inner`
        break;
      }
      outer = inner;
    }
  }
}

// BucketHook layers on a parameter (tests: a removed DDP leaves none behind).
int64_t ddp_hooks_depth(const at::Tensor& p) {
  int64_t n = 0;
  for (auto* h = dynamic_cast<BucketHook*>(torch::autograd::impl::post_acc_grad_hooks(p).get()); h != nullptr;
       h = dynamic_cast<BucketHook*>(h->prev.get()))
    ++n;
  return n;
}

}  // namespace ddp_hooks
}  // namespace nbd

// bookkeeping only (no device work): catch-all kernels
TORCH_LIBRARY_FRAGMENT(nbd, m) {
  m.def("ddp_hooks_install(Tensor[] params, int[] bucket_of, int callback) -> int", &nbd::ddp_hooks::ddp_hooks_install);
  m.def("ddp_hooks_rearm(int handle) -> ()", &nbd::ddp_hooks::ddp_hooks_rearm);
  m.def("ddp_hooks_pending(int handle) -> int[]", &nbd::ddp_hooks::ddp_hooks_pending);
  m.def("ddp_hooks_intact(int handle, Tensor[] params) -> int", &nbd::ddp_hooks::ddp_hooks_intact);
  m.def("ddp_hooks_reattach(int handle, Tensor[] params, int[] bucket_of) -> ()", &nbd::ddp_hooks::ddp_hooks_reattach);
  m.def("ddp_hooks_remove(int handle, Tensor[] params) -> ()", &nbd::ddp_hooks::ddp_hooks_remove);
  m.def("ddp_hooks_depth(Tensor param) -> int", &nbd::ddp_hooks::ddp_hooks_depth);
}
