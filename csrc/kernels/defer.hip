// defer.hip — deferred weight-gradient reductions (graddst.h, namespace defer).
//
// Two small reductions end a Linear's / a norm's weight gradient: the split-K sum of a weight-
// gradient GEMM's fp32 slabs (gemm.hip reduce_kernel) and the column sum of a LayerNorm /
// RMSNorm backward's per-workgroup partial rows (norm.hip col_reduce_kernel).  For a small model
// each is a ≈5 µs, launch-latency-bound kernel — SmolLM2's step ran 90 + 61 of them.  When the
// gradient's home is its DDP bucket slice nothing reads it before the bucket is consumed, so the
// autograd nodes (autograd.hip) open a Scope and the producers queue the reduction here; flush()
// issues every queued one in a single launch per kind.  Each descriptor is exactly one original
// launch's work with the same fixed-order sums, so the gradients are bit-identical.
//
// Flushes: at the end of the backward that queued (an autograd-engine callback registered by the
// first push), DDP before a bucket's collective (parallel/ddp.py), a second use of a handed-out
// slice and a new pass (graddst.cpp), a change of stream or of graph-capture state, and by itself
// once the queue holds NBD_GRAD_DEFER_FLUSH_MB of partials (so a flush reads MALL-warm data).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/csrc/autograd/engine.h>

#include <atomic>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

#include "graddst.h"
#include "nbd_common.h"

namespace nbd {
namespace defer {

constexpr int kMaxD = 64;  // descriptors per launch (kernel-argument table)
constexpr int kPer = 4;    // split-K: 8-element groups per thread

// ---- split-K slabs: out[i] (+)= Σ_s ws[s][i] as bf16; row sums the same way into rs_out
struct SplitTable {
  const float* ws[kMaxD];
  uint16_t* out[kMaxD];
  uint16_t* rs_out[kMaxD];
  int64_t n8[kMaxD], m8[kMaxD], slab[kMaxD];
  int splits[kMaxD], accum[kMaxD];
  int block0[kMaxD + 1];  // first workgroup of each descriptor
};

__device__ __forceinline__ void splitk_body(const SplitTable& t, int nd, int blk) {
  int d = 0;  // block-uniform forward scan over <= 64 prefixes
  while (d + 1 < nd && t.block0[d + 1] <= blk) ++d;
  const int64_t n8 = t.n8[d], m8 = t.m8[d], slab = t.slab[d];
  const int splits = t.splits[d], accum = t.accum[d];
  const int64_t base = (int64_t)(blk - t.block0[d]) * kPer * 256;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t i = base + u * 256 + threadIdx.x;
    if (i >= n8 + m8) break;
    const bool rs = i >= n8;
    const float* src = rs ? t.ws[d] + splits * slab + 8 * (i - n8) : t.ws[d] + 8 * i;
    const int64_t stride = rs ? m8 * 8 : slab;
    float v[8];
    load8<float>(src, v);
    for (int s = 1; s < splits; ++s) {
      float w[8];
      load8<float>(src + s * stride, w);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += w[e];
    }
    bf16_t* dst = reinterpret_cast<bf16_t*>(rs ? t.rs_out[d] : t.out[d]) + 8 * (rs ? i - n8 : i);
    if (accum & (rs ? 2 : 1)) {
      float o[8];
      load8<bf16_t>(dst, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += o[e];
    }
    store8<bf16_t>(dst, v);
  }
}

__global__ __launch_bounds__(256) void multi_splitk_kernel(SplitTable t, int nd) { splitk_body(t, nd, (int)blockIdx.x); }

// ---- norm partial rows: out0[c] / out1[c - C] (+)= Σ_p part[p][c], c < W (row stride ld)
// (col_reduce_kernel's shape: a workgroup = 16 columns x 16 partial-row groups, combined in LDS)
struct ColTable {
  const float* part[kMaxD];
  uint16_t* out0[kMaxD];
  uint16_t* out1[kMaxD];
  int nparts[kMaxD], ld[kMaxD], W[kMaxD], C[kMaxD], accum[kMaxD];
  int block0[kMaxD + 1];
};

__device__ __forceinline__ void colred_body(const ColTable& t, int nd, int blk) {
  __shared__ float red[16][17];
  int d = 0;
  while (d + 1 < nd && t.block0[d + 1] <= blk) ++d;
  const int nparts = t.nparts[d], ld = t.ld[d], W = t.W[d], C = t.C[d], accum = t.accum[d];
  const float* part = t.part[d];
  const int cx = threadIdx.x & 15, pg = threadIdx.x >> 4;
  const int c = (blk - t.block0[d]) * 16 + cx;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < W) {
    int p = pg;
    for (; p + 48 < nparts; p += 64) {
      a0 += part[(int64_t)p * ld + c];
      a1 += part[(int64_t)(p + 16) * ld + c];
      a2 += part[(int64_t)(p + 32) * ld + c];
      a3 += part[(int64_t)(p + 48) * ld + c];
    }
    for (; p < nparts; p += 16) a0 += part[(int64_t)p * ld + c];
  }
  red[pg][cx] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (pg == 0 && c < W) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) s += red[g][cx];
    const bool second = c >= C;
    bf16_t* dst = reinterpret_cast<bf16_t*>(second ? t.out1[d] : t.out0[d]);
    const int j = second ? c - C : c;
    if (accum & (second ? 2 : 1)) s += Elem<bf16_t>::load(dst, j);
    Elem<bf16_t>::store(dst, j, s);
  }
}

__global__ __launch_bounds__(256) void multi_colred_kernel(ColTable t, int nd) { colred_body(t, nd, (int)blockIdx.x); }

// both kinds of a flush in one launch: workgroups [0, sblocks) sum split-K slabs, the rest column
// partials (the branch is per workgroup; the two sets of outputs are disjoint)
__global__ __launch_bounds__(256) void multi_reduce_kernel(SplitTable st, int ns, int sblocks, ColTable ct, int nc) {
  const int blk = (int)blockIdx.x;
  if (blk < sblocks) splitk_body(st, ns, blk);
  else colred_body(ct, nc, blk - sblocks);
}

// ---- queue -------------------------------------------------------------------------------------
namespace {
struct Item {
  int kind;        // 0 split-K slabs, 1 norm partial rows
  at::Tensor buf;  // keeps the fp32 partials alive (stream-ordered caching allocator) until the flush
  uint16_t* out0;
  uint16_t* out1;
  int64_t a, b, c;  // split-K: n8, m8, slab; colred: nparts, ld, W
  int d;            // split-K: splits; colred: C
  int accum;
};

// Only small reductions are queued: one of a few MB is launch-latency bound (≈5 µs whatever its
// size); a large one is bandwidth bound and best run right after its producer while the partials
// are still in the MALL (GPT-2's 14-38 MB split-K slabs: deferring them made the step 1.5 %
// slower, profiles/grad_defer_ab_r3.txt).  NBD_GRAD_DEFER_MAX_MB / NBD_GRAD_DEFER_FLUSH_MB.
int64_t env_mb(const char* name, int64_t dflt) {
  const char* e = std::getenv(name);
  return ((e != nullptr && std::atoll(e) > 0) ? std::atoll(e) : dflt) << 20;
}
int64_t max_item_bytes() {
  static const int64_t v = env_mb("NBD_GRAD_DEFER_MAX_MB", 8);
  return v;
}
int64_t flush_bytes() {
  static const int64_t v = env_mb("NBD_GRAD_DEFER_FLUSH_MB", 64);
  return v;
}

std::mutex q_mu;
std::vector<Item> q_items;
int64_t q_bytes = 0;
hipStream_t q_stream = nullptr;
int q_device = -1;
bool q_capturing = false;  // the queued items belong to a HIP-graph capture (or to eager work)
std::atomic<bool> g_enabled{false};
thread_local bool t_scope = false;
bool q_callback = false;  // an end-of-backward flush is registered with the running backward

// fill a table from items[pos..] (at most kMaxD): returns (descriptors, workgroups), advances pos
std::pair<int, int> fill_split(SplitTable& tab, const std::vector<const Item*>& items, size_t& pos) {
  int nd = 0, blocks = 0;
  for (; pos < items.size() && nd < kMaxD; ++pos, ++nd) {
    const Item& it = *items[pos];
    tab.ws[nd] = it.buf.data_ptr<float>();
    tab.out[nd] = it.out0;
    tab.rs_out[nd] = it.out1;
    tab.n8[nd] = it.a;
    tab.m8[nd] = it.b;
    tab.slab[nd] = it.c;
    tab.splits[nd] = it.d;
    tab.accum[nd] = it.accum;
    tab.block0[nd] = blocks;
    const int64_t nb = (it.a + it.b + kPer * 256 - 1) / (kPer * 256);
    TORCH_CHECK(blocks + nb < (int64_t)INT32_MAX / 2, "grad_defer: too many workgroups in one flush");
    blocks += (int)nb;
  }
  tab.block0[nd] = blocks;
  return {nd, blocks};
}

std::pair<int, int> fill_col(ColTable& tab, const std::vector<const Item*>& items, size_t& pos) {
  int nd = 0, blocks = 0;
  for (; pos < items.size() && nd < kMaxD; ++pos, ++nd) {
    const Item& it = *items[pos];
    tab.part[nd] = it.buf.data_ptr<float>();
    tab.out0[nd] = it.out0;
    tab.out1[nd] = it.out1;
    tab.nparts[nd] = (int)it.a;
    tab.ld[nd] = (int)it.b;
    tab.W[nd] = (int)it.c;
    tab.C[nd] = it.d;
    tab.accum[nd] = it.accum;
    tab.block0[nd] = blocks;
    blocks += (int)((it.c + 15) / 16);
  }
  tab.block0[nd] = blocks;
  return {nd, blocks};
}

bool merge_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NBD_GRAD_DEFER_MERGE");  // 0: one launch per kind (A/B)
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

void launch_split(const std::vector<const Item*>& items) {
  size_t pos = 0;
  while (pos < items.size()) {
    SplitTable tab{};
    const auto [nd, blocks] = fill_split(tab, items, pos);
    hipLaunchKernelGGL(multi_splitk_kernel, dim3(blocks), dim3(256), 0, q_stream, tab, nd);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
}

void launch_col(const std::vector<const Item*>& items) {
  size_t pos = 0;
  while (pos < items.size()) {
    ColTable tab{};
    const auto [nd, blocks] = fill_col(tab, items, pos);
    hipLaunchKernelGGL(multi_colred_kernel, dim3(blocks), dim3(256), 0, q_stream, tab, nd);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  }
}

// ---- the carried split-K reduce (graddst.h push_carry / take_carry): one slot
bool carry_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NBD_GEMM_CARRY");  // 0: launch large reduces at once (A/B)
    return e == nullptr || e[0] != '0';
  }();
  return on;
}
bool c_has = false;
Item c_item;
hipStream_t c_stream = nullptr;
int c_device = -1;
bool c_capturing = false;

void flush_carry_locked() {
  if (!c_has) return;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)c_device));
  hipStream_t prev = q_stream;
  q_stream = c_stream;
  launch_split({&c_item});
  q_stream = prev;
  c_item = Item{};
  c_has = false;
}

void flush_locked() {
  // a carried reduce on the queue's stream joins the queue's launch (the outputs are disjoint
  // slices: a second claim of a slice flushes before it is written again)
  const bool carry_joins = c_has && !q_items.empty() && c_stream == q_stream && c_device == q_device &&
                           c_capturing == q_capturing && merge_enabled();
  if (!carry_joins) flush_carry_locked();
  if (q_items.empty()) return;
  const c10::hip::HIPGuardMasqueradingAsCUDA guard(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)q_device));
  std::vector<const Item*> split, col;
  if (carry_joins) split.push_back(&c_item);
  for (const Item& it : q_items) (it.kind == 0 ? split : col).push_back(&it);
  if (merge_enabled() && !split.empty() && !col.empty() && split.size() <= (size_t)kMaxD &&
      col.size() <= (size_t)kMaxD) {
    // one launch for both kinds (each table holds all its items)
    SplitTable st{};
    ColTable ct{};
    size_t ps = 0, pc = 0;
    const auto [ns, sblocks] = fill_split(st, split, ps);
    const auto [nc, cblocks] = fill_col(ct, col, pc);
    hipLaunchKernelGGL(multi_reduce_kernel, dim3((unsigned)(sblocks + cblocks)), dim3(256), 0, q_stream, st, ns,
                       sblocks, ct, nc);
    C10_HIP_KERNEL_LAUNCH_CHECK();
  } else {
    if (!split.empty()) launch_split(split);
    if (!col.empty()) launch_col(col);
  }
  q_items.clear();  // the partials go back to the allocator (reuse is ordered after the flush)
  q_bytes = 0;
  if (carry_joins) {
    c_item = Item{};
    c_has = false;
  }
}

thread_local std::vector<Item>* t_record = nullptr;  // record_begin(): queued for replays instead

bool push(Item&& it, void* stream) {
  const int64_t bytes = (int64_t)it.buf.numel() * (int64_t)it.buf.element_size();
  if (bytes > max_item_bytes()) return false;
  if (t_record != nullptr) {
    t_record->push_back(std::move(it));
    return true;
  }
  std::lock_guard<std::mutex> lk(q_mu);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int dev = it.buf.get_device();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  C10_HIP_CHECK(hipStreamIsCapturing(st, &cs));
  const bool capturing = cs == hipStreamCaptureStatusActive;
  // one stream per queue, and never a flush that mixes eager work into a graph capture (the
  // eager partials would be freed while the graph still reads them)
  if (!q_items.empty() && (st != q_stream || dev != q_device || capturing != q_capturing)) flush_locked();
  q_stream = st;
  q_device = dev;
  q_capturing = capturing;
  q_items.push_back(std::move(it));
  q_bytes += bytes;
  if (!q_callback) {
    // whoever runs this backward (DDP or not), the queue is flushed when it ends: a gradient in
    // a slice is never left unfinished after backward() returns.  (Outside a backward pass the
    // engine refuses the callback: then nothing is deferred.)
    try {
      torch::autograd::Engine::get_default_engine().queue_callback([] { flush(); });
      q_callback = true;
    } catch (const std::exception&) {
      flush_locked();
    }
  }
  if (q_bytes >= flush_bytes() || (int)q_items.size() >= 4 * kMaxD) flush_locked();
  return true;
}
}  // namespace

bool enabled() { return g_enabled.load(std::memory_order_relaxed); }
std::atomic<bool> g_force{false};  // benchmarks: queue every split-K reduce (no scope needed)
bool want() { return (t_scope || g_force.load(std::memory_order_relaxed)) && enabled(); }
void set_force(bool on) { g_force.store(on, std::memory_order_relaxed); }
Scope::Scope(bool on) : prev(t_scope) { t_scope = on; }
Scope::~Scope() { t_scope = prev; }

void set_enabled(bool on) {
  if (!on) flush();
  g_enabled.store(on, std::memory_order_relaxed);
}

void flush() {
  std::lock_guard<std::mutex> lk(q_mu);
  flush_locked();
  q_callback = false;  // (a later push registers again; a stale registration only flushes an empty queue)
}

int64_t pending() {
  std::lock_guard<std::mutex> lk(q_mu);
  return (int64_t)q_items.size() + (c_has ? 1 : 0);
}

// A captured graph's deferred reductions: recorded at capture instead of queued (their partial
// buffers live in the graph's memory and stay allocated with the record), queued again after each
// replay — so they still join the one flush per backward instead of a flush per graph.
void record_begin() {
  TORCH_CHECK(t_record == nullptr, "grad_defer: nested record");
  t_record = new std::vector<Item>();
}

std::shared_ptr<void> record_end() {
  std::shared_ptr<std::vector<Item>> r(t_record);
  t_record = nullptr;
  return r;
}

void replay(const std::shared_ptr<void>& rec, void* stream) {
  if (!rec) return;
  for (const Item& it : *static_cast<const std::vector<Item>*>(rec.get())) {
    Item c = it;
    TORCH_CHECK(push(std::move(c), stream), "grad_defer: a recorded reduction cannot be queued");
  }
}

bool push_splitk(const at::Tensor& ws, int splits, int64_t n8, int64_t m8, int64_t slab, uint16_t* out,
                 uint16_t* rs_out, int accum, void* stream) {
  return push(Item{0, ws, out, rs_out, n8, m8, slab, splits, accum}, stream);
}

bool push_carry(const at::Tensor& ws, int splits, int64_t n8, int64_t m8, int64_t slab, uint16_t* out,
                uint16_t* rs_out, int accum, void* stream) {
  if (!carry_enabled() || t_record != nullptr) return false;  // (block-graph records: launch at once)
  std::lock_guard<std::mutex> lk(q_mu);
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  C10_HIP_CHECK(hipStreamIsCapturing(st, &cs));
  flush_carry_locked();  // (one slot: a carry nobody took goes now)
  c_item = Item{0, ws, out, rs_out, n8, m8, slab, splits, accum};
  c_stream = st;
  c_device = ws.get_device();
  c_capturing = cs == hipStreamCaptureStatusActive;
  c_has = true;
  if (!q_callback) {  // finished by the end of this backward at the latest (as push)
    try {
      torch::autograd::Engine::get_default_engine().queue_callback([] { flush(); });
      q_callback = true;
    } catch (const std::exception&) {
      flush_carry_locked();
    }
  }
  return true;
}

static void to_carry(Item& it, Carry* c) {
  c->buf = std::move(it.buf);
  c->out = it.out0;
  c->rs_out = it.out1;
  c->n8 = it.a;
  c->m8 = it.b;
  c->slab = it.c;
  c->splits = it.d;
  c->accum = it.accum;
}

int take_carry(void* stream, Carry* c, int max) {
  std::lock_guard<std::mutex> lk(q_mu);
  if (max <= 0 || (!c_has && q_items.empty())) return 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  C10_HIP_CHECK(hipStreamIsCapturing(st, &cs));
  const bool capturing = cs == hipStreamCaptureStatusActive;
  int n = 0;
  if (c_has) {
    if (st != c_stream || capturing != c_capturing) {
      flush_carry_locked();  // another stream / capture state: launch it on its own
    } else {
      to_carry(c_item, &c[n++]);
      c_item = Item{};
      c_has = false;
    }
  }
  // queued split-K reduces of this stream and capture state, oldest first
  if (!q_items.empty() && st == q_stream && capturing == q_capturing) {
    for (size_t i = 0; i < q_items.size() && n < max;) {
      if (q_items[i].kind != 0) {
        ++i;
        continue;
      }
      q_bytes -= (int64_t)q_items[i].buf.numel() * (int64_t)q_items[i].buf.element_size();
      to_carry(q_items[i], &c[n++]);
      q_items.erase(q_items.begin() + (int64_t)i);
    }
  }
  return n;
}

bool push_colred(const at::Tensor& part, int nparts, int ld, int W, int C, uint16_t* out0, uint16_t* out1, int accum,
                 void* stream) {
  return push(Item{1, part, out0, out1, nparts, ld, W, C, accum}, stream);
}

}  // namespace defer
}  // namespace nbd
