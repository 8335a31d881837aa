// graddst.h — gradient destinations: where a parameter's gradient should be written.
//
// Data parallelism reduces gradients in flat buckets.  Instead of letting every backward node
// allocate a fresh gradient that the DDP hook then copies into its bucket (bucket_flatten), DDP
// registers, per parameter, the bucket slice that is the gradient's home (a view of the bucket
// with the parameter's shape).  The backward nodes (autograd.hip: Linear / MLP weight and bias
// gradients; ops/loss.py: the LM head) ask for it with claim() and write their GEMM output
// straight into it — overwriting, or accumulating in the GEMM epilogue (beta = 1) when the
// parameter's .grad already is that slice (gradient accumulation / no_sync micro-batches) — and
// return hand_back(), a fresh view that AccumulateGrad steals as .grad without a copy.
//
// The engine sums the incoming gradients of a parameter used twice before AccumulateGrad runs,
// so only the first writer of a backward pass may use the slice: claim() returns an undefined
// tensor once the slice was handed out in the current pass (grad_dest_new_pass(), called by DDP's
// forward, starts a pass); later writers allocate as before and the engine adds.
#pragma once
#include <ATen/ATen.h>

#include <memory>
#include <vector>

namespace nbd {
namespace graddst {

// Register `dst` as `param`'s gradient destination (undefined dst: remove).  `param` is normally a
// leaf (DDP's parameters); a non-leaf registered here — a kept compute-dtype cast of an fp32
// master weight (autograd.hip CastGroupFn) — has no .grad, so its writes never accumulate.
void set(const at::Tensor& param, const at::Tensor& dst);

// The registered destination of `param`'s gradient if this write may go there (else undefined).
// `acc` = the destination already holds `param`'s accumulated gradient: add to it.
at::Tensor claim(const at::Tensor& param, bool& acc);

// The tensor to return from backward for a gradient written into `dst` (claimed with `acc`).
at::Tensor hand_back(const at::Tensor& param, const at::Tensor& dst, bool acc);

// What claim() would return for `param` now, without handing it out (no pass bookkeeping, no
// flush): the per-block backward graphs (autograd.hip) check their captured destinations with it.
at::Tensor peek(const at::Tensor& param, bool& acc);

// Claims made on this thread while a log is set are appended to it (nullptr stops recording).
struct ClaimRecord {
  const c10::TensorImpl* param;
  const void* dst;  // nullptr: no destination (the writer allocated)
  bool acc;
};
void record_claims(std::vector<ClaimRecord>* log);

// Undo the pass bookkeeping of recorded claims (a graph capture that failed: nothing it captured
// ran, so the slices were never written and may be claimed again in this pass).
void release(const std::vector<ClaimRecord>& claims);

}  // namespace graddst

// Deferred weight-gradient reductions (defer.hip).  A split-K weight-gradient GEMM writes fp32
// partial slabs that a second kernel sums into the gradient, a norm backward per-workgroup
// partial rows; for a small model each such reduce is a ≈5 µs launch (90 + 61 per SmolLM2 step).
// When the gradient goes to its claimed bucket slice nothing reads it before the bucket is
// consumed, so the autograd node opens a Scope and the producer queues the reduce instead of
// launching it; flush() issues every queued reduce in one launch per kind.  DDP flushes before a
// bucket's collective and at the end of backward (parallel/ddp.py); a second use of a handed-out
// slice (claim / join) and a new pass flush first.  enabled() is process-wide
// (torch.ops.nbd.grad_defer_enable; NBD_GRAD_DEFER=0 keeps it off).
namespace defer {
bool enabled();
void set_enabled(bool on);
bool want();  // enabled and inside a Scope(true) on this thread (or forced)
void set_force(bool on);  // benchmarks only: treat every split-K reduce as deferrable
struct Scope {
  explicit Scope(bool on);
  ~Scope();
  bool prev;
};
// queue one reduce (reduce_kernel's arguments; `ws` kept alive until the flush); false = launch now
bool push_splitk(const at::Tensor& ws, int splits, int64_t n8, int64_t m8, int64_t slab, uint16_t* out,
                 uint16_t* rs_out, int accum, void* stream);
// queue one norm weight-gradient column sum (norm.hip col_reduce: `part` [nparts][ld] fp32,
// columns [0, C) -> out0, [C, W) -> out1, bf16); false = launch now
bool push_colred(const at::Tensor& part, int nparts, int ld, int W, int C, uint16_t* out0, uint16_t* out1, int accum,
                 void* stream);
void flush();
int64_t pending();
// A split-K reduce too large to queue (its slabs are read best while still in the MALL) can ride
// in the NEXT grouped GEMM launch on the same stream as extra workgroups (gemm.hip pair_kernel's
// tail) instead of a launch of its own; flush() and every flush point above launch it alone.
struct Carry {
  at::Tensor buf;  // the fp32 slabs (kept alive until the launch that reads them is enqueued)
  uint16_t* out;
  uint16_t* rs_out;
  int64_t n8, m8, slab;
  int splits, accum;
};
bool push_carry(const at::Tensor& ws, int splits, int64_t n8, int64_t m8, int64_t slab, uint16_t* out,
                uint16_t* rs_out, int accum, void* stream);
// up to `max` reduces for a launch on `stream`: the carry first, then queued split-K reduces
// (theirs are small; summed in a grid's tail they need no flush launch); returns how many
int take_carry(void* stream, Carry* c, int max);
// Recording (this thread, around a graph capture): pushes are kept in the record, not queued;
// replay() queues the recorded reductions on `stream` (after each replay of that graph).
void record_begin();
std::shared_ptr<void> record_end();
void replay(const std::shared_ptr<void>& rec, void* stream);
}  // namespace defer
}  // namespace nbd
