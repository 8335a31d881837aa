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

namespace nbd {
namespace graddst {

// The registered destination of `param`'s gradient if this write may go there (else undefined).
// `acc` = the destination already holds `param`'s accumulated gradient: add to it.
at::Tensor claim(const at::Tensor& param, bool& acc);

// The tensor to return from backward for a gradient written into `dst` (claimed with `acc`).
at::Tensor hand_back(const at::Tensor& param, const at::Tensor& dst, bool acc);

}  // namespace graddst
}  // namespace nbd
