"""Hot-path GPU ops: hand-written gfx950 HIP kernels exposed as ``torch.ops.nbd.*``.

=====================  ==============================================  =========================
op                     what it fuses                                    kernel (csrc/kernels)
=====================  ==============================================  =========================
bucket_flatten (K1)    N grads -> 1 bucket + cast (fp32->bf16) + scale  bucket.hip multi_copy
bucket_unflatten (K2)  bucket -> N grads + scale (1/world) + cast (+=)  bucket.hip multi_copy
local_prereduce (K3)   sum of k buffers, fp32 accumulate, scale, cast   bucket.hip prereduce
prereduce_into_bucket  K3 multi-tensor: bucket slices += grads (no_sync)  bucket.hip multi_copy<ACC>
graddst                gradient destinations: backward GEMMs write into   graddst.cpp + autograd.hip
                       DDP bucket slices (accumulating in the epilogue)
tensor_summary (K4)    count/sum/mean/std/norm/min/max/absmax/nan/inf   summary.hip (MFMA Σx, Σx²)
adamw_flat (K5)        AdamW step over a DDP bucket: fp32 master/m/v,   optim.hip
                       param cast, optional device clip coefficient
cross_entropy (K6)     online-softmax logsumexp fwd + softmax-onehot    xent.hip
                       bwd over [N, V] logits, no fp32 copy
flash_attention (K7)   QKᵀ→online softmax→PV fwd; FA2 dK/dV + dQ bwd    attn.hip (MFMA 32x32x16,
                       (bf16, head dim 64, causal or not)               LDS tr-reads)
add_layer_norm (K8)    residual add + LayerNorm fwd; LN bwd + residual   norm.hip
                       grad + dγ/dβ column partials
colsum / linear (K9)   bias gradient column sums                        norm.hip
embedding (K10)        counting-sort embedding backward (graph-safe)     embed.hip
rms_norm / rope_ /     RMSNorm (+ residual), rotary in place on packed   norm.hip, act.hip
swiglu (K11)           QKV, fused SwiGLU fwd/bwd (Llama family)
gemm_linear /          bf16 GEMM on MFMA 16x16x32: x·Wᵀ, dy·W, dyᵀ·x     gemm.hip (glds + LDS
mlp_gelu /             + bias / GELU / GELU' / SwiGLU / SwiGLU'          swizzles, tr-reads)
mlp_swiglu (K12)       epilogues, split-K, K-groups
decode_attention (K13) one-token attention over a KV cache: RoPE +      decode.hip (split keys,
                       cache append + softmax·V + chunk merge           merge kernel)
linear_small (K14)     decode linear: LN/RMS prologue + x·Wᵀ (MFMA) +   smallm.hip
                       bias / GELU / SwiGLU / residual epilogue, M ≤ 64
=====================  ==============================================  =========================

GPU tensors always go to the HIP kernels; if ``libnbd_ops.so`` cannot be loaded on a GPU box the
call raises (no silent eager fallback).  CPU tensors use the PyTorch reference implementations
below — the same semantics, and the oracle the GPU numerics tests compare against.
"""
from __future__ import annotations

from . import _lib
from ._lib import _require, load_library, native_available
from .attention import attention_qkv, flash_attention, flash_supported
from . import graddst
from .bucket import (_ref_flatten, _ref_prereduce, _ref_unflatten, bucket_flatten, bucket_unflatten, local_prereduce,
                     plan_offsets, prereduce_into_bucket)
from .decode import decode_attention, decode_attention_reference, linear_small, linear_small_reference
from .embedding import embedding, embedding_tok_pos
from .gemm import (block_graphs, block_graphs_memory, block_graphs_reset, block_graphs_stats, cast_buffers_memory,
                   gemm_linear, llama_block, mlp_gelu, mlp_swiglu)
from .llama import rope_, rope_tables, swiglu
from .loss import cross_entropy, linear_cross_entropy
from .mask import seqcls_prep
from .norm import add_layer_norm, add_rms_norm, colsum, embed_rms_norm, layer_norm, linear, rms_norm, tokpos_layer_norm
from .optim import _ref_adamw, adamw_flat
from .tiny import linear_tiny
from .summary import SUMMARY_FIELDS, _ref_summary, tensor_summary, tensor_summary_raw, tensor_summary_text


def __getattr__(name):
    if name in ("_load_error", "_loaded"):  # live values of the loader's state
        return getattr(_lib, name)
    raise AttributeError(name)


__all__ = ["linear_tiny", "bucket_flatten", "bucket_unflatten", "local_prereduce", "prereduce_into_bucket", "graddst", "adamw_flat", "cross_entropy", "linear_cross_entropy",
           "flash_attention", "attention_qkv", "decode_attention", "decode_attention_reference", "linear_small", "linear_small_reference", "flash_supported", "layer_norm", "add_layer_norm", "linear",
           "colsum", "embedding", "embedding_tok_pos", "gemm_linear", "llama_block", "block_graphs", "block_graphs_memory", "block_graphs_reset", "block_graphs_stats", "cast_buffers_memory", "mlp_gelu", "mlp_swiglu", "rms_norm", "add_rms_norm", "embed_rms_norm", "tokpos_layer_norm", "rope_", "rope_tables", "swiglu", "tensor_summary",
           "tensor_summary_text", "tensor_summary_raw", "plan_offsets", "native_available", "load_library",
           "SUMMARY_FIELDS", "seqcls_prep"]
