"""Hot-path GPU ops: hand-written gfx950 HIP kernels exposed as ``torch.ops.nbd.*``.

=====================  ==============================================  =========================
op                     what it fuses                                    kernel (csrc/kernels)
=====================  ==============================================  =========================
bucket_flatten (K1)    N grads -> 1 bucket + cast (fp32->bf16) + scale  bucket.hip multi_copy
bucket_unflatten (K2)  bucket -> N grads + scale (1/world) + cast (+=)  bucket.hip multi_copy
local_prereduce (K3)   sum of k buffers, fp32 accumulate, scale, cast   bucket.hip prereduce
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
=====================  ==============================================  =========================

GPU tensors always go to the HIP kernels; if ``libnbd_ops.so`` cannot be loaded on a GPU box the
call raises (no silent eager fallback).  CPU tensors use the PyTorch reference implementations
below — the same semantics, and the oracle the GPU numerics tests compare against.
"""
from __future__ import annotations

import os
import threading
from typing import Dict, List, Optional, Sequence, Tuple

_lock = threading.Lock()
_loaded: Optional[bool] = None
_load_error: Optional[str] = None


def load_library(build: bool = True) -> bool:
    """Load libnbd_ops.so into this process (building it first if stale and ``build``)."""
    global _loaded, _load_error
    if _loaded is not None:
        return _loaded
    with _lock:
        if _loaded is not None:
            return _loaded
        import torch

        from .._native import OPS_HIP_SOURCES, OPS_LIB, build_ops

        try:
            path = os.environ.get("NBD_OPS_LIB")
            if not path:
                path = str(build_ops()) if build and OPS_HIP_SOURCES else str(OPS_LIB)
            torch.ops.load_library(path)
            _loaded = True
        except Exception as e:  # pragma: no cover - reported by native_available()/_require
            _loaded = False
            _load_error = f"{type(e).__name__}: {e}"
    return _loaded


def native_available() -> bool:
    return load_library()


def _require() -> None:
    if not load_library():
        raise RuntimeError(f"nbdistributed_amd HIP ops unavailable ({_load_error}); "
                           "run `python -m nbdistributed_amd._native` to build libnbd_ops.so")


def plan_offsets(numels: Sequence[int], align: int = 64) -> Tuple[List[int], int]:
    """Bucket layout: each tensor starts at a multiple of ``align`` elements (128 B for bf16,
    256 B for fp32) so every tensor takes the kernels' 16-B vector path.  Returns (offsets,
    total numel)."""
    offs = []
    pos = 0
    for n in numels:
        offs.append(pos)
        pos += (int(n) + align - 1) // align * align
    return offs, pos


# ---------------------------------------------------------------- reference implementations
def _ref_flatten(tensors, bucket, offsets, scale):
    for t, o in zip(tensors, offsets):
        n = t.numel()
        bucket[o:o + n].copy_((t.reshape(-1).float() * scale).to(bucket.dtype))


def _ref_unflatten(bucket, tensors, offsets, scale, accumulate):
    for t, o in zip(tensors, offsets):
        n = t.numel()
        v = bucket[o:o + n].float() * scale
        if accumulate:
            v = v + t.reshape(-1).float()
        t.view(-1).copy_(v.to(t.dtype))


def _ref_prereduce(inputs, out, scale):
    acc = inputs[0].reshape(-1).float().clone()
    for x in inputs[1:]:
        acc += x.reshape(-1).float()
    out.view(-1).copy_((acc * scale).to(out.dtype))


def _ref_summary(x):
    import torch

    xf = x.detach().reshape(-1).double()
    n = xf.numel()
    nan = torch.isnan(xf)
    inf = torch.isinf(xf)
    fin = xf[~nan]
    mn = float(fin.min()) if fin.numel() else float("inf")
    mx = float(fin.max()) if fin.numel() else float("-inf")
    amx = float(fin.abs().max()) if fin.numel() else 0.0
    s = float(xf.sum())
    mean = s / n if n else float("nan")
    std = float(xf.std()) if n > 1 else float("nan")
    norm = float(xf.square().sum().sqrt())
    return torch.tensor([n, s, mean, std, norm, mn, mx, amx, float(nan.sum()), float(inf.sum()),
                         n - float(nan.sum()) - float(inf.sum()), 0.0], dtype=torch.float64)


# ---------------------------------------------------------------- public API
def bucket_flatten(tensors: Sequence, bucket=None, offsets: Optional[Sequence[int]] = None, dtype=None,
                   scale: float = 1.0, align: int = 64):
    """Copy ``tensors`` into one flat ``bucket`` (allocated if None), casting to the bucket's dtype
    and multiplying by ``scale``.  Returns (bucket, offsets)."""
    import torch

    tensors = list(tensors)
    if offsets is None:
        offsets, total = plan_offsets([t.numel() for t in tensors], align)
    else:
        total = max((o + t.numel() for o, t in zip(offsets, tensors)), default=0)
    if bucket is None:
        dev = tensors[0].device if tensors else "cpu"
        bucket = torch.zeros(total, dtype=dtype or (tensors[0].dtype if tensors else torch.float32), device=dev)
    if not tensors:
        return bucket, list(offsets)
    flat = [t if t.is_contiguous() else t.contiguous() for t in tensors]
    if bucket.is_cuda:
        _require()
        torch.ops.nbd.bucket_flatten(flat, bucket, list(offsets), float(scale))
    else:
        _ref_flatten(flat, bucket, offsets, scale)
    return bucket, list(offsets)


def bucket_unflatten(bucket, tensors: Sequence, offsets: Sequence[int], scale: float = 1.0,
                     accumulate: bool = False) -> None:
    """Scatter ``bucket`` back into ``tensors`` (in place), times ``scale``, cast to each
    tensor's dtype, optionally accumulating (``t += scale * bucket[...]``)."""
    import torch

    tensors = list(tensors)
    if not tensors:
        return
    for t in tensors:
        if not t.is_contiguous():
            raise ValueError("bucket_unflatten targets must be contiguous")
    if bucket.is_cuda:
        _require()
        torch.ops.nbd.bucket_unflatten(bucket, tensors, list(offsets), float(scale), bool(accumulate))
    else:
        _ref_unflatten(bucket, tensors, offsets, scale, accumulate)


def local_prereduce(inputs: Sequence, out=None, scale: float = 1.0, dtype=None):
    """``out = scale * Σ inputs`` with fp32 accumulation.  Returns ``out``."""
    import torch

    inputs = [x if x.is_contiguous() else x.contiguous() for x in inputs]
    if not inputs:
        raise ValueError("local_prereduce needs at least one input")
    if out is None:
        out = torch.empty_like(inputs[0], dtype=dtype or inputs[0].dtype)
    if out.is_cuda:
        _require()
        if len(inputs) > 16:
            partials = []
            for i in range(0, len(inputs), 16):
                p = torch.empty(out.shape, dtype=torch.float32, device=out.device)
                torch.ops.nbd.local_prereduce(inputs[i:i + 16], p, 1.0)
                partials.append(p)
            return local_prereduce(partials, out, scale)
        torch.ops.nbd.local_prereduce(inputs, out, float(scale))
    else:
        _ref_prereduce(inputs, out, scale)
    return out


def _ref_adamw(grad, param, master, m, v, lr, beta1, beta2, eps, wd, step, grad_scale, grad_scale_t=None,
               step_t=None, lr_t=None):
    import math

    if step_t is not None:
        step, lr = float(step_t.reshape(())), float(lr_t.reshape(()))
    n = param.numel()
    g = grad.reshape(-1)[:n].float() * grad_scale
    if grad_scale_t is not None:
        g = g * grad_scale_t.float().reshape(())
    master.mul_(1 - lr * wd)
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    master.addcdiv_(m, denom, value=-lr / bc1)
    param.view(-1).copy_(master.to(param.dtype))


def adamw_flat(grad, param, master, exp_avg, exp_avg_sq, lr: float, beta1: float, beta2: float, eps: float,
               weight_decay: float, step: int, grad_scale: float = 1.0, grad_scale_t=None, step_t=None,
               lr_t=None) -> None:
    """One fused AdamW step over flat buffers (see csrc/kernels/optim.hip): fp32 master weights
    and moments, ``param`` (any float dtype) rewritten from the master copy.  The gradient is
    multiplied by ``grad_scale`` and, if given, by the 1-element device tensor ``grad_scale_t``
    (a clip coefficient computed on the GPU — no host sync).  ``step_t``/``lr_t`` (1-element
    float32 device tensors, together) override ``step``/``lr`` for HIP-graph replay."""
    import torch

    if param.is_cuda:
        _require()
        torch.ops.nbd.adamw_flat(grad, param, master, exp_avg, exp_avg_sq, float(lr), float(beta1), float(beta2),
                                 float(eps), float(weight_decay), int(step), float(grad_scale), grad_scale_t,
                                 step_t, lr_t)
    else:
        _ref_adamw(grad, param, master, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step, grad_scale,
                   grad_scale_t, step_t, lr_t)


_XentFn = None


def _xent_fn():
    global _XentFn
    if _XentFn is not None:
        return _XentFn
    import torch

    class _FusedCrossEntropy(torch.autograd.Function):
        @staticmethod
        def forward(ctx, logits, target, ignore_index, reduction, inplace_backward):
            loss_rows, lse = torch.ops.nbd.xent_fwd(logits, target, ignore_index)
            if reduction == "mean":
                denom = (target != ignore_index).sum()
                loss = loss_rows.sum() / denom  # 0/0 = nan when every row is ignored, as torch
            else:
                denom = torch.ones((), dtype=torch.int64, device=logits.device)
                loss = loss_rows.sum()
            ctx.save_for_backward(logits, target, lse, denom)
            ctx.ignore_index = ignore_index
            ctx.inplace = inplace_backward
            return loss

        @staticmethod
        def backward(ctx, grad):
            logits, target, lse, denom = ctx.saved_tensors
            scale = (grad.float() / denom).reshape(1)
            dlogits = logits if ctx.inplace else torch.empty_like(logits)
            torch.ops.nbd.xent_bwd(logits, target, lse, scale, ctx.ignore_index, dlogits)
            return dlogits, None, None, None, None

    _XentFn = _FusedCrossEntropy
    return _XentFn


def cross_entropy(logits, target, ignore_index: int = -100, reduction: str = "mean", inplace_backward: bool = False):
    """Softmax cross-entropy of ``logits`` [N, V] (any float dtype) against int64 ``target`` [N]
    — ``F.cross_entropy(logits.float(), target)`` semantics (mean over non-ignored rows, or sum)
    without materialising fp32 logits: one fused HIP pass forward (per-row logsumexp), one pass
    backward writing dlogits in the logits' dtype (``csrc/kernels/xent.hip``).
    ``inplace_backward=True`` writes the gradient over the logits storage (use when nothing reads
    the logits after the loss — saves a [N, V] allocation)."""
    import torch
    import torch.nn.functional as F

    if reduction not in ("mean", "sum"):
        raise ValueError("cross_entropy: reduction must be 'mean' or 'sum'")
    if not logits.is_cuda:
        return F.cross_entropy(logits.float(), target, ignore_index=ignore_index, reduction=reduction)
    _require()
    if logits.stride(-1) != 1:
        logits = logits.contiguous()
    return _xent_fn().apply(logits, target.contiguous().long(), int(ignore_index), reduction, bool(inplace_backward))


_AttnFns = None


def _attn_fns():
    global _AttnFns
    if _AttnFns is not None:
        return _AttnFns
    import torch

    def _ok_view(t):
        return t.stride(-1) == 1 and all(st % 8 == 0 for st in t.stride()[:-1]) and t.data_ptr() % 16 == 0

    def _fix(t):
        return t if _ok_view(t) else t.contiguous()

    class _FlashAttention(torch.autograd.Function):
        @staticmethod
        def forward(ctx, q, k, v, causal, scale):
            q, k, v = _fix(q), _fix(k), _fix(v)
            o, lse = torch.ops.nbd.attn_fwd(q, k, v, causal, scale)
            ctx.save_for_backward(q, k, v, o, lse)
            ctx.causal, ctx.scale = causal, scale
            return o

        @staticmethod
        def backward(ctx, do):
            q, k, v, o, lse = ctx.saved_tensors
            B, H, T, D = q.shape
            Hkv = k.shape[1]
            dq = torch.empty(B, T, H, D, dtype=q.dtype, device=q.device).transpose(1, 2)
            dkv = torch.empty(B, T, 2, Hkv, D, dtype=q.dtype, device=q.device)
            dk, dv = dkv[:, :, 0].transpose(1, 2), dkv[:, :, 1].transpose(1, 2)
            torch.ops.nbd.attn_bwd(_fix(do), q, k, v, o, lse, ctx.causal, ctx.scale, dq, dk, dv)
            return dq, dk, dv, None, None

    def _split(qkv, H, Hkv):
        B, T, W = qkv.shape
        D = W // (H + 2 * Hkv)
        q = qkv[:, :, : H * D].view(B, T, H, D).transpose(1, 2)
        k = qkv[:, :, H * D:(H + Hkv) * D].view(B, T, Hkv, D).transpose(1, 2)
        v = qkv[:, :, (H + Hkv) * D:].view(B, T, Hkv, D).transpose(1, 2)
        return q, k, v

    class _FlashAttentionQKV(torch.autograd.Function):
        """[B, T, (H + 2·Hkv)·D] packed projection in, [B, T, H·D] out; the backward writes the
        packed gradient directly (no split/cat, no transposes).  Hkv < H: grouped-query attention."""

        @staticmethod
        def forward(ctx, qkv, n_head, n_kv, causal, scale):
            B, T, _ = qkv.shape
            q, k, v = _split(qkv, n_head, n_kv)
            o, lse = torch.ops.nbd.attn_fwd(q, k, v, causal, scale)
            ctx.save_for_backward(qkv, o, lse)
            ctx.n_head, ctx.n_kv, ctx.causal, ctx.scale = n_head, n_kv, causal, scale
            return o.transpose(1, 2).reshape(B, T, -1)  # o is stored [B, T, H, D]: a view

        @staticmethod
        def backward(ctx, dy):
            qkv, o, lse = ctx.saved_tensors
            B, T, _ = qkv.shape
            q, k, v = _split(qkv, ctx.n_head, ctx.n_kv)
            dy = dy if dy.is_contiguous() else dy.contiguous()
            dqkv = torch.empty_like(qkv, memory_format=torch.contiguous_format)
            dq, dk, dv = _split(dqkv, ctx.n_head, ctx.n_kv)
            do = dy.view(B, T, ctx.n_head, -1).transpose(1, 2)
            torch.ops.nbd.attn_bwd(do, q, k, v, o, lse, ctx.causal, ctx.scale, dq, dk, dv)
            return dqkv, None, None, None, None

    _AttnFns = (_FlashAttention, _FlashAttentionQKV)
    return _AttnFns


def flash_supported(q) -> bool:
    """The HIP kernels cover bf16, head dim 64, T a multiple of 128 (GPT-2's shapes)."""
    import torch

    return (q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] == 64 and q.shape[-2] % 128 == 0
            and q.shape[-2] >= 128)


def flash_attention(q, k, v, causal: bool = False, scale: Optional[float] = None):
    """softmax(q·kᵀ·scale [+ causal mask])·v for [B, H, T, D] tensors — the HIP flash kernels
    (``csrc/kernels/attn.hip``) where :func:`flash_supported`, else PyTorch SDPA."""
    import torch.nn.functional as F

    sc = float(scale) if scale is not None else q.shape[-1] ** -0.5
    gqa = k.shape[1] != q.shape[1]
    if (flash_supported(q) and k.shape == v.shape and q.shape[0] == k.shape[0] and q.shape[2:] == k.shape[2:]
            and q.shape[1] % k.shape[1] == 0 and k.dtype == v.dtype == q.dtype):
        _require()
        return _attn_fns()[0].apply(q, k, v, bool(causal), sc)
    return F.scaled_dot_product_attention(q, k, v, is_causal=causal, scale=sc, enable_gqa=gqa)


def attention_qkv(qkv, n_head: int, causal: bool = True, scale: Optional[float] = None,
                  n_kv_head: Optional[int] = None):
    """Multi-head attention straight from a packed [B, T, (H + 2·Hkv)·D] projection (GPT-2's
    ``c_attn`` output, or a fused Llama q|k|v projection) to [B, T, H·D].  ``n_kv_head`` < ``n_head``
    is grouped-query attention."""
    import torch
    import torch.nn.functional as F

    B, T, W = qkv.shape
    Hkv = n_kv_head or n_head
    D = W // (n_head + 2 * Hkv)
    sc = float(scale) if scale is not None else D ** -0.5
    if (qkv.is_cuda and qkv.dtype == torch.bfloat16 and D == 64 and T % 128 == 0 and qkv.stride(-1) == 1
            and qkv.stride(1) % 8 == 0 and qkv.stride(0) % 8 == 0 and qkv.data_ptr() % 16 == 0
            and n_head % Hkv == 0):
        _require()
        return _attn_fns()[1].apply(qkv, int(n_head), int(Hkv), bool(causal), sc)
    q = qkv[:, :, : n_head * D].view(B, T, n_head, D).transpose(1, 2)
    k = qkv[:, :, n_head * D:(n_head + Hkv) * D].view(B, T, Hkv, D).transpose(1, 2)
    v = qkv[:, :, (n_head + Hkv) * D:].view(B, T, Hkv, D).transpose(1, 2)
    y = F.scaled_dot_product_attention(q, k, v, is_causal=causal, scale=sc, enable_gqa=Hkv != n_head)
    return y.transpose(1, 2).reshape(B, T, n_head * D)


_NormFns = None


def _norm_fns():
    global _NormFns
    if _NormFns is not None:
        return _NormFns
    import torch

    def _c(t):
        return t if t.is_contiguous() else t.contiguous()

    class _LayerNorm(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, b, eps):
            y, _, mean, rstd = torch.ops.nbd.ln_fwd(x, None, w, b, eps)
            ctx.save_for_backward(x, w, mean, rstd)
            return y

        @staticmethod
        def backward(ctx, dy):
            x, w, mean, rstd = ctx.saved_tensors
            dx, dw, db = torch.ops.nbd.ln_bwd(x, _c(dy), None, w, mean, rstd)
            return dx, dw, db, None

    class _AddLayerNorm(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, delta, w, b, eps):
            y, s, mean, rstd = torch.ops.nbd.ln_fwd(x, delta, w, b, eps)
            ctx.save_for_backward(s, w, mean, rstd)
            return s, y

        @staticmethod
        def backward(ctx, ds, dy):
            s, w, mean, rstd = ctx.saved_tensors
            if dy is None:
                return ds, ds, None, None, None
            dx, dw, db = torch.ops.nbd.ln_bwd(s, _c(dy), None if ds is None else _c(ds), w, mean, rstd)
            return dx, dx, dw, db, None

    class _Linear(torch.autograd.Function):
        """F.linear forward (hipBLASLt, bias fused in the epilogue); backward with the two GEMMs
        and the bias gradient from the HIP column-sum kernel."""

        @staticmethod
        def forward(ctx, x, w, b):
            ctx.save_for_backward(x, w)
            ctx.has_bias = b is not None
            return torch.nn.functional.linear(x, w, b)

        @staticmethod
        def backward(ctx, dy):
            x, w = ctx.saved_tensors
            dy2 = _c(dy).view(-1, dy.shape[-1])
            dx = dw = db = None
            if ctx.needs_input_grad[0]:
                dx = (dy2 @ w).view(x.shape)
            if ctx.needs_input_grad[1]:
                dw = dy2.t() @ _c(x).view(-1, x.shape[-1])
            if ctx.has_bias and ctx.needs_input_grad[2]:
                db = torch.ops.nbd.colsum(dy2, w.dtype)
            return dx, dw, db

    _NormFns = (_LayerNorm, _AddLayerNorm, _Linear)
    return _NormFns


_LlamaFns = None


def _llama_fns():
    global _LlamaFns
    if _LlamaFns is not None:
        return _LlamaFns
    import torch

    def _c(t):
        return t if t.is_contiguous() else t.contiguous()

    class _RMSNorm(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w, eps):
            y, _, rstd = torch.ops.nbd.rms_fwd(x, None, w, eps)
            ctx.save_for_backward(x, w, rstd)
            return y

        @staticmethod
        def backward(ctx, dy):
            x, w, rstd = ctx.saved_tensors
            dx, dw = torch.ops.nbd.rms_bwd(x, _c(dy), None, w, rstd)
            return dx, dw, None

    class _AddRMSNorm(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, delta, w, eps):
            y, s, rstd = torch.ops.nbd.rms_fwd(x, delta, w, eps)
            ctx.save_for_backward(s, w, rstd)
            return s, y

        @staticmethod
        def backward(ctx, ds, dy):
            s, w, rstd = ctx.saved_tensors
            if dy is None:
                return ds, ds, None, None
            dx, dw = torch.ops.nbd.rms_bwd(s, _c(dy), None if ds is None else _c(ds), w, rstd)
            return dx, dx, dw, None

    class _Rope(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, cos, sin, n_rot, head_dim):
            torch.ops.nbd.rope_(x, cos, sin, n_rot, head_dim, False)
            ctx.mark_dirty(x)
            ctx.save_for_backward(cos, sin)
            ctx.n_rot, ctx.head_dim = n_rot, head_dim
            return x

        @staticmethod
        def backward(ctx, g):
            cos, sin = ctx.saved_tensors
            g = g.contiguous().clone()  # never rotate a gradient buffer someone else may hold
            torch.ops.nbd.rope_(g, cos, sin, ctx.n_rot, ctx.head_dim, True)
            return g, None, None, None, None

    class _SwiGLU(torch.autograd.Function):
        @staticmethod
        def forward(ctx, gu):
            ctx.save_for_backward(gu)
            return torch.ops.nbd.swiglu_fwd(gu)

        @staticmethod
        def backward(ctx, d):
            (gu,) = ctx.saved_tensors
            return torch.ops.nbd.swiglu_bwd(gu, _c(d))

    _LlamaFns = (_RMSNorm, _AddRMSNorm, _Rope, _SwiGLU)
    return _LlamaFns


def _rms_ok(x, w) -> bool:
    import torch

    C = x.shape[-1]
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and C % 8 == 0 and C <= 2048
            and w.dtype == x.dtype and not torch.is_autocast_enabled())


def rms_norm(x, weight, eps: float = 1e-6):
    """RMSNorm over the last dim: ``x · rsqrt(mean(x²) + eps) · weight`` (HIP on GPU)."""
    import torch

    if _rms_ok(x, weight):
        _require()
        return _llama_fns()[0].apply(x if x.is_contiguous() else x.contiguous(), weight, float(eps))
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype) * weight


def add_rms_norm(x, delta, weight, eps: float = 1e-6):
    """``s = x + delta; return s, RMSNorm(s)`` in one HIP pass (and one for the backward)."""
    if _rms_ok(x, weight) and delta.dtype == x.dtype and delta.shape == x.shape:
        _require()
        return _llama_fns()[1].apply(x if x.is_contiguous() else x.contiguous(),
                                     delta if delta.is_contiguous() else delta.contiguous(), weight, float(eps))
    s = x + delta
    return s, rms_norm(s, weight, eps)


def rope_tables(T: int, head_dim: int, theta: float, device) -> tuple:
    """cos/sin [T, head_dim/2] float32 for :func:`rope_` (HF default rope)."""
    import torch

    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float32, device=device) / head_dim))
    f = torch.outer(torch.arange(T, dtype=torch.float32, device=device), inv)
    return f.cos().contiguous(), f.sin().contiguous()


def rope_(x, cos, sin, n_rot: int, head_dim: int):
    """Rotary embedding in place on the first ``n_rot`` heads of each row of a packed
    [B, T, H_total·head_dim] projection (HF rotate_half convention).  Returns ``x``."""
    import torch

    if x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and head_dim % 8 == 0 and x.is_contiguous():
        _require()
        return _llama_fns()[2].apply(x, cos, sin, int(n_rot), int(head_dim))
    B, T, W = x.shape
    half = head_dim // 2
    r = x[:, :, : n_rot * head_dim].view(B, T, n_rot, head_dim)
    a, b = r[..., :half].float(), r[..., half:].float()
    c, s_ = cos[:T, None, :], sin[:T, None, :]
    rot = torch.cat([a * c - b * s_, b * c + a * s_], -1).to(x.dtype).view(B, T, n_rot * head_dim)
    return torch.cat([rot, x[:, :, n_rot * head_dim:]], -1)


def swiglu(gu):
    """``silu(g) · u`` for a fused [..., 2I] gate|up projection (HIP fwd/bwd on GPU)."""
    import torch
    import torch.nn.functional as F

    I2 = gu.shape[-1]
    if gu.is_cuda and I2 % 16 == 0 and gu.dtype in (torch.bfloat16, torch.float16, torch.float32):
        _require()
        return _llama_fns()[3].apply(gu if gu.is_contiguous() else gu.contiguous())
    g, u = gu[..., : I2 // 2], gu[..., I2 // 2:]
    return F.silu(g) * u


_EmbFn = None


def _emb_fn():
    global _EmbFn
    if _EmbFn is None:
        import torch

        class _Embedding(torch.autograd.Function):
            @staticmethod
            def forward(ctx, idx, weight):
                ctx.save_for_backward(idx)
                ctx.V = weight.shape[0]
                return torch.nn.functional.embedding(idx, weight)

            @staticmethod
            def backward(ctx, dy):
                (idx,) = ctx.saved_tensors
                C = dy.shape[-1]
                dy2 = dy.reshape(-1, C)
                dy2 = dy2 if dy2.is_contiguous() else dy2.contiguous()
                return None, torch.ops.nbd.embedding_bwd(dy2, idx.reshape(-1).contiguous(), ctx.V)

        _EmbFn = _Embedding
    return _EmbFn


def embedding(idx, weight):
    """``F.embedding`` whose weight gradient comes from the HIP counting-sort kernels
    (``csrc/kernels/embed.hip``): deterministic launch shapes and caching-allocator memory only,
    so a step containing it can be captured in a HIP graph (torch's sort/unique path cannot)."""
    import torch

    C = weight.shape[-1]
    if (weight.is_cuda and idx.dtype == torch.int64 and C % 4 == 0 and C <= 4096 and weight.requires_grad
            and weight.dtype in (torch.bfloat16, torch.float16, torch.float32)):
        _require()
        return _emb_fn().apply(idx, weight)
    return torch.nn.functional.embedding(idx, weight)


def _norm_ok(x, C: int) -> bool:
    import torch

    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and C % 8 == 0 and C <= 2048
            and not torch.is_autocast_enabled())


def layer_norm(x, weight, bias, eps: float = 1e-5):
    """LayerNorm over the last dim (HIP kernels on GPU; ``F.layer_norm`` otherwise)."""
    import torch.nn.functional as F

    C = x.shape[-1]
    if _norm_ok(x, C) and weight is not None and bias is not None and weight.dtype == x.dtype:
        _require()
        return _norm_fns()[0].apply(x if x.is_contiguous() else x.contiguous(), weight, bias, float(eps))
    return F.layer_norm(x, (C,), weight, bias, eps)


def add_layer_norm(x, delta, weight, bias, eps: float = 1e-5):
    """``s = x + delta; return s, LayerNorm(s)`` — the residual add and the norm in one HIP pass
    (and their backward in one pass: dx includes the residual stream's gradient)."""
    import torch.nn.functional as F

    C = x.shape[-1]
    if (_norm_ok(x, C) and weight is not None and bias is not None and weight.dtype == x.dtype
            and delta.dtype == x.dtype and delta.shape == x.shape):
        _require()
        return _norm_fns()[1].apply(x if x.is_contiguous() else x.contiguous(),
                                    delta if delta.is_contiguous() else delta.contiguous(), weight, bias, float(eps))
    s = x + delta
    return s, F.layer_norm(s, (C,), weight, bias, eps)


def linear(x, weight, bias=None):
    """``F.linear`` whose backward computes the bias gradient with the HIP column-sum kernel."""
    import torch.nn.functional as F

    import torch

    if (bias is not None and x.is_cuda and weight.shape[0] % 8 == 0 and x.dtype == weight.dtype == bias.dtype
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32) and not torch.is_autocast_enabled()):
        _require()
        return _norm_fns()[2].apply(x, weight, bias)
    return F.linear(x, weight, bias)


def colsum(x, dtype=None):
    """Σ over all rows of ``x`` [..., C] (fp32 accumulation), as ``dtype`` (default x.dtype)."""
    import torch

    C = x.shape[-1]
    if x.is_cuda and C % 8 == 0:
        _require()
        return torch.ops.nbd.colsum(x if x.is_contiguous() else x.contiguous(), dtype or x.dtype)
    return x.reshape(-1, C).float().sum(0).to(dtype or x.dtype)


SUMMARY_FIELDS = ("count", "sum", "mean", "std", "norm", "min", "max", "absmax", "nan", "inf", "finite", "shift")


def tensor_summary_raw(x):
    """float64[12] on x's device: see ``SUMMARY_FIELDS``."""
    import torch

    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16, torch.float16):
        _require()
        return torch.ops.nbd.tensor_summary(x.detach())
    if x.is_cuda:
        return _ref_summary(x).to(x.device)
    return _ref_summary(x)


def tensor_summary(x) -> Dict[str, float]:
    """One-pass statistics of ``x`` (HIP kernel on GPU); one 96-byte device->host copy."""
    import torch

    if not x.is_floating_point():
        x = x.float() if not x.is_cuda else x.to(torch.float32)
    raw = tensor_summary_raw(x).cpu().tolist()
    d = dict(zip(SUMMARY_FIELDS, raw))
    for k in ("count", "nan", "inf", "finite"):
        d[k] = int(d[k])
    d.pop("shift", None)
    return d


def tensor_summary_text(x) -> str:
    s = tensor_summary(x)
    shape = "x".join(str(d) for d in x.shape) or "scalar"
    parts = [f"mean={s['mean']:.6g}", f"std={s['std']:.6g}", f"min={s['min']:.6g}", f"max={s['max']:.6g}",
             f"norm={s['norm']:.6g}"]
    if s["nan"] or s["inf"]:
        parts.append(f"nan={s['nan']} inf={s['inf']}")
    return f"[{shape} {str(x.dtype).replace('torch.', '')} {x.device}] " + " ".join(parts)


__all__ = ["bucket_flatten", "bucket_unflatten", "local_prereduce", "adamw_flat", "cross_entropy",
           "flash_attention", "attention_qkv", "flash_supported", "layer_norm", "add_layer_norm", "linear",
           "colsum", "embedding", "rms_norm", "add_rms_norm", "rope_", "rope_tables", "swiglu", "tensor_summary", "tensor_summary_text",
           "tensor_summary_raw", "plan_offsets", "native_available", "load_library", "SUMMARY_FIELDS"]
