"""Decode attention over a KV cache (K13): one new token per sequence, cache append fused.

``csrc/kernels/decode.hip`` on GPU (bf16, head dim 64, up to 8 query heads per key/value head);
the same math in PyTorch otherwise (CPU, fp32) — also the numerics reference of the GPU tests.
"""
from __future__ import annotations

from typing import Optional

from ._lib import _require


def partials_numel(batch: int, n_head: int, t_max: int) -> int:
    """fp32 workspace the kernel needs for its chunk partials (worst case over key bounds ≤ ``t_max``)."""
    nchunks = min(64, max(1, -(-t_max // 128)))
    return batch * n_head * nchunks * 65


def decode_supported(qkv, k_cache, n_head: int) -> bool:
    import torch

    Hkv = k_cache.shape[1]
    return (qkv.is_cuda and qkv.dtype == torch.bfloat16 and k_cache.dtype == torch.bfloat16
            and k_cache.shape[-1] == 64 and n_head % Hkv == 0 and n_head // Hkv <= 8)


def _rope_at(x, cos, sin, pos):
    """HF rotate_half RoPE of x [B, h, D] at per-row positions pos [B] (fp32 math)."""
    import torch

    half = x.shape[-1] // 2
    c, s = cos[pos][:, None, :], sin[pos][:, None, :]
    a, b = x[..., :half].float(), x[..., half:].float()
    return torch.cat([a * c - b * s, b * c + a * s], -1)


def decode_attention_reference(qkv, k_cache, v_cache, pos, n_head: int, scale: Optional[float] = None, rope=None):
    """PyTorch version of :func:`decode_attention` (writes the caches the same way)."""
    import torch

    B, W = qkv.shape
    Hkv, Tmax, D = k_cache.shape[1], k_cache.shape[2], k_cache.shape[3]
    H, G = n_head, n_head // Hkv
    sc = float(scale) if scale is not None else D ** -0.5
    pos = pos.long().clamp(0, Tmax - 1)
    q = qkv[:, : H * D].view(B, H, D)
    k = qkv[:, H * D:(H + Hkv) * D].view(B, Hkv, D)
    v = qkv[:, (H + Hkv) * D:].view(B, Hkv, D)
    if rope is not None:
        q = _rope_at(q, rope[0], rope[1], pos)
        k = _rope_at(k, rope[0], rope[1], pos)
    bi = torch.arange(B, device=qkv.device)
    k_cache[bi, :, pos] = k.to(k_cache.dtype)
    v_cache[bi, :, pos] = v.to(v_cache.dtype)
    s = torch.einsum("bkgd,bktd->bkgt", q.float().view(B, Hkv, G, D), k_cache.float()) * sc
    mask = torch.arange(Tmax, device=qkv.device)[None, :] > pos[:, None]  # [B, Tmax]
    s = s.masked_fill(mask[:, None, None, :], float("-inf"))
    p = torch.softmax(s, -1)
    o = torch.einsum("bkgt,bktd->bkgd", p, v_cache.float())
    return o.reshape(B, H * D).to(qkv.dtype)


def decode_attention(qkv, k_cache, v_cache, pos, n_head: int, scale: Optional[float] = None, rope=None,
                     kv_len_max: Optional[int] = None, workspace=None):
    """Attention of one new token per sequence over its KV cache.

    ``qkv`` [B, (H + 2·Hkv)·D] is the new tokens' packed projection, ``k_cache``/``v_cache``
    [B, Hkv, Tmax, D] the caches (rows ≥ ``pos[b]`` are free), ``pos`` int64 [B] the new tokens'
    positions (on the device: a decode step graph-captures).  The new k (rotated when ``rope`` =
    (cos, sin) tables) and v are written into the caches at ``pos[b]`` and the token attends to
    rows 0..pos[b].  ``kv_len_max`` bounds max(pos) + 1 (default Tmax; smaller = fewer idle
    workgroups); ``workspace`` = fp32 chunk partials [≥ :func:`partials_numel`] (held by
    ``generation.KVCache``; allocated per call if None).  Returns [B, H·D]."""
    import torch

    D = k_cache.shape[-1]
    sc = float(scale) if scale is not None else D ** -0.5
    if decode_supported(qkv, k_cache, n_head):
        _require()
        B, Tmax = k_cache.shape[0], k_cache.shape[2]
        if workspace is None:
            workspace = torch.empty(partials_numel(B, n_head, Tmax), dtype=torch.float32, device=qkv.device)
        cos, sin = rope if rope is not None else (None, None)
        if qkv.stride(-1) != 1 or qkv.stride(0) % 8 or qkv.data_ptr() % 16:
            qkv = qkv.contiguous()
        return torch.ops.nbd.decode_attn(qkv, k_cache, v_cache, pos, int(n_head), sc, int(kv_len_max or Tmax),
                                         cos, sin, workspace)
    return decode_attention_reference(qkv, k_cache, v_cache, pos, n_head, sc, rope)


# ------------------------------------------------------------------ small-M fused linear (K14)
_NORM = {None: 0, "ln": 1, "rms": 2}
_ACT = {"none": 0, "gelu": 1, "swiglu": 2}


def _lds_bytes(M: int, K: int, norm: int, act: int) -> int:
    mt = 1 if norm else -(-M // 16)  # the kernel falls back to one m-tile per workgroup
    return (mt * 16 * (K + 8) * 2 + 4 * K if norm else 0) + 8 * (2 if act == 2 else 1) * mt * 256 * 4


def linear_small_supported(x, w, norm=None, act: str = "none") -> bool:
    import torch

    M, K = x.shape
    return (x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and 1 <= M <= 64
            and K % 32 == 0 and K <= (2048 if act == "swiglu" else 4096) and x.stride(-1) == 1
            and _lds_bytes(M, K, _NORM[norm[0] if norm else None], _ACT[act]) <= 160 * 1024)


def _apply_norm(x, norm):
    from .norm import layer_norm, rms_norm

    return layer_norm(x, norm[1], norm[2], norm[3]) if norm[0] == "ln" else rms_norm(x, norm[1], norm[2])


def linear_small_reference(x, w, bias=None, norm=None, act: str = "none", residual=None):
    """PyTorch version of :func:`linear_small` (fp32 math, output in x's dtype)."""
    import torch
    import torch.nn.functional as F

    h = x
    if norm is not None:
        if norm[0] == "ln":
            h = F.layer_norm(x.float(), (x.shape[-1],), norm[1].float(), norm[2].float(), norm[3]).to(x.dtype)
        else:
            xf = x.float()
            h = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + norm[2]) * norm[1].float()).to(x.dtype)
    y = h.float() @ w.float().t()
    if act == "swiglu":
        g, u = y.chunk(2, -1)
        y = F.silu(g) * u
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = F.gelu(y, approximate="tanh")
    if residual is not None:
        y = y + residual.float()
    return y.to(x.dtype)


# Measured on MI355X (benchmarks/smallm_bench.py, profiles/smallm_bench_r2.txt), graph-replayed:
# the in-kernel norm prologue is recomputed by every workgroup — a win up to ~8 rows (one node
# instead of two), a loss beyond (+10 µs at 64 rows vs a 2-3 µs norm kernel); and hipBLASLt
# beats this kernel on the LM head (N ≈ 50k) from a few rows up.
FUSE_NORM_MAX_ROWS = 8
LIBRARY_MIN_N = 16384
LIBRARY_MIN_ROWS = 4


def linear_small(x, w, bias=None, norm=None, act: str = "none", residual=None):
    """``residual + act(norm(x) · Wᵀ + bias)`` for a few token rows (decode), one HIP kernel.

    ``x`` [M ≤ 64, K]; ``w`` [N, K] (``act="swiglu"``: [gate; up] = [2N, K], out = silu(g)·u);
    ``norm`` = ``("ln", γ, β, eps)`` or ``("rms", γ, eps)`` applied to x first; ``residual``
    [M, N].  GPU bf16 → ``csrc/kernels/smallm.hip``; elsewhere the same math in PyTorch."""
    import torch
    import torch.nn.functional as F

    if act == "swiglu" and bias is not None:
        raise ValueError("linear_small: no bias with SwiGLU")
    M = x.shape[0]
    if norm is not None and x.is_cuda and M > FUSE_NORM_MAX_ROWS:
        x, norm = _apply_norm(x, norm), None
    if x.is_cuda and M >= LIBRARY_MIN_ROWS and w.shape[0] >= LIBRARY_MIN_N and act == "none" and residual is None:
        return F.linear(x if norm is None else _apply_norm(x, norm), w, bias)
    if linear_small_supported(x, w, norm, act):
        _require()
        nk = _NORM[norm[0] if norm else None]
        nw = norm[1] if norm else None
        nb = norm[2] if norm and norm[0] == "ln" else None
        eps = float(norm[-1]) if norm else 0.0
        return torch.ops.nbd.linear_small(x, w, bias, nw, nb, eps, nk, _ACT[act], residual)
    # the same steps as separate ops (more rows than the kernel takes, CPU, other dtypes)
    from .llama import swiglu

    h = x if norm is None else _apply_norm(x, norm)
    y = F.linear(h, w, bias)
    if act == "gelu":
        y = F.gelu(y, approximate="tanh")
    elif act == "swiglu":
        y = swiglu(y)
    return y if residual is None else residual + y
