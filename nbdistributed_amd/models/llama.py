"""Llama-family models (SmolLM2, Llama 2/3-style) built on the framework's HIP kernels.

The reference notebook fine-tunes SmolLM2-135M (``AutoModelForSequenceClassification``,
``00_accelerate.ipynb`` exec 22) — a Llama with grouped-query attention.  Through HF modules its
small-batch step is launch-bound (≈4,600 kernels, GPU busy 25 ms of a 40 ms step on MI355X:
``profiles/notebook_prof_r1.md``).  This implementation keeps HF's weights and numerics
(``from_hf`` / ``load_hf_state_dict``) but runs a block as:

    x ─ rms_norm ─ qkv GEMM (fused q|k|v) ─ flash attention (GQA, RoPE fused into its loads) ─ o GEMM ─┐
    └──────────────────────────── add_rms_norm (residual + norm in one pass) ◄───────────────┘
      ─ gate|up GEMM (fused, SwiGLU in its epilogue) ─ down GEMM ─ add_rms_norm (into the next block's norm)

i.e. ~12 kernels per block instead of ~70, nothing that synchronises with the host, and only
caching-allocator memory — so the whole training step captures into a HIP graph
(``nbdistributed_amd.graphs.GraphedStep``).  The GPU path needs bf16/f16, head_dim 64 and a
sequence length that is a multiple of 128; anything else (CPU, fp32) runs the same math in
plain PyTorch.

HF semantics kept by the one-line swap (``native()``):

* ``attention_mask``: the fused path runs causal attention without a key mask, exact for right
  padding.  The sequence classifier rotates left-padded rows into right-padded ones in one kernel
  (``ops.seqcls_prep``; RoPE scores depend on position differences only) and re-indexes the
  pooled token; a mask with holes is reported (ValueError at the next call: the check is read
  without a host sync, so the reported batch has already been applied — ``NBD_MASK_CHECK_SYNC=1``
  raises on the offending call instead; inside a ``GraphedStep`` the check follows the replays).
  The causal LM needs right padding (reported the same way).
* forward (pre-)hooks and backward hooks on the decoder layers or any of their submodules (or
  global module hooks): the model then runs module by module, HF's structure — each layer is
  called as ``layer(hidden_states, ...)`` and returns the residual stream, attention honours the
  full ``attention_mask`` — so every hook fires and sees HF's activations.
"""
from __future__ import annotations

import itertools
import logging
import os
import weakref
from dataclasses import dataclass
from typing import Any, Dict, NamedTuple, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


@dataclass
class LlamaConfig:
    vocab_size: int = 49152
    hidden_size: int = 576
    intermediate_size: int = 1536
    num_hidden_layers: int = 30
    num_attention_heads: int = 9
    num_key_value_heads: int = 3
    max_position_embeddings: int = 8192
    rms_norm_eps: float = 1e-5
    rope_theta: float = 100000.0
    tie_word_embeddings: bool = True
    num_labels: int = 2
    pad_token_id: Optional[int] = 0
    initializer_range: float = 0.02
    # family variants: Qwen2 (biased q/k/v), Llama with attention_bias (q/k/v and o), Mistral
    # (explicit head_dim, sliding window), Llama 3.x rope scaling ({"rope_type": "llama3", ...})
    qkv_bias: bool = False
    o_bias: bool = False
    explicit_head_dim: Optional[int] = None
    sliding_window: Optional[int] = None
    rope_scaling: Optional[Dict[str, Any]] = None

    @property
    def head_dim(self) -> int:
        return self.explicit_head_dim or self.hidden_size // self.num_attention_heads

    @classmethod
    def smollm2_135m(cls, **kw) -> "LlamaConfig":
        return cls(**kw)

    @classmethod
    def tiny(cls, **kw) -> "LlamaConfig":
        d = dict(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                 num_key_value_heads=2, max_position_embeddings=1024)
        d.update(kw)
        return cls(**d)

    @classmethod
    def from_hf(cls, hf) -> "LlamaConfig":
        """From an HF ``LlamaConfig`` / ``Qwen2Config`` / ``MistralConfig`` (transformers 4.x or 5.x)."""
        kind = getattr(hf, "model_type", "llama")
        if kind not in ("llama", "qwen2", "mistral"):
            raise NotImplementedError(f"LlamaConfig.from_hf: model_type {kind!r}")
        params = dict(getattr(hf, "rope_parameters", None) or {})
        legacy = getattr(hf, "rope_scaling", None)  # transformers 4.x
        if legacy:
            params.update(legacy)
        rope = getattr(hf, "rope_theta", None) or params.get("rope_theta", 10000.0)
        rtype = params.get("rope_type", params.get("type", "default"))
        if rtype not in ("default", "llama3"):
            raise NotImplementedError(f"LlamaConfig.from_hf: rope_type {rtype!r}")
        scaling = None
        if rtype == "llama3":
            scaling = {k: float(params[k]) for k in ("factor", "low_freq_factor", "high_freq_factor",
                                                     "original_max_position_embeddings")}
        if getattr(hf, "mlp_bias", False):
            raise NotImplementedError("LlamaConfig.from_hf: mlp_bias")
        attn_bias = bool(getattr(hf, "attention_bias", False))
        window = getattr(hf, "sliding_window", None)
        if kind == "qwen2" and not getattr(hf, "use_sliding_window", False):
            window = None
        hd = getattr(hf, "head_dim", None)
        return cls(vocab_size=hf.vocab_size, hidden_size=hf.hidden_size, intermediate_size=hf.intermediate_size,
                   num_hidden_layers=hf.num_hidden_layers, num_attention_heads=hf.num_attention_heads,
                   num_key_value_heads=hf.num_key_value_heads or hf.num_attention_heads,
                   max_position_embeddings=hf.max_position_embeddings, rms_norm_eps=hf.rms_norm_eps,
                   rope_theta=float(rope), tie_word_embeddings=bool(getattr(hf, "tie_word_embeddings", False)),
                   num_labels=getattr(hf, "num_labels", 2), pad_token_id=getattr(hf, "pad_token_id", None),
                   qkv_bias=kind == "qwen2" or attn_bias, o_bias=kind != "qwen2" and attn_bias,
                   explicit_head_dim=hd if hd and hd != hf.hidden_size // hf.num_attention_heads else None,
                   sliding_window=window, rope_scaling=scaling)


class SequenceClassifierOutput(NamedTuple):
    """``(loss, logits)`` that also reads like HF's output object: ``out.loss``, ``out.logits``."""
    loss: Optional[torch.Tensor]
    logits: torch.Tensor


class CausalLMOutput(NamedTuple):
    """``(loss, logits)`` with HF-style attribute access (``logits`` None when not returned)."""
    loss: Optional[torch.Tensor]
    logits: Optional[torch.Tensor]


class _CastGroup(torch.autograd.Function):
    """Mixed precision for fp32 master parameters: one fused HIP pass
    (``nbd::bucket_flatten``) casts a group of parameters into one flat compute-dtype buffer, and
    the backward casts their gradients back into one flat fp32 buffer — two launches per group
    instead of two per parameter (what per-op autocast would issue).  The model casts one decoder
    layer per group, so under DDP each layer's fp32 gradients are ready as soon as that layer's
    backward is done (bucket all-reduces keep overlapping backward)."""

    @staticmethod
    def forward(ctx, dtype, *ps):
        offs, total = ops.plan_offsets([p.numel() for p in ps])
        buf = torch.empty(total, dtype=dtype, device=ps[0].device)
        torch.ops.nbd.bucket_flatten(list(ps), buf, offs, 1.0, False)
        ctx.meta = ([p.shape for p in ps], offs, total, ps[0].dtype)
        return tuple(buf[o:o + p.numel()].view(p.shape) for p, o in zip(ps, offs))

    @staticmethod
    def backward(ctx, *gs):
        shapes, offs, total, dt = ctx.meta
        have = [i for i, g in enumerate(gs) if g is not None]
        out = [None] * len(gs)
        if have:
            buf = torch.empty(total, dtype=dt, device=gs[have[0]].device)
            torch.ops.nbd.bucket_flatten([gs[i].contiguous() for i in have], buf, [offs[i] for i in have], 1.0, False)
            for i in have:
                out[i] = buf[offs[i]:offs[i] + shapes[i].numel()].view(shapes[i])
        return (None, *out)


_SCALAR_TYPE = {torch.float16: 5, torch.float32: 6, torch.bfloat16: 15}  # c10::ScalarType codes
NATIVE_CAST = os.environ.get("NBD_NATIVE_CAST", "1") != "0"


def cast_group(dtype, ps):
    """``ps`` cast to ``dtype`` through one flat buffer, gradients cast back the same way: the C++
    node (``torch.ops.nbd.cast_group_ag``, csrc/kernels/autograd.hip ``CastGroupFn``) on the GPU,
    the Python ``_CastGroup`` otherwise (``NBD_NATIVE_CAST=0``: always)."""
    ps = list(ps)
    if NATIVE_CAST and ps[0].is_cuda and dtype in _SCALAR_TYPE and ops.native_available():
        return tuple(torch.ops.nbd.cast_group_ag(ps, _SCALAR_TYPE[dtype]))
    return _CastGroup.apply(dtype, *ps)


class RMSNorm(nn.Module):
    def __init__(self, n: int, eps: float):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(n))
        self.eps = eps

    def forward(self, x):
        return ops.rms_norm(x, self.weight, self.eps)


def _masked_attention(qkv, H: int, Hkv: int, cos, sin, key_mask):
    """Causal GQA attention where key ``j`` of row ``b`` is visible only if ``key_mask[b, j]``
    (HF's 4-D mask from ``attention_mask``).  A query with no visible key (a left pad) attends to
    itself — its output feeds nothing a real token reads.  PyTorch SDPA: the module path only."""
    from ..ops.llama import rope_

    B, T, W = qkv.shape
    D = W // (H + 2 * Hkv)
    qkv = rope_(qkv.contiguous().clone(), cos, sin, H + Hkv, D)
    q = qkv[:, :, : H * D].view(B, T, H, D).transpose(1, 2)
    k = qkv[:, :, H * D:(H + Hkv) * D].view(B, T, Hkv, D).transpose(1, 2)
    v = qkv[:, :, (H + Hkv) * D:].view(B, T, Hkv, D).transpose(1, 2)
    causal = torch.ones(T, T, dtype=torch.bool, device=qkv.device).tril()
    allow = causal[None] & key_mask.bool()[:, None, :]
    allow = allow | torch.eye(T, dtype=torch.bool, device=qkv.device)[None]
    y = F.scaled_dot_product_attention(q, k, v, attn_mask=allow[:, None], scale=D ** -0.5, enable_gqa=Hkv != H)
    return y.transpose(1, 2).reshape(B, T, H * D)


class LlamaAttention(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.H, self.Hkv, self.D = c.num_attention_heads, c.num_key_value_heads, c.head_dim
        self.qkv_proj = nn.Linear(c.hidden_size, (self.H + 2 * self.Hkv) * self.D, bias=c.qkv_bias)
        self.o_proj = nn.Linear(self.H * self.D, c.hidden_size, bias=c.o_bias)
        self.window = c.sliding_window

    def forward(self, x, cos, sin, kv=None, key_mask=None):
        if self.window is not None and x.shape[1] > self.window:
            raise NotImplementedError(f"sliding-window attention: {x.shape[1]} positions > window {self.window}")
        # RoPE is applied inside the attention kernels on the HIP path (rope_ + SDPA otherwise)
        qkv = ops.gemm_linear(x, self.qkv_proj.weight, self.qkv_proj.bias)  # HIP MFMA GEMM on GPU bf16
        if kv is not None:  # (KVCache, layer): generation prefill, before anything rotates qkv in place
            kv[0].store(kv[1], qkv, rope=(cos, sin))
        if key_mask is not None:
            a = _masked_attention(qkv, self.H, self.Hkv, cos, sin, key_mask)
        else:
            a = ops.attention_qkv(qkv, self.H, causal=True, n_kv_head=self.Hkv, rope=(cos, sin))
        return ops.gemm_linear(a, self.o_proj.weight, self.o_proj.bias)

    def decode(self, x, norm_w, eps, cache, layer: int, pos, rope):
        """Generation step: ``x + o_proj(attn(rms(x)))`` — fused norm + q|k|v, decode attention
        (RoPE, cache append), fused o_proj + residual."""
        qkv = ops.linear_small(x, self.qkv_proj.weight, self.qkv_proj.bias, norm=("rms", norm_w, eps))
        a = cache.attend(layer, qkv, pos, rope=rope)
        return ops.linear_small(a, self.o_proj.weight, self.o_proj.bias, residual=x)


class LlamaMLP(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.gate_up_proj = nn.Linear(c.hidden_size, 2 * c.intermediate_size, bias=False)
        self.down_proj = nn.Linear(c.intermediate_size, c.hidden_size, bias=False)

    def forward(self, x):
        # SwiGLU (and its backward) run in the gate|up GEMM's (the down dgrad's) epilogue
        return ops.mlp_swiglu(x, self.gate_up_proj.weight, self.down_proj.weight)

    def decode(self, x, norm_w, eps):
        f = ops.linear_small(x, self.gate_up_proj.weight, norm=("rms", norm_w, eps), act="swiglu")
        return ops.linear_small(f, self.down_proj.weight, residual=x)


class LlamaDecoderLayer(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.input_layernorm = RMSNorm(c.hidden_size, c.rms_norm_eps)
        self.self_attn = LlamaAttention(c)
        self.post_attention_layernorm = RMSNorm(c.hidden_size, c.rms_norm_eps)
        self.mlp = LlamaMLP(c)

    def forward(self, hidden_states, cos, sin, key_mask=None):
        """HF ``LlamaDecoderLayer.forward``'s structure (the module path, taken when hooks are
        registered): residual stream in, residual stream out, every submodule called as a module."""
        kw = {} if key_mask is None else {"key_mask": key_mask}
        x = hidden_states + self.self_attn(self.input_layernorm(hidden_states), cos, sin, **kw)
        return x + self.mlp(self.post_attention_layernorm(x))


def _drop_block_graphs(owner: int) -> None:
    try:
        ops.block_graphs_reset(owner)
    except Exception:  # interpreter shutdown
        pass


_OWNER_IDS = itertools.count(1)


def _global_hooks() -> bool:
    from torch.nn.modules import module as _m

    return bool(_m._global_forward_hooks or _m._global_forward_pre_hooks or _m._global_backward_hooks
                or getattr(_m, "_global_backward_pre_hooks", None))


# NBD_MASK_CHECK_SYNC=1: read the mask check right after the prep kernel (one host sync per
# call) and raise before the batch is used, instead of at the next call
_MASK_CHECK_SYNC = os.environ.get("NBD_MASK_CHECK_SYNC", "0") == "1"


class _MaskCheck:
    """A device-side flag about the attention masks seen (``ops.seqcls_prep``), read one call
    late without a host sync: a pinned copy and an event per call; the next call raises if the
    flag had a failing bit by then.  THE REPORTED BATCH HAS ALREADY BEEN APPLIED: its loss and
    gradients were computed on the fused path (wrong for that mask) and may already have gone
    through ``optimizer.step()``.  ``NBD_MASK_CHECK_SYNC=1`` checks synchronously instead (the
    call that got the bad mask raises, before anything uses it).  Inside a HIP graph capture the
    check is attached to the graph (``graphs.note_capture_check``): ``GraphedStep`` copies the
    flag after every replay and raises at the next replay."""

    def __init__(self):
        self.dev = None
        self.host = None
        self.ev = None

    def flag(self, device):
        if self.dev is None or self.dev.device != device:
            self.dev = torch.zeros(1, dtype=torch.int32, device=device)
            self.host = torch.zeros(1, dtype=torch.int32, pin_memory=device.type == "cuda")
            self.ev = None
        return self.dev

    def _raise(self, what: str, late: bool) -> None:
        self.dev.zero_()
        if late:
            raise ValueError(f"nbd Llama: an attention_mask {what}.  It was seen in an EARLIER call, whose batch has "
                             "already been applied (its loss and gradients were computed on the fused path without "
                             "that mask, and may have gone through optimizer.step()).  NBD_MASK_CHECK_SYNC=1 raises "
                             "on the offending call instead; register a forward hook on the model to run the module "
                             "path, which honours any mask (models/llama.py module docstring)")
        raise ValueError(f"nbd Llama: attention_mask {what} (nothing of this batch was applied; register a forward "
                         "hook on the model to run the module path, which honours any mask)")

    def poll(self, fail_bits: int, what: str) -> None:
        if self.ev is not None and not torch.cuda.is_current_stream_capturing() and self.ev.query():
            v = int(self.host[0])
            self.ev = None
            if v & fail_bits:
                self._raise(what, late=True)

    def arm(self, fail_bits: int, what: str) -> None:
        if self.dev.device.type != "cuda":
            if int(self.dev[0]) & fail_bits:
                self._raise(what, late=False)
            return
        if torch.cuda.is_current_stream_capturing():
            from ..graphs import note_capture_check

            note_capture_check(_CapturedMaskCheck(self, fail_bits, what))
            return
        if _MASK_CHECK_SYNC:
            if int(self.dev[0]) & fail_bits:  # (a host sync: opt-in)
                self._raise(what, late=False)
            return
        self.host.copy_(self.dev, non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record()


class _CapturedMaskCheck:
    """A mask check captured into a HIP graph: the prep kernel (and its flag update) replays with
    the graph, so ``GraphedStep`` arms the flag's copy after each replay and polls it before the
    next one."""

    def __init__(self, chk: _MaskCheck, fail_bits: int, what: str):
        self.chk, self.fail_bits, self.what = chk, fail_bits, what

    def before_replay(self) -> None:
        self.chk.poll(self.fail_bits, self.what)

    def after_replay(self) -> None:
        self.chk.arm(self.fail_bits, self.what)


class LlamaModel(nn.Module):
    """Decoder stack; ``forward`` returns the final-normed hidden states [B, T, C]."""

    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.config = c
        self.embed_tokens = nn.Embedding(c.vocab_size, c.hidden_size)
        self.layers = nn.ModuleList([LlamaDecoderLayer(c) for _ in range(c.num_hidden_layers)])
        self.norm = RMSNorm(c.hidden_size, c.rms_norm_eps)
        self._rope: Dict[Any, tuple] = {}
        # fp32 parameters computed in this dtype on the fused GPU path (``native()``): the
        # parameters stay fp32 for the optimizer, each layer is cast once per forward
        self.compute_dtype: Optional[torch.dtype] = None
        # per-block HIP graphs for this model (0 / 1 / 2, ops.block_graphs); None = process setting
        self.block_graphs: Optional[int] = None
        # per-block HIP graphs (ops.block_graphs) hold static activations: drop this model's
        # graphs (only) with it
        self._bg_owner = next(_OWNER_IDS)
        weakref.finalize(self, _drop_block_graphs, self._bg_owner)
        self._hook_probe = None

    def cast_dtype(self, input_ids) -> Optional[torch.dtype]:
        """The dtype the fp32 parameters are cast to for this forward, or None (run as stored).
        Only where the whole stack takes the fused per-block path."""
        cd = self.compute_dtype
        if cd is None or not input_ids.is_cuda or self.embed_tokens.weight.dtype != torch.float32:
            return None
        c = self.config
        if c.head_dim != 64 or input_ids.shape[1] % 128 or not ops.native_available():
            return None
        for layer in self.layers:
            at = layer.self_attn
            if type(at) is not LlamaAttention or type(layer.mlp) is not LlamaMLP:
                return None
            if at.window is not None and input_ids.shape[1] > at.window:
                return None
        return cd

    def rope(self, T: int, device) -> tuple:
        key = (str(device), T)
        if key not in self._rope:  # built once per (device, length), outside any graph capture
            self._rope[key] = ops.rope_tables(T, self.config.head_dim, self.config.rope_theta, device,
                                              scaling=self.config.rope_scaling)
        return self._rope[key]

    def hooked(self) -> bool:
        """Any forward / backward hook on the embedding, a decoder layer, one of their submodules,
        the final norm — or a global module hook: then ``forward`` runs module by module."""
        key = (len(self.layers), id(self.layers[0]) if len(self.layers) else 0,
               id(self.layers[-1].self_attn) if len(self.layers) else 0, id(self.layers[-1].mlp) if len(self.layers) else 0)
        if self._hook_probe is None or self._hook_probe[0] != key:
            mods = [self.embed_tokens, self.norm] + [m for layer in self.layers for m in layer.modules()]
            dicts = []
            for m in mods:
                dicts += [m._forward_hooks, m._forward_pre_hooks, m._backward_hooks,
                          getattr(m, "_backward_pre_hooks", {})]
            self._hook_probe = (key, dicts)
        return any(self._hook_probe[1]) or _global_hooks()

    def forward_modules(self, input_ids, attention_mask=None):
        """Module-by-module forward in HF's structure (hooks fire; ``attention_mask`` masks keys
        exactly as HF does).  Parameters compute in their own dtype."""
        T = input_ids.shape[1]
        cos, sin = self.rope(T, input_ids.device)
        key_mask = None if attention_mask is None else attention_mask != 0
        x = self.embed_tokens(input_ids)
        for layer in self.layers:
            x = layer(x, cos, sin, key_mask) if key_mask is not None else layer(x, cos, sin)
        return self.norm(x)

    def forward(self, input_ids, cache=None, attention_mask=None):
        """``cache`` (a ``generation.KVCache``) receives every layer's rotated k and v.
        ``attention_mask`` given, or hooks registered: the module path (``forward_modules``)."""
        if cache is None and (attention_mask is not None or self.hooked()):
            return self.forward_modules(input_ids, attention_mask)
        c = self.config
        T = input_ids.shape[1]
        cos, sin = self.rope(T, input_ids.device)
        cd = self.cast_dtype(input_ids) if cache is None else None
        if cd is not None:
            return self._forward_cast(input_ids, cd, cos, sin)
        # the residual stream: each block's two residual adds are fused with the RMSNorm after them
        # (and the embedding with the first one)
        ln0 = self.layers[0].input_layernorm
        x, h = ops.embed_rms_norm(input_ids, self.embed_tokens.weight, ln0.weight, ln0.eps)
        for i, layer in enumerate(self.layers):
            nxt = self.layers[i + 1].input_layernorm if i + 1 < len(self.layers) else self.norm
            at = layer.self_attn
            # (plain modules only: tensor / context parallelism swap in their own attention / MLP)
            if (cache is None and type(at) is LlamaAttention and type(layer.mlp) is LlamaMLP
                    and (at.window is None or T <= at.window)):
                # the whole block as one autograd node (GPU bf16; None -> the op-by-op path below)
                r = ops.llama_block(x, h, at.qkv_proj.weight, at.qkv_proj.bias, at.o_proj.weight, at.o_proj.bias,
                                    layer.post_attention_layernorm.weight, layer.mlp.gate_up_proj.weight,
                                    layer.mlp.down_proj.weight, nxt.weight, at.H, at.Hkv, c.rms_norm_eps, cos, sin,
                                    self._graph_mode(), self._bg_owner)
                if r is not None:
                    x, h = r
                    continue
            a = layer.self_attn(h, cos, sin) if cache is None else layer.self_attn(h, cos, sin, kv=(cache, i))
            x, h = ops.add_rms_norm(x, a, layer.post_attention_layernorm.weight, c.rms_norm_eps)
            m = layer.mlp(h)
            x, h = ops.add_rms_norm(x, m, nxt.weight, c.rms_norm_eps)
        if h.is_cuda and self._graphs_on():
            # per-block graphs: the last block's output is its graph's static memory — the model's
            # output is the caller's to keep
            h = h.clone()
        return h

    def _graph_mode(self) -> int:
        return -1 if self.block_graphs is None else int(self.block_graphs)

    def _graphs_on(self) -> bool:
        if self.block_graphs is not None:
            return self.block_graphs > 0
        return ops.native_available() and ops.block_graphs() > 0

    def _forward_cast(self, input_ids, cd, cos, sin):
        """fp32 parameters, ``cd`` compute: the embedding gathers fp32 rows (no table cast) and
        casts them; each block's weights — with the NEXT norm's weight, so every parameter is
        cast exactly once — go through one fused cast (``_CastGroup``).  Every layer is cast
        before the first block runs: a stack graph (ops.block_graphs) replays all the blocks at the
        first block's call, so a cast issued between two block calls would land after the stack
        had read that layer's weights — the previous step's."""
        c = self.config
        x = ops.embedding(input_ids, self.embed_tokens.weight).to(cd)
        (w_in,) = cast_group(cd, [self.layers[0].input_layernorm.weight])
        h = ops.rms_norm(x, w_in, c.rms_norm_eps)
        per_layer = []
        for i, layer in enumerate(self.layers):
            nxt = self.layers[i + 1].input_layernorm if i + 1 < len(self.layers) else self.norm
            at, mlp = layer.self_attn, layer.mlp
            ps = [at.qkv_proj.weight, at.o_proj.weight, layer.post_attention_layernorm.weight,
                  mlp.gate_up_proj.weight, mlp.down_proj.weight, nxt.weight]
            if at.qkv_proj.bias is not None:
                ps.append(at.qkv_proj.bias)
            if at.o_proj.bias is not None:
                ps.append(at.o_proj.bias)
            per_layer.append(ps)
        # layers per cast node: all of them at world size 1 (one cast launch forward; backward, one
        # flush of the queued reductions and one cast back — instead of one of each per layer);
        # one per layer when gradients are all-reduced (DDP's buckets then fill as the backward
        # goes, overlapping the collectives with it).  NBD_NATIVE_CAST_LAYERS overrides.
        k = _cast_layers(len(per_layer))
        casts = []
        for g in range(0, len(per_layer), k):
            grp = per_layer[g:g + k]
            out = cast_group(cd, [p for ps in grp for p in ps])
            pos = 0
            for ps in grp:
                casts.append(out[pos:pos + len(ps)])
                pos += len(ps)
        for layer, ws in zip(self.layers, casts):
            at = layer.self_attn
            w_qkv, w_o, w_post, w_gu, w_down, w_next = ws[:6]
            extra = list(ws[6:])
            b_qkv = extra.pop(0) if at.qkv_proj.bias is not None else None
            b_o = extra.pop(0) if at.o_proj.bias is not None else None
            r = ops.llama_block(x, h, w_qkv, b_qkv, w_o, b_o, w_post, w_gu, w_down, w_next, at.H, at.Hkv,
                                c.rms_norm_eps, cos, sin, self._graph_mode(), self._bg_owner)
            if r is None:  # (cast_dtype() checked the conditions: not expected)
                qkv = ops.gemm_linear(h, w_qkv, b_qkv)
                a = ops.gemm_linear(ops.attention_qkv(qkv, at.H, causal=True, n_kv_head=at.Hkv, rope=(cos, sin)),
                                    w_o, b_o)
                x, h = ops.add_rms_norm(x, a, w_post, c.rms_norm_eps)
                x, h = ops.add_rms_norm(x, ops.mlp_swiglu(h, w_gu, w_down), w_next, c.rms_norm_eps)
            else:
                x, h = r
        if self._graphs_on():  # (see forward)
            h = h.clone()
        return h


def _cast_layers(n: int) -> int:
    env = os.environ.get("NBD_NATIVE_CAST_LAYERS")
    if env:
        return max(1, min(n, int(env)))
    import torch.distributed as dist

    return 1 if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1 else max(1, n)


class _LlamaPreTrained(nn.Module):
    def _init_weights(self) -> None:
        std = self.config.initializer_range
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, mean=0.0, std=std)
            if isinstance(m, nn.Linear) and m.bias is not None:
                nn.init.zeros_(m.bias)


class LlamaForSequenceClassification(_LlamaPreTrained):
    """HF ``LlamaForSequenceClassification`` semantics: score the rightmost non-pad token;
    cross-entropy loss when ``labels`` are given.  Returns ``SequenceClassifierOutput`` —
    a ``(loss, logits)`` tuple with ``.loss`` / ``.logits``, so a notebook written against the HF
    model (``out = model(input_ids=..., attention_mask=..., labels=...)``; ``out.loss``) runs
    unchanged on it."""

    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.config = c
        self.model = LlamaModel(c)
        self.score = nn.Linear(c.hidden_size, c.num_labels, bias=False)
        self._init_weights()

    def forward(self, input_ids, attention_mask=None, labels=None, **hf_kwargs):
        _check_hf_kwargs(hf_kwargs)
        if self.model.hooked():  # HF's structure, exact key masking: every hook fires
            h = self.model.forward_modules(input_ids, attention_mask)
            last = ops.mask._ref_seqcls_prep(input_ids, None, self.config.pad_token_id)[1]
        else:
            # fused path: left-padded rows rotated to right padding, pooled index in the rotated
            # rows — one kernel, no host sync (ops.seqcls_prep); holes are reported next call
            chk = self.__dict__.setdefault("_mask_check", _MaskCheck())
            chk.poll(1, "with holes (not one contiguous run per row) is not supported by the fused path")
            ids, last = ops.seqcls_prep(input_ids, attention_mask, self.config.pad_token_id,
                                        chk.flag(input_ids.device))
            chk.arm(1, "with holes (not one contiguous run per row) is not supported by the fused path")
            h = self.model(ids)
        B, T, C = h.shape
        w = self.score.weight
        no_hooks = not self.score._forward_hooks and not self.score._forward_pre_hooks
        if (labels is not None and self.score.bias is None and no_hooks and w.dtype == h.dtype
                and ops.tiny.seqcls_ok(h, w, labels.view(-1))):
            # the whole tail (pooling gather, score head, mean cross-entropy) in one HIP launch,
            # its backward in one (csrc/kernels/tiny.hip seqcls): ≈ 14 torch / library launches less
            loss, logits = ops.tiny.seqcls_head_loss(h, last, w, labels.view(-1))
            return SequenceClassifierOutput(loss, logits)
        # gather (backward = scatter-add: no sort, graph-safe) instead of advanced indexing
        pooled = torch.gather(h, 1, last.view(B, 1, 1).expand(B, 1, C)).squeeze(1)
        if (pooled.is_cuda and self.score.bias is None and no_hooks
                and ops.tiny.shape_ok(pooled, w.shape[0], w.shape[1])):
            # the classifier head (N = num_labels) on the tiny-linear HIP kernels: one launch
            # forward, one backward (dx, dW together) instead of three library GEMMs
            logits = ops.linear_tiny(pooled, w if w.dtype == pooled.dtype else w.to(pooled.dtype))
        else:
            logits = self.score(pooled) if w.dtype == pooled.dtype else F.linear(pooled, w.to(pooled.dtype))
        loss = None
        if labels is not None:
            loss = F.cross_entropy(logits.float(), labels.view(-1))
        return SequenceClassifierOutput(loss, logits)


class LlamaForCausalLM(_LlamaPreTrained):
    """Causal LM head (tied to the embedding when ``tie_word_embeddings``); the loss runs
    through the fused HIP cross-entropy on GPU.  Returns (loss, logits or None)."""

    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.config = c
        self.model = LlamaModel(c)
        self.lm_head = nn.Linear(c.hidden_size, c.vocab_size, bias=False)
        self._init_weights()
        if c.tie_word_embeddings:
            self.lm_head.weight = self.model.embed_tokens.weight

    def forward(self, input_ids, labels=None, return_logits: bool = True, attention_mask=None):
        """Next-token loss of ``labels`` (shifted here: ``logits[:, t]`` predicts ``labels[:, t+1]``).
        Under context parallelism (``parallel.context.parallelize_llama_context``) the shard's
        ``labels`` must come already shifted on the full sequence (``context.shift_labels``) and
        the loss is this rank's ``context_loss`` share of the group-wide token mean.
        ``attention_mask``: right padding on the fused path (real tokens' logits and the loss
        over them equal HF's; anything else is reported at the next call); with hooks registered
        any mask, exactly (the module path)."""
        if self.model.hooked():
            h = self.model.forward_modules(input_ids, attention_mask)
        else:
            if attention_mask is not None:
                chk = self.__dict__.setdefault("_mask_check", _MaskCheck())
                what = "that is not right-padded is not supported by the fused causal-LM path"
                chk.poll(3, what)
                ops.seqcls_prep(input_ids, attention_mask, None, chk.flag(input_ids.device))
                chk.arm(3, what)
            h = self.model(input_ids)
        logits = self.lm_head(h)
        loss = None
        if labels is not None:
            V = logits.shape[-1]
            cp = getattr(self, "context_group", None)
            if cp is None:  # next-token prediction
                shift, tgt, red = logits[:, :-1].reshape(-1, V), labels[:, 1:].reshape(-1), "mean"
            else:  # pre-shifted targets, one per position of the shard
                shift, tgt, red = logits.reshape(-1, V), labels.reshape(-1), "sum"
            loss = (ops.cross_entropy(shift, tgt, reduction=red) if logits.is_cuda
                    else F.cross_entropy(shift.float(), tgt, ignore_index=-100, reduction=red))
            if cp is not None:
                from ..parallel.context import context_loss

                loss = context_loss(loss, (tgt != -100).sum(), cp[0])
        return CausalLMOutput(loss, logits if return_logits else None)

    # ------------------------------------------------------------------ generation (generation.py)
    def kv_layout(self):
        """(layers, query heads, kv heads, head dim) of this rank's cache (its heads under TP)."""
        at = self.model.layers[0].self_attn
        return self.config.num_hidden_layers, at.H, at.Hkv, self.config.head_dim

    def max_positions(self) -> int:
        return self.config.max_position_embeddings

    def prefill_length(self, T: int) -> int:
        """Prompt length the prefill runs at: a multiple of 128 where that selects the HIP path."""
        p = self.lm_head.weight
        return -(-T // 128) * 128 if p.is_cuda and p.dtype in (torch.bfloat16, torch.float16) else T

    @torch.no_grad()
    def prefill(self, input_ids, cache, lengths):
        """Run the prompts (right-padded), fill ``cache``; logits [B, V] at positions lengths-1."""
        h = self.model(input_ids, cache=cache)
        B, _, C = h.shape
        last = torch.gather(h, 1, (lengths - 1).view(B, 1, 1).expand(B, 1, C)).squeeze(1)
        return self.lm_head(last)

    @torch.no_grad()
    def decode_step(self, tok, pos, cache):
        """Logits [B, V] of one new token per sequence (``tok``, ``pos``: int64 [B]); appends to
        ``cache``.  Device-side only (graph-capturable)."""
        m, c = self.model, self.config
        rope = m.rope(cache.t_max, tok.device)
        x = ops.embedding(tok, m.embed_tokens.weight)
        eps = c.rms_norm_eps
        # four fused kernels + attention per block (ops.linear_small: RMSNorm prologue, SwiGLU /
        # residual epilogues); tensor-parallel layers (parallel.tensor) add one all-reduce per half
        for i, layer in enumerate(m.layers):
            x = layer.self_attn.decode(x, layer.input_layernorm.weight, eps, cache, i, pos, rope)
            x = layer.mlp.decode(x, layer.post_attention_layernorm.weight, eps)
        return ops.linear_small(x, self.lm_head.weight, norm=("rms", m.norm.weight, eps))

    def generate(self, input_ids, max_new_tokens: int, **kw):
        """``generation.generate`` (KV cache, HIP decode attention, graph-captured decode loop)."""
        from ..generation import generate

        return generate(self, input_ids, max_new_tokens, **kw)


# ---------------------------------------------------------------------------- HF interop
def hf_to_nbd_state_dict(sd: Dict[str, torch.Tensor], c: LlamaConfig) -> Dict[str, torch.Tensor]:
    """Map an HF Llama state dict (q/k/v and gate/up as separate projections) onto this layout
    (fused q|k|v and gate|up projections)."""
    out: Dict[str, torch.Tensor] = {}
    for k, v in sd.items():
        if ".self_attn.q_proj." in k or ".self_attn.k_proj." in k or ".self_attn.v_proj." in k:
            continue
        if ".mlp.gate_proj." in k or ".mlp.up_proj." in k:
            continue
        if k.endswith("rotary_emb.inv_freq"):
            continue
        out[k] = v
    for i in range(c.num_hidden_layers):
        p = f"model.layers.{i}"
        out[f"{p}.self_attn.qkv_proj.weight"] = torch.cat(
            [sd[f"{p}.self_attn.q_proj.weight"], sd[f"{p}.self_attn.k_proj.weight"], sd[f"{p}.self_attn.v_proj.weight"]])
        if f"{p}.self_attn.q_proj.bias" in sd:
            out[f"{p}.self_attn.qkv_proj.bias"] = torch.cat(
                [sd[f"{p}.self_attn.q_proj.bias"], sd[f"{p}.self_attn.k_proj.bias"], sd[f"{p}.self_attn.v_proj.bias"]])
        out[f"{p}.mlp.gate_up_proj.weight"] = torch.cat([sd[f"{p}.mlp.gate_proj.weight"], sd[f"{p}.mlp.up_proj.weight"]])
    return out


# keyword arguments an HF call may pass that change nothing here
_HF_NEUTRAL = {"return_dict": (True, None), "output_attentions": (False, None), "output_hidden_states": (False, None),
               "use_cache": (False, None, True), "token_type_ids": (None,), "position_ids": (None,)}


def _check_hf_kwargs(kw) -> None:
    for k, v in kw.items():
        if k not in _HF_NEUTRAL or not any(v is x or (x is not None and v == x) for x in _HF_NEUTRAL[k]):
            raise TypeError(f"nbd Llama: unsupported argument {k}={v!r}")


def from_hf(hf_model, compute_dtype: Optional[torch.dtype] = None) -> nn.Module:
    """Build the equivalent nbd model from an instantiated HF Llama sequence-classification or
    causal-LM model (weights copied, same dtype and device).  ``compute_dtype`` (e.g. bf16) with
    fp32 weights: keep the fp32 parameters (the optimizer's master copy) and run the fused HIP
    path in that dtype (mixed precision, one cast per decoder layer — ``LlamaModel.compute_dtype``)."""
    c = LlamaConfig.from_hf(hf_model.config)
    cls = LlamaForSequenceClassification if hasattr(hf_model, "score") else LlamaForCausalLM
    m = cls(c)
    sd = hf_to_nbd_state_dict(hf_model.state_dict(), c)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not (k == "lm_head.weight" and c.tie_word_embeddings)]
    if missing or unexpected:
        raise ValueError(f"from_hf: missing {missing}, unexpected {unexpected}")
    p0 = next(hf_model.parameters())
    m = m.to(device=p0.device, dtype=p0.dtype)
    m.train(hf_model.training)
    if compute_dtype is not None and compute_dtype != p0.dtype:
        m.model.compute_dtype = compute_dtype
    return m


def native(hf_model, compute_dtype: Optional[torch.dtype] = torch.bfloat16, fused_optimizer: bool = True,
           block_graphs: Optional[int] = None) -> nn.Module:
    """The one-line swap for a notebook written against HF transformers: call it on the HF
    Llama / SmolLM2 / Qwen2 / Mistral model BEFORE creating the optimizer and
    ``accelerator.prepare``.  The returned module takes the same keyword arguments, returns
    outputs with ``.loss`` / ``.logits``, keeps the HF parameters' dtype (fp32 master weights for
    ``torch.optim.AdamW``) and computes in ``compute_dtype`` on the fused HIP path (bf16 by
    default: the same mixed-precision recipe as ``Accelerator(mixed_precision="bf16")``).

    ``fused_optimizer``: a ``torch.optim.AdamW`` / ``Adam`` later built on exactly this model's GPU
    parameters, with neither ``fused`` nor ``foreach`` given, uses torch's fused (one kernel per
    step) implementation instead of the multi-tensor default — the same update, and on the
    notebook's SmolLM2 step the default's optimizer phase is 3.0-5.8 ms of GPU time against
    0.9 ms fused (docs/FINDINGS.md §30); an ``AdamW`` then steps through ``nbd::adamw_tensors``
    (one HIP launch per 128 parameters, torch's state; ``NBD_NATIVE_NBD_ADAMW=0`` keeps torch's
    fused kernel).  Other optimizers and parameters are untouched; ``NBD_NATIVE_FUSED_OPTIM=0``
    or ``fused_optimizer=False`` keeps torch's default.

    ``block_graphs``: each decoder block's forward replayed from its own HIP graph (1, the
    default; 2 adds the backward where gradients go to DDP bucket slices; 0 off — also with
    ``NBD_BLOCK_GRAPHS=0``): the swapped loop's forward is host-bound (docs/FINDINGS.md §30).
    The model's output is a fresh tensor as always; block-internal activations stay allocated
    between steps (at most 4 sequence lengths per block are graphed)."""
    m = from_hf(hf_model, compute_dtype=compute_dtype)
    if block_graphs is None:
        block_graphs = int(os.environ.get("NBD_NATIVE_BLOCK_GRAPHS", "1"))
    if os.environ.get("NBD_BLOCK_GRAPHS") == "0":
        block_graphs = 0
    if hasattr(m, "model") and isinstance(m.model, LlamaModel):
        m.model.block_graphs = int(block_graphs)
    # the decoder blocks write the cast weights' gradients into kept buffers (autograd.hip
    # CastGroupFn): their split-K and norm-column reductions can be queued and issued together
    # (graddst.h defer; the cast node's backward flushes them) — 4 launches per layer become 2
    if os.environ.get("NBD_GRAD_DEFER", "1") != "0" and ops.native_available():
        ops.graddst.defer_enable(True)
    if fused_optimizer and os.environ.get("NBD_NATIVE_FUSED_OPTIM", "1") != "0":
        for p in m.parameters():
            p._nbd_native_fused = True
        _install_fused_default()
        global _NATIVE_LIVE
        _NATIVE_LIVE += 1
        weakref.finalize(m, _native_released)
    return m


# torch.optim.AdamW / Adam __init__ wrapped while native() models are alive: originals + wrappers
_FUSED_ORIG: Dict[type, Any] = {}
_FUSED_WRAP: Dict[type, Any] = {}
_NATIVE_LIVE = 0
_LOG = logging.getLogger("nbdistributed_amd")
_LOGGED = [False]


def _native_released() -> None:
    global _NATIVE_LIVE
    _NATIVE_LIVE -= 1
    if _NATIVE_LIVE <= 0:
        _NATIVE_LIVE = 0
        restore_optimizer_defaults()


def restore_optimizer_defaults() -> None:
    """Undo ``native()``'s fused-AdamW default now (it is undone by itself when the last
    ``native()`` model is garbage-collected).  A wrapper someone installed over ours stays."""
    for cls, orig in list(_FUSED_ORIG.items()):
        if cls.__init__ is _FUSED_WRAP.get(cls):
            cls.__init__ = orig
        _FUSED_ORIG.pop(cls, None)
        _FUSED_WRAP.pop(cls, None)


def _install_fused_default() -> None:
    """Wrap ``torch.optim.AdamW.__init__`` / ``Adam.__init__`` while ``native()`` models live:
    when ``fused`` and ``foreach`` are both unspecified and every parameter is a CUDA
    floating-point parameter of a ``native()`` model, pass ``fused=True``.  Said once in the log;
    undone when the last such model is collected (or ``restore_optimizer_defaults()``)."""
    import functools

    for cls in (torch.optim.AdamW, torch.optim.Adam):
        if cls in _FUSED_ORIG:
            continue
        orig = cls.__init__

        def make(orig):
            @functools.wraps(orig)
            def __init__(self, params, *args, **kwargs):
                ours = False
                if kwargs.get("fused") is None and kwargs.get("foreach") is None:
                    params = list(params)
                    flat = [p for g in params for p in (g["params"] if isinstance(g, dict) else [g])]
                    if flat and all(isinstance(p, torch.Tensor) and getattr(p, "_nbd_native_fused", False) and p.is_cuda
                                    and p.is_floating_point() for p in flat):
                        kwargs["fused"] = True
                        ours = True
                orig(self, params, *args, **kwargs)
                if ours and os.environ.get("NBD_NATIVE_NBD_ADAMW", "1") != "0":
                    # AdamW: the same update as one HIP launch per <= 128 parameters, torch's state
                    # layout (optim.install_fast_adamw; torch's fused step whenever they could differ)
                    from ..optim import install_fast_adamw

                    install_fast_adamw(self)

            return __init__

        w = make(orig)
        _FUSED_ORIG[cls] = orig
        _FUSED_WRAP[cls] = w
        cls.__init__ = w
    if not _LOGGED[0]:
        _LOGGED[0] = True
        _LOG.warning("nbdistributed_amd: native(): torch.optim.AdamW/Adam built on a native() model's GPU parameters "
                     "without fused=/foreach= use fused=True (the same update, one kernel); restored when the last "
                     "native() model is collected. Keep torch's default with native(..., fused_optimizer=False) or "
                     "NBD_NATIVE_FUSED_OPTIM=0.")


__all__ = ["LlamaConfig", "LlamaModel", "LlamaForSequenceClassification", "LlamaForCausalLM", "RMSNorm",
           "from_hf", "native", "hf_to_nbd_state_dict", "SequenceClassifierOutput", "CausalLMOutput",
           "restore_optimizer_defaults"]
