"""GPT-2 (124M "small" by default) for the BASELINE config-5 DDP loop.

BASELINE.json config 5: "00_accelerate.ipynb-style GPT-2-small DDP loop, bf16, synthetic tokens"
(124,439,808 parameters with the tied LM head).  On MI355X in bf16 the hot path
is the framework's own gfx950 kernels: every transformer Linear runs on the hand-written MFMA
GEMMs (``ops.gemm_linear`` / ``ops.mlp_gelu``: csrc/kernels/gemm.hip, fused bias / GELU
epilogues, grouped dgrad + wgrad backward writing into the DDP buckets), attention on the HIP
flash kernels (``ops.attention_qkv``, csrc/kernels/attn.hip), add + LayerNorm on norm.hip and the
loss on the fused HIP cross-entropy (``ops.linear_cross_entropy``, no fp32 copy of the
8192 x 50257 logits).  The tied LM-head products (8192 x 50432 x 768, three per step) follow the
plan the step measured fastest (``ops.loss.HEAD_PRODUCTS``): the weight gradient on the
hand-written 256x256 kernel (gemm256.hip; the table padded to a multiple of 256 for it), the
forward and input gradient on hipBLASLt (docs/FINDINGS.md §35; ``NBD_LMHEAD_HIP=1`` all three
hand-written, ``=0`` all three on the library with a 128-padded table).  CPU / fp32: the same
model in plain PyTorch.
Random init (no checkpoints: no network), GPT-2 initialisation scheme.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


def _table_pad() -> int:
    from ..ops.loss import table_pad

    return table_pad()


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    dropout: float = 0.0
    bias: bool = True
    tie_weights: bool = True
    fused_ce: bool = True  # GPU: nbd.ops.cross_entropy (HIP) instead of F.cross_entropy(logits.float())
    fused_attn: bool = True  # GPU bf16: nbd.ops.attention_qkv (HIP flash fwd/bwd) instead of SDPA
    fused_norm: bool = True  # GPU, no autocast: HIP residual-add+LayerNorm and bias-grad kernels
    hip_gemm: bool = True  # GPU bf16 fast path: Linear layers on the HIP MFMA GEMM (GELU fused in its epilogues)
    # the token table (and the tied LM head) is stored with its rows padded to a multiple of this
    # from 4096 classes up: zero rows that never receive a gradient, so the LM-head GEMMs run on an
    # aligned vocabulary (hipBLASLt on 50257 vs 50304 columns: 2.18 vs 1.75 ms per GPT-2 step,
    # docs/FINDINGS.md §16) with no per-step padded copy of the weight.  1 = no padding.  The
    # multiple follows the LM head's kernel plan (ops.loss.table_pad: 256 for the default plan's
    # hand-written weight gradient on 256x256 tiles, 512 when the input gradient is hand-written too,
    # 128 for hipBLASLt alone); NBD_GPT2_VOCAB_PAD overrides (A/B measurements).
    vocab_pad: int = field(default_factory=lambda: int(os.environ.get("NBD_GPT2_VOCAB_PAD", "0")) or _table_pad())

    @property
    def padded_vocab(self) -> int:
        v, a = self.vocab_size, max(1, self.vocab_pad)
        return -(-v // a) * a if v >= 4096 else v

    @classmethod
    def small(cls):
        return cls()

    @classmethod
    def tiny(cls):
        return cls(vocab_size=512, n_positions=128, n_embd=64, n_layer=2, n_head=4)


class CausalSelfAttention(nn.Module):
    def __init__(self, c: GPT2Config):
        super().__init__()
        assert c.n_embd % c.n_head == 0
        self.n_head = c.n_head
        self.fused = c.fused_attn
        self.c_attn = nn.Linear(c.n_embd, 3 * c.n_embd, bias=c.bias)
        self.c_proj = nn.Linear(c.n_embd, c.n_embd, bias=c.bias)
        self.dropout = c.dropout
        self.hip_gemm = c.hip_gemm

    def forward(self, x: torch.Tensor, fast: bool = False, kv=None) -> torch.Tensor:
        """``kv`` = (KVCache, layer): prefill for generation (k and v of every position stored)."""
        B, T, C = x.shape
        if fast:  # HIP path: bias grads by the column-sum kernel, flash attention on the packed QKV
            from .. import ops

            lin = ops.gemm_linear if self.hip_gemm else ops.linear
            qkv = lin(x, self.c_attn.weight, self.c_attn.bias)
            if kv is not None:
                kv[0].store(kv[1], qkv)
            return lin(ops.attention_qkv(qkv, self.n_head, causal=True), self.c_proj.weight, self.c_proj.bias)
        qkv = self.c_attn(x)
        if kv is not None:
            kv[0].store(kv[1], qkv)
        if self.fused and qkv.is_cuda and (self.dropout == 0.0 or not self.training):
            from .. import ops

            return self.c_proj(ops.attention_qkv(qkv, self.n_head, causal=True))
        q, k, v = qkv.split(C, dim=2)
        hd = C // self.n_head
        q = q.view(B, T, self.n_head, hd).transpose(1, 2)
        k = k.view(B, T, self.n_head, hd).transpose(1, 2)
        v = v.view(B, T, self.n_head, hd).transpose(1, 2)
        y = F.scaled_dot_product_attention(q, k, v, is_causal=True, dropout_p=self.dropout if self.training else 0.0)
        y = y.transpose(1, 2).reshape(B, T, C)
        return self.c_proj(y)


    def decode(self, x, ln, cache, layer: int, pos):
        """One token per sequence (generation): ``x + c_proj(attn(ln(x)))``, three fused kernels."""
        from .. import ops

        qkv = ops.linear_small(x, self.c_attn.weight, self.c_attn.bias, norm=("ln", ln.weight, ln.bias, ln.eps))
        a = cache.attend(layer, qkv, pos)
        return ops.linear_small(a, self.c_proj.weight, self.c_proj.bias, residual=x)


class MLP(nn.Module):
    def __init__(self, c: GPT2Config):
        super().__init__()
        self.c_fc = nn.Linear(c.n_embd, 4 * c.n_embd, bias=c.bias)
        self.c_proj = nn.Linear(4 * c.n_embd, c.n_embd, bias=c.bias)
        self.hip_gemm = c.hip_gemm

    def forward(self, x: torch.Tensor, fast: bool = False) -> torch.Tensor:
        if fast:
            from .. import ops

            if self.hip_gemm:  # GELU and GELU' ride in the GEMM epilogues
                return ops.mlp_gelu(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias)
            h = F.gelu(ops.linear(x, self.c_fc.weight, self.c_fc.bias), approximate="tanh")
            return ops.linear(h, self.c_proj.weight, self.c_proj.bias)
        return self.c_proj(F.gelu(self.c_fc(x), approximate="tanh"))

    def decode(self, x, ln):
        """``x + mlp(ln(x))`` for a few token rows: two fused kernels (norm + GELU, bias + residual)."""
        from .. import ops

        f = ops.linear_small(x, self.c_fc.weight, self.c_fc.bias, norm=("ln", ln.weight, ln.bias, ln.eps), act="gelu")
        return ops.linear_small(f, self.c_proj.weight, self.c_proj.bias, residual=x)


class Block(nn.Module):
    def __init__(self, c: GPT2Config):
        super().__init__()
        self.ln_1 = nn.LayerNorm(c.n_embd, bias=c.bias)
        self.attn = CausalSelfAttention(c)
        self.ln_2 = nn.LayerNorm(c.n_embd, bias=c.bias)
        self.mlp = MLP(c)

    def forward(self, x: torch.Tensor, kv=None) -> torch.Tensor:
        h = self.ln_1(x)
        x = x + (self.attn(h) if kv is None else self.attn(h, kv=kv))
        return x + self.mlp(self.ln_2(x))


class GPT2(nn.Module):
    def __init__(self, config: Optional[GPT2Config] = None):
        super().__init__()
        c = config or GPT2Config()
        self.config = c
        Vp = c.padded_vocab
        self.wte = nn.Embedding(Vp, c.n_embd)
        self.wpe = nn.Embedding(c.n_positions, c.n_embd)
        self.h = nn.ModuleList([Block(c) for _ in range(c.n_layer)])
        self.ln_f = nn.LayerNorm(c.n_embd, bias=c.bias)
        self.lm_head = nn.Linear(c.n_embd, Vp, bias=False)
        if c.tie_weights:
            self.lm_head.weight = self.wte.weight
        self.apply(self._init)
        for n, p in self.named_parameters():
            if n.endswith("c_proj.weight"):
                nn.init.normal_(p, mean=0.0, std=0.02 / math.sqrt(2 * c.n_layer))
        if Vp != c.vocab_size:
            with torch.no_grad():  # the pad rows stay zero: no id reaches them, their gradient is 0
                self.wte.weight[c.vocab_size:].zero_()
                self.lm_head.weight[c.vocab_size:].zero_()
        # the table's padding (vocab_pad) is a storage choice of the process that built the model
        # (it follows which kernel runs the LM head): a state_dict saved with another padding —
        # or the unpadded HF layout — loads by zero-padding / trimming the rows past vocab_size
        self._register_load_state_dict_pre_hook(self._repad_vocab)

    def _repad_vocab(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                     error_msgs) -> None:
        c = self.config
        Vp, V = c.padded_vocab, c.vocab_size
        for name in ("wte.weight", "lm_head.weight"):
            k = prefix + name
            t = state_dict.get(k)
            if not isinstance(t, torch.Tensor) or t.dim() != 2 or t.shape[0] == Vp or t.shape[0] < V:
                continue
            if t.shape[1] != c.n_embd:
                continue  # a genuine mismatch: load_state_dict reports it
            if t.shape[0] > Vp:
                extra = t[Vp:]
                if extra.numel() and bool((extra != 0).any()):
                    error_msgs.append(f"{k}: rows {Vp}..{t.shape[0] - 1} past the vocabulary ({V}) are not zero; "
                                      "they cannot be trimmed to this model's padding")
                    continue
                state_dict[k] = t[:Vp]
            else:
                state_dict[k] = torch.cat([t, t.new_zeros(Vp - t.shape[0], t.shape[1])])

    @staticmethod
    def _init(m: nn.Module) -> None:
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, mean=0.0, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, mean=0.0, std=0.02)

    @property
    def fused_attn_ok(self) -> bool:
        c = self.config
        return c.fused_attn and c.n_embd // c.n_head == 64 and (c.dropout == 0.0 or not self.training)

    def _fast(self, x: torch.Tensor) -> bool:
        c = self.config
        return (c.fused_norm and c.bias and x.is_cuda and not torch.is_autocast_enabled()
                and x.dtype in (torch.bfloat16, torch.float16) and c.n_embd % 8 == 0 and c.n_embd <= 2048
                and x.shape[1] % 128 == 0)

    def _fast_ok(self, idx: torch.Tensor) -> bool:
        c = self.config
        return (c.fused_norm and idx.is_cuda and not torch.is_autocast_enabled()
                and self.wte.weight.dtype in (torch.bfloat16, torch.float16))

    def num_params(self) -> int:
        """Parameters of the architecture (the vocabulary's pad rows not counted)."""
        pad = (self.config.padded_vocab - self.config.vocab_size) * self.config.n_embd
        return sum(p.numel() for p in self.parameters()) - pad * (1 if self.config.tie_weights else 2)

    def _logits(self, h: torch.Tensor) -> torch.Tensor:
        logits = self.lm_head(h)
        V = self.config.vocab_size
        return logits[..., :V] if logits.shape[-1] != V else logits

    def _positions(self, T: int, device) -> torch.Tensor:
        """``arange(T)`` on ``device``, kept between calls (one launch less per step; made only
        outside a stream capture, so a captured graph never owns the kept tensor)."""
        cache = self.__dict__.setdefault("_pos_cache", {})
        key = (T, str(device))
        p = cache.get(key)
        if p is None:
            p = torch.arange(T, device=device)
            if not (p.is_cuda and torch.cuda.is_current_stream_capturing()):
                cache[key] = p
        return p

    def _trunk(self, idx: torch.Tensor, cache=None):
        """Final-normed hidden states [B, T, C] (and whether the HIP fast path ran); ``cache``
        (a ``generation.KVCache``) receives every layer's k / v."""
        B, T = idx.shape
        pos_fn = getattr(self, "position_ids", None)  # set by parallel.context (global positions)
        pos = pos_fn(T, idx.device) if pos_fn is not None else self._positions(T, idx.device)
        c = self.config
        fused_in = (self._fast_ok(idx) and c.fused_norm and c.bias and c.n_embd % 8 == 0 and c.n_embd <= 2048
                    and T % 128 == 0 and c.n_layer > 0)
        if fused_in:
            # the input and the first LayerNorm as one node (and one launch)
            from .. import ops

            ln = self.h[0].ln_1
            x, h = ops.tokpos_layer_norm(idx, self.wte.weight, pos, self.wpe.weight, c.vocab_size, ln.weight,
                                         ln.bias, ln.eps)
        elif self._fast_ok(idx):
            from .. import ops

            x = ops.embedding_tok_pos(idx, self.wte.weight, pos, self.wpe.weight, self.config.vocab_size)
        else:
            x = self.wte(idx) + self.wpe(pos)
        if fused_in or self._fast(x):
            # residual stream through the HIP add+LayerNorm kernels: each block's two residual adds
            # are fused with the LayerNorm that follows them (ln_2, then the next block's ln_1 / ln_f)
            from .. import ops

            if not fused_in:
                ln = self.h[0].ln_1
                h = ops.layer_norm(x, ln.weight, ln.bias, ln.eps)
            for i, blk in enumerate(self.h):
                fa = self.fused_attn_ok
                a = blk.attn(h, fast=fa) if cache is None else blk.attn(h, fast=fa, kv=(cache, i))
                x, h = ops.add_layer_norm(x, a, blk.ln_2.weight, blk.ln_2.bias, blk.ln_2.eps)
                nxt = self.h[i + 1].ln_1 if i + 1 < c.n_layer else self.ln_f
                x, h = ops.add_layer_norm(x, blk.mlp(h, fast=True), nxt.weight, nxt.bias, nxt.eps)
            return h, True
        for i, blk in enumerate(self.h):
            x = blk(x) if cache is None else blk(x, kv=(cache, i))
        return self.ln_f(x), False

    def forward(self, idx: torch.Tensor, targets: Optional[torch.Tensor] = None, return_logits: bool = True):
        """Returns (logits, loss).  With ``targets`` and ``return_logits=False`` the logits are
        not returned (None) and the fused loss writes its gradient over their storage."""
        cp = getattr(self, "context_group", None)  # set by parallel.context: (group,)
        h, fast = self._trunk(idx)
        c = self.config
        if fast and targets is not None and not return_logits and c.fused_ce:
            from .. import ops

            if ops.loss.FUSED_XENT:
                # LM head + loss: one pass over the logits for the loss forward and backward
                red = "sum" if cp is not None else "mean"
                return None, self._cp_loss(ops.linear_cross_entropy(h, self.lm_head.weight, targets, reduction=red,
                                                                    vocab=c.vocab_size), targets, cp)
        logits = self._logits(h)
        loss = None
        if targets is not None:
            flat, tgt = logits.reshape(-1, logits.size(-1)), targets.reshape(-1)
            red = "sum" if cp is not None else "mean"
            if self.config.fused_ce and logits.is_cuda:
                from .. import ops

                loss = ops.cross_entropy(flat, tgt, reduction=red, inplace_backward=not return_logits)
            else:
                loss = F.cross_entropy(flat.float(), tgt, reduction=red)
            loss = self._cp_loss(loss, targets, cp)
        return (logits if return_logits or targets is None else None), loss

    @classmethod
    def from_hf(cls, hf_model) -> "GPT2":
        """The equivalent model from an instantiated HF ``GPT2LMHeadModel`` / ``GPT2Model`` (weights
        copied; HF's Conv1D [in, out] weights transposed to nn.Linear [out, in])."""
        hc = hf_model.config
        if getattr(hc, "activation_function", "gelu_new") not in ("gelu_new", "gelu_pytorch_tanh"):
            raise NotImplementedError(f"GPT2.from_hf: activation {hc.activation_function!r}")
        c = GPT2Config(vocab_size=hc.vocab_size, n_positions=hc.n_positions, n_embd=hc.n_embd, n_layer=hc.n_layer,
                       n_head=hc.n_head, tie_weights=bool(getattr(hc, "tie_word_embeddings", True)))
        m = cls(c)
        for blk in m.h:
            for ln in (blk.ln_1, blk.ln_2):
                ln.eps = hc.layer_norm_epsilon
        m.ln_f.eps = hc.layer_norm_epsilon
        sd = {}
        Vp = c.padded_vocab
        for k, v in hf_model.state_dict().items():
            k = k[len("transformer."):] if k.startswith("transformer.") else k
            if k.endswith(".attn.bias") or k.endswith(".attn.masked_bias"):
                continue  # causal-mask buffers of older transformers
            if k.endswith(".weight") and any(f".{n}.weight" in "." + k for n in ("c_attn", "c_proj", "c_fc")):
                v = v.t()
            if k in ("wte.weight", "lm_head.weight") and v.shape[0] != Vp:  # zero pad rows
                v = torch.cat([v, v.new_zeros(Vp - v.shape[0], v.shape[1])])
            sd[k] = v
        missing, unexpected = m.load_state_dict(sd, strict=False)
        missing = [k for k in missing if not (k == "lm_head.weight" and c.tie_weights)]
        if missing or unexpected:
            raise ValueError(f"GPT2.from_hf: missing {missing}, unexpected {unexpected}")
        return m.to(next(hf_model.parameters()).dtype)

    # ------------------------------------------------------------------ generation (generation.py)
    def kv_layout(self):
        """(layers, query heads, kv heads, head dim) of this rank's cache (its heads under TP)."""
        c = self.config
        h = self.h[0].attn.n_head
        return c.n_layer, h, h, c.n_embd // c.n_head

    def max_positions(self) -> int:
        return self.config.n_positions

    def prefill_length(self, T: int) -> int:
        """Prompt length the prefill runs at: a multiple of 128 where that selects the HIP path."""
        p = self.wte.weight
        return -(-T // 128) * 128 if p.is_cuda and p.dtype in (torch.bfloat16, torch.float16) else T

    @torch.no_grad()
    def prefill(self, idx: torch.Tensor, cache, lengths: torch.Tensor) -> torch.Tensor:
        """Run the prompts (right-padded), fill ``cache``; logits [B, V] at positions lengths-1."""
        h, _ = self._trunk(idx, cache)
        B, _, C = h.shape
        last = torch.gather(h, 1, (lengths - 1).view(B, 1, 1).expand(B, 1, C)).squeeze(1)
        return self._logits(last)

    @torch.no_grad()
    def decode_step(self, tok: torch.Tensor, pos: torch.Tensor, cache) -> torch.Tensor:
        """Logits [B, V] of one new token per sequence (``tok``, ``pos``: int64 [B]); appends to
        ``cache``.  Device-side only (graph-capturable)."""
        from .. import ops

        c = self.config
        if self._fast_ok(tok):
            x = ops.embedding_tok_pos(tok.view(1, -1), self.wte.weight, pos, self.wpe.weight,
                                      c.vocab_size).view(-1, c.n_embd)
        else:
            x = self.wte(tok) + self.wpe(pos)
        # five fused kernels per block (ops.linear_small: norm prologue, bias / GELU / residual
        # epilogue); tensor-parallel blocks (parallel.tensor) add one all-reduce after each half
        for i, blk in enumerate(self.h):
            x = blk.attn.decode(x, blk.ln_1, cache, i, pos)
            x = blk.mlp.decode(x, blk.ln_2)
        # the first vocab_size rows of the (padded) table: a contiguous view, no copy
        w = self.lm_head.weight[:c.vocab_size]
        return ops.linear_small(x, w, norm=("ln", self.ln_f.weight, self.ln_f.bias, self.ln_f.eps))

    def generate(self, idx: torch.Tensor, max_new_tokens: int, **kw) -> torch.Tensor:
        """``generation.generate`` (KV cache, HIP decode attention, graph-captured decode loop)."""
        from ..generation import generate

        return generate(self, idx, max_new_tokens, **kw)

    @staticmethod
    def _cp_loss(loss, targets, cp):
        """Context parallelism (``parallel.context.parallelize_gpt2_context``): ``loss`` is this
        rank's sum; return its share of the group-wide token mean (``context_loss``)."""
        if cp is None:
            return loss
        from ..parallel.context import context_loss

        return context_loss(loss, (targets != -100).sum(), cp[0])
