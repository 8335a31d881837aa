"""Autoregressive generation with a KV cache for the framework's causal LMs (GPT-2, Llama).

The reference's notebooks train; after training, a user of an interactive notebook wants to
*sample* from the model in the next cell.  ``generate`` does that MI355X-first:

* **prefill** — one pass over the (right-padded) prompts through the model's training kernels
  (HIP flash attention, fused GEMMs), storing each layer's k (rotated) and v into a
  ``KVCache`` laid out [layer, batch, kv-head, position, 64] so a decode step streams one
  contiguous run of rows per head;
* **decode** — one token per sequence per step: GEMMs on hipBLASLt (M = batch rows), and one HIP
  kernel per layer for RoPE + cache append + split-key attention with its merge
  (``ops.decode_attention``, ``csrc/kernels/decode.hip``);
* the positions live on the device, so the whole decode step — sampling included (Gumbel-max on
  the device RNG) — is captured once into a HIP graph and replayed per token: no host launch
  cost and no host sync per token (sequences that reach ``eos_token_id`` keep emitting it; the
  host checks for all-finished every ``sync_every`` tokens).

Models opt in by providing ``kv_layout()``, ``prefill(ids, cache, lengths)`` and
``decode_step(tok, pos, cache)``; see ``models/gpt2.py`` and ``models/llama.py``.
"""
from __future__ import annotations

from typing import Optional

import torch


class KVCache:
    """k / v caches [n_layer, B, Hkv, t_max, D] plus the decode kernel's workspace."""

    def __init__(self, n_layer: int, batch: int, n_head: int, n_kv: int, t_max: int, head_dim: int,
                 dtype=torch.bfloat16, device="cuda"):
        self.n_layer, self.batch, self.n_head, self.n_kv, self.t_max, self.head_dim = (
            n_layer, batch, n_head, n_kv, t_max, head_dim)
        shape = (n_layer, batch, n_kv, t_max, head_dim)
        self.k = torch.zeros(shape, dtype=dtype, device=device)
        self.v = torch.zeros(shape, dtype=dtype, device=device)
        from .ops.decode import partials_numel

        self.workspace = torch.empty(partials_numel(batch, n_head, t_max), dtype=torch.float32, device=device)
        self.kv_len_max: Optional[int] = None  # host bound on max(pos) + 1 (None = t_max)

    @classmethod
    def for_model(cls, model, batch: int, t_max: int, device=None, dtype=None) -> "KVCache":
        L, H, Hkv, D = model.kv_layout()
        p = next(model.parameters())
        return cls(L, batch, H, Hkv, t_max, D, dtype=dtype or p.dtype, device=device or p.device)

    @property
    def nbytes(self) -> int:
        return 2 * self.k.numel() * self.k.element_size()

    def store(self, layer: int, qkv: torch.Tensor, rope=None) -> None:
        """Prefill: copy k (rotated by ``rope`` = (cos, sin)) and v of a packed [B, T, W]
        projection into positions [0, T) of ``layer``."""
        from . import ops

        B, T, _ = qkv.shape
        H, Hkv, D = self.n_head, self.n_kv, self.head_dim
        if T > self.t_max:
            raise ValueError(f"KVCache.store: {T} positions > t_max {self.t_max}")
        k = qkv[:, :, H * D:(H + Hkv) * D]
        if rope is not None:
            k = ops.rope_(k.contiguous(), rope[0], rope[1], Hkv, D)
        self.k[layer, :, :, :T] = k.reshape(B, T, Hkv, D).transpose(1, 2)
        self.v[layer, :, :, :T] = qkv[:, :, (H + Hkv) * D:].reshape(B, T, Hkv, D).transpose(1, 2)

    def attend(self, layer: int, qkv: torch.Tensor, pos: torch.Tensor, rope=None, scale=None) -> torch.Tensor:
        """Decode: append the new tokens of ``qkv`` [B, W] at ``pos`` and attend (``ops.decode_attention``)."""
        from . import ops

        return ops.decode_attention(qkv, self.k[layer], self.v[layer], pos, self.n_head, scale=scale, rope=rope,
                                    kv_len_max=self.kv_len_max, workspace=self.workspace)


def sample(logits: torch.Tensor, temperature: float = 0.0, top_k: Optional[int] = None,
           top_p: Optional[float] = None, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """Next tokens [B] from logits [B, V]: greedy at ``temperature`` 0, else a softmax sample
    (restricted to the ``top_k`` best and/or the ``top_p`` nucleus) by the Gumbel-max trick —
    device-only ops, so it captures into a graph."""
    if temperature <= 0.0:
        return logits.argmax(-1)
    x = logits.float() / temperature
    idx = None
    if top_k is not None and 0 < top_k < x.shape[-1]:
        x, idx = torch.topk(x, top_k, dim=-1)
    if top_p is not None and 0.0 < top_p < 1.0:
        xs, order = torch.sort(x, dim=-1, descending=True)
        cum = torch.softmax(xs, -1).cumsum(-1)
        drop = (cum - torch.softmax(xs, -1)) >= top_p  # keep the smallest prefix reaching top_p
        xs = xs.masked_fill(drop, float("-inf"))
        x = torch.empty_like(x).scatter_(-1, order, xs)
    u = torch.rand(x.shape, device=x.device, generator=generator).clamp_(1e-20, 1.0)
    choice = (x - torch.log(-torch.log(u))).argmax(-1)
    return choice if idx is None else idx.gather(-1, choice[:, None]).squeeze(-1)


class _DecodeLoop:
    """One decode step (model step + sampling + bookkeeping) on static buffers; eager or graphed."""

    def __init__(self, model, cache: KVCache, tok, pos, out, done, eos: Optional[int], sampling: dict):
        self.model, self.cache = model, cache
        self.tok, self.pos, self.out, self.done, self.eos = tok, pos, out, done, eos
        self.sampling = sampling
        self.graph = None

    def step(self):
        logits = self.model.decode_step(self.tok, self.pos, self.cache)
        if (self.sampling["temperature"] <= 0.0 and logits.is_cuda and logits.dtype == torch.bfloat16
                and logits.stride(-1) == 1 and self.out.dtype == torch.int64):
            # greedy: arg-max, eos bookkeeping, position and output update in one HIP kernel
            from .ops._lib import _require

            _require()
            torch.ops.nbd.greedy_advance(logits, self.tok, self.pos, self.out,
                                         self.done if self.eos is not None else None,
                                         -1 if self.eos is None else int(self.eos))
            return
        nxt = sample(logits, **self.sampling)
        if self.eos is not None:
            nxt = torch.where(self.done, torch.full_like(nxt, self.eos), nxt)
            self.done |= nxt == self.eos
        self.tok.copy_(nxt)
        self.pos += 1
        self.out.scatter_(1, self.pos.view(-1, 1), nxt.view(-1, 1))

    def capture(self, warmup: int = 2):
        """Warm up ``warmup`` real steps on a side stream, restore the state, capture one step.
        The caller bounds ``warmup`` by the number of decode steps it will run, so the warm-up's
        position advances stay inside ``out`` and the cache (every step scatters at pos + 1)."""
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        saved = [t.clone() for t in (self.tok, self.pos, self.out, self.done)]
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self.step()
        torch.cuda.current_stream().wait_stream(side)
        for t, s in zip((self.tok, self.pos, self.out, self.done), saved):
            t.copy_(s)
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: tensor-parallel decode steps hold RCCL all-reduces, and ProcessGroupNCCL's
        # watchdog thread keeps querying its events during capture
        from .graphs import _capture

        _capture(self.graph, self.step)  # (a failed capture leaves the stream and RNG usable)
        # capture does not execute: the state is still the pre-capture one

    def __call__(self):
        if self.graph is not None:
            self.graph.replay()
        else:
            self.step()


@torch.no_grad()
def generate(model, input_ids: torch.Tensor, max_new_tokens: int, *, lengths: Optional[torch.Tensor] = None,
             temperature: float = 0.0, top_k: Optional[int] = None, top_p: Optional[float] = None,
             eos_token_id: Optional[int] = None, pad_token_id: int = 0, graph: Optional[bool] = None,
             t_max: Optional[int] = None, sync_every: int = 32, generator: Optional[torch.Generator] = None,
             return_cache: bool = False):
    """Continue each prompt of ``input_ids`` [B, T0] (right-padded; ``lengths`` [B] = prompt
    lengths, default T0) by ``max_new_tokens`` tokens.  Returns [B, T0 + max_new_tokens]: row b
    holds its prompt, then its new tokens from position lengths[b] on, then ``pad_token_id``.

    ``temperature`` 0 = greedy; ``top_k`` / ``top_p`` restrict sampling.  ``graph`` (default: on
    for a GPU model without an explicit ``generator``) captures the decode step into a HIP graph.
    """
    device = input_ids.device
    B, T0 = input_ids.shape
    if max_new_tokens <= 0:
        return input_ids.clone()
    lens = (torch.full((B,), T0, dtype=torch.int64, device=device) if lengths is None
            else lengths.to(device=device, dtype=torch.int64))
    max_len = int(lens.max())  # one host sync, before any decoding
    if int(lens.min()) < 1:
        raise ValueError("generate: every prompt needs at least one token")
    t_pad = model.prefill_length(T0)
    need = max(t_pad, max_len + max_new_tokens)
    t_max = t_max or need
    limit = model.max_positions()
    if t_max < need or (limit is not None and need > limit):
        raise ValueError(f"generate: needs {need} positions (t_max {t_max}, model limit {limit})")
    window = getattr(getattr(model, "config", None), "sliding_window", None)
    if window is not None and max_len + max_new_tokens > window:
        # the decode kernel attends over every cached position: past the window its logits would
        # silently differ from a sliding-window model's (the training forward refuses T > window too)
        raise NotImplementedError(f"generate: {max_len + max_new_tokens} positions exceed the model's "
                                  f"sliding window ({window}); sliding-window decoding is not implemented")
    cache = KVCache.for_model(model, B, t_max, device=device)
    ids = input_ids
    if t_pad > T0:
        ids = torch.cat([ids, torch.full((B, t_pad - T0), pad_token_id, dtype=ids.dtype, device=device)], 1)
    sampling = dict(temperature=temperature, top_k=top_k, top_p=top_p, generator=generator)
    logits = model.prefill(ids, cache, lens)
    tok = sample(logits, **sampling)
    out = torch.full((B, T0 + max_new_tokens), pad_token_id, dtype=input_ids.dtype, device=device)
    out[:, :T0] = input_ids
    ar = torch.arange(T0, device=device)
    out[:, :T0].masked_fill_(ar[None, :] >= lens[:, None], pad_token_id)
    pos = lens.clone()  # position of `tok`
    out.scatter_(1, pos.view(-1, 1), tok.view(-1, 1))
    done = (tok == eos_token_id) if eos_token_id is not None else torch.zeros(B, dtype=torch.bool, device=device)
    if graph is None:
        graph = device.type == "cuda" and generator is None
    loop = _DecodeLoop(model, cache, tok, pos, out, done, eos_token_id, sampling)
    n = max_new_tokens - 1
    if graph and n > 0:
        loop.capture(warmup=min(2, n))
    try:
        for i in range(n):
            if not graph:
                cache.kv_len_max = max_len + i + 1  # known on the host: fewer idle workgroups
            loop()
            if eos_token_id is not None and (i + 1) % sync_every == 0 and bool(done.all()):
                break
    finally:
        cache.kv_len_max = None  # the bound only held inside this call (a returned cache is reused later)
    return (out, cache) if return_cache else out


__all__ = ["KVCache", "generate", "sample"]
