"""Embedding with a counting-sort weight gradient (K10): graph-safe, padding-robust."""
from __future__ import annotations

import os

from ._lib import _require

# NBD_FUSED_EMBED=0: token and position lookups as two gathers + an add (A/B)
FUSED_EMBED = os.environ.get("NBD_FUSED_EMBED", "1") != "0"
# out-of-range token ids: the fused lookup kernel raises a device-side flag; it is read back
# asynchronously every CHECK_EVERY calls (never a sync on the hot path) and raised at the next call
CHECK_EVERY = max(1, int(os.environ.get("NBD_EMBED_CHECK_EVERY", "8")))
_ERR: dict = {}


def _err_state(device):
    import torch

    st = _ERR.get(device.index)
    if st is None:
        st = _ERR[device.index] = {"flag": torch.zeros(1, dtype=torch.int32, device=device),
                                   "host": torch.zeros(1, dtype=torch.int32).pin_memory(), "event": None, "n": 0}
    return st


def _raise_ids(st) -> None:
    st["flag"].zero_()
    st["host"][0] = 0
    raise IndexError("embedding: a token id outside [0, vocab) was looked up (F.embedding would raise); "
                     "detected by the fused HIP lookup's error flag (read back lazily, ops/embedding.py)")


def _poll_ids(device) -> "torch.Tensor":  # noqa: F821
    """The error flag for this call's launch; raises if an earlier launch saw a bad id."""
    import torch

    st = _err_state(device)
    if torch.cuda.is_current_stream_capturing():
        return st["flag"]  # replays set it too; read at the next eager call or check_ids()
    ev = st["event"]
    if ev is not None and ev.query():
        st["event"] = None
        if int(st["host"][0]):
            _raise_ids(st)
    st["n"] += 1
    if st["event"] is None and st["n"] % CHECK_EVERY == 0:
        st["host"].copy_(st["flag"], non_blocking=True)
        st["event"] = torch.cuda.Event()
        st["event"].record()
    return st["flag"]


def check_ids(device=None) -> None:
    """Synchronously check the out-of-range-id flag of ``embedding_tok_pos`` (raises IndexError)."""
    import torch

    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    st = _ERR.get(dev.index)
    if st is not None and int(st["flag"].item()):
        _raise_ids(st)


_EmbFn = None
# the token embedding's gradient written into its DDP bucket slice (NBD_EMB_BUCKET=0: a dense
# gradient tensor, copied into the bucket by DDP — A/B)
_EMB_BUCKET = os.environ.get("NBD_EMB_BUCKET", "1") != "0"

def _emb_fn():
    global _EmbFn
    if _EmbFn is None:
        import torch

        class _Embedding(torch.autograd.Function):
            @staticmethod
            def forward(ctx, idx, weight):
                ctx.save_for_backward(idx)
                ctx.V = weight.shape[0]
                # (the parameter itself, for its DDP bucket slice: a plain reference, never read)
                ctx.weight = weight if isinstance(weight, torch.nn.Parameter) else None
                return torch.nn.functional.embedding(idx, weight)

            @staticmethod
            def backward(ctx, dy):
                from . import graddst

                (idx,) = ctx.saved_tensors
                C = dy.shape[-1]
                dy2 = dy.reshape(-1, C)
                dy2 = dy2 if dy2.is_contiguous() else dy2.contiguous()
                ids = idx.reshape(-1).contiguous()
                w = ctx.weight
                if w is not None and dy2.dtype == w.dtype and _EMB_BUCKET:
                    # straight into the DDP bucket slice (no dense gradient + flatten copy: 56 MB
                    # each way for SmolLM2's table); a tied head that already wrote the slice in
                    # this pass gets the token rows added
                    dst = graddst.join(w)
                    if dst is not None:
                        torch.ops.nbd.embedding_bwd(dy2, ids, ctx.V, dst, True)
                        return None, None
                    dst, acc = graddst.claim(w)
                    if dst is not None:
                        torch.ops.nbd.embedding_bwd(dy2, ids, ctx.V, dst, acc)
                        return None, graddst.hand_back(w, dst, acc)
                return None, torch.ops.nbd.embedding_bwd(dy2, ids, ctx.V)

        _EmbFn = _Embedding
    return _EmbFn

_TokPosFn = None


def _tokpos_fn():
    global _TokPosFn
    if _TokPosFn is None:
        import torch

        class _TokPos(torch.autograd.Function):
            @staticmethod
            def forward(ctx, idx, wte, pos, wpe, vocab):
                ctx.save_for_backward(idx, pos, wte)
                # (the parameter itself, for its DDP bucket slice; a plain reference, not a saved
                # tensor: its value is never read)
                ctx.wpe = wpe if isinstance(wpe, torch.nn.Parameter) else None
                V = vocab if 0 < vocab < wte.shape[0] else wte.shape[0]
                ctx.shapes = (V, wpe.shape[0])
                return torch.ops.nbd.embedding_tokpos(idx, wte, pos, wpe, V, _poll_ids(wte.device))

            @staticmethod
            def backward(ctx, dy):
                from . import graddst

                idx, pos, wte = ctx.saved_tensors
                V, P = ctx.shapes
                C = dy.shape[-1]
                dy2 = dy.reshape(-1, C)
                dy2 = dy2 if dy2.is_contiguous() else dy2.contiguous()
                d_wte = None
                if ctx.needs_input_grad[1]:
                    ids = idx.reshape(-1)
                    dst = graddst.join(wte)
                    if dst is not None:
                        # the tied LM head already wrote this step's gradient into the DDP bucket
                        # slice: add the rows the tokens hit and contribute nothing else
                        torch.ops.nbd.embedding_bwd(dy2, ids, V, dst, True)
                    else:
                        dst, acc = graddst.claim(wte)
                        if dst is not None:
                            torch.ops.nbd.embedding_bwd(dy2, ids, V, dst, acc)
                            d_wte = graddst.hand_back(wte, dst, acc)
                        elif V < wte.shape[0]:  # padded table: the pad rows get zeros
                            d_wte = torch.empty_like(wte)
                            torch.ops.nbd.embedding_bwd(dy2, ids, V, d_wte, False)
                        else:
                            d_wte = torch.ops.nbd.embedding_bwd(dy2, ids, V)
                d_wpe = None
                if ctx.needs_input_grad[3]:
                    # positions repeat every T rows: the batch summed per position in fp32 and
                    # placed at its (unique) row — one launch, straight into the DDP bucket slice
                    # when DDP registered one (graddst.py)
                    wpe = ctx.wpe
                    dst, acc = graddst.claim(wpe) if wpe is not None else (None, False)
                    if dst is not None and (dst.dtype != dy2.dtype or tuple(dst.shape) != (P, C)):
                        dst = dst.view(P, C) if dst.numel() == P * C and dst.dtype == dy2.dtype else None
                        if dst is None:  # (a slice this op cannot write: return the gradient instead)
                            raise RuntimeError("embedding_pos_bwd: unexpected DDP gradient slice for the position table")
                    if dst is not None:
                        torch.ops.nbd.embedding_pos_bwd(dy2, pos, P, dst, acc)
                        d_wpe = graddst.hand_back(wpe, dst, acc)
                    else:
                        d_wpe = torch.ops.nbd.embedding_pos_bwd(dy2, pos, P)
                return None, d_wte, None, d_wpe, None

        _TokPosFn = _TokPos
    return _TokPosFn


def embedding_tok_pos(idx, wte, pos, wpe, vocab: int = -1):
    """``F.embedding(idx, wte) + F.embedding(pos, wpe)`` (GPT-2's input: token + learned position
    embeddings, ``idx`` [..., T], ``pos`` [T] of unique positions) in one HIP pass on the GPU; the
    backward sums the batch for the position table and uses the counting-sort kernels for the
    token table.  ``vocab`` < ``wte.shape[0]``: rows past it are padding (ids must be < vocab).
    Out-of-range ids raise IndexError — lazily (a device flag read back without syncing, see
    ``check_ids``), where F.embedding raises at once."""
    import torch

    C = wte.shape[-1]
    if (FUSED_EMBED and wte.is_cuda and idx.dtype == torch.int64 and pos.dtype == torch.int64 and C % 8 == 0 and C <= 4096
            and wte.dtype == wpe.dtype and wte.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and idx.shape[-1] == pos.numel() and pos.dim() == 1):
        _require()
        return _tokpos_fn().apply(idx.contiguous(), wte, pos.contiguous(), wpe, int(vocab))
    if 0 < vocab < wte.shape[0]:
        if not idx.is_cuda and idx.numel() and int(idx.max()) >= vocab:
            raise IndexError(f"embedding: token id {int(idx.max())} >= vocab {vocab}")
    return embedding(idx, wte) + embedding(pos, wpe)


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
