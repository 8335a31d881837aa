"""Padding-mask preparation for the fused sequence-classification path (K15, ``csrc/kernels/mask.hip``).

HF's ``LlamaForSequenceClassification`` takes ``attention_mask`` and masks padded keys in every
layer (``00_accelerate.ipynb:1089`` trains with ``model(**batch)``).  The fused decoder runs causal
flash attention without a key mask — exact for right padding.  :func:`seqcls_prep` rotates each
left-padded row into a right-padded one (RoPE attention depends on position differences only, so
real tokens see exactly what HF computes) and re-indexes the pooled token; one launch per batch.
"""
from __future__ import annotations

from ._lib import _require


def seqcls_prep(input_ids, attention_mask, pad_token_id, bad=None):
    """(ids for the fused stack [B, T], pooled position in it [B] int64).  ``bad`` (int32 [1] on
    the ids' device) gets 1 OR-ed in when a row's mask is not one contiguous run (a mask with
    holes: no rotation makes it exact) and 2 when a row is not right-padded — read lazily by the
    caller, never synchronised here."""
    import torch

    has_pad = pad_token_id is not None
    pad = int(pad_token_id) if has_pad else 0
    if input_ids.is_cuda:
        _require()
        if bad is None:
            bad = torch.zeros(1, dtype=torch.int32, device=input_ids.device)
        ids = input_ids if input_ids.dtype == torch.int64 and input_ids.is_contiguous() else \
            input_ids.to(torch.int64).contiguous()
        return torch.ops.nbd.seqcls_prep(ids, attention_mask, pad, has_pad, bad)
    return _ref_seqcls_prep(input_ids, attention_mask, pad_token_id, bad)


def _ref_seqcls_prep(input_ids, attention_mask, pad_token_id, bad=None):
    """PyTorch reference (CPU; the GPU tests compare the kernel against it)."""
    import torch

    B, T = input_ids.shape
    ar = torch.arange(T, device=input_ids.device)
    if attention_mask is None:
        off = torch.zeros(B, dtype=torch.int64, device=input_ids.device)
    else:
        m = attention_mask != 0
        cnt = m.sum(-1)
        first = torch.where(m, ar, T).min(-1).values
        last = torch.where(m, ar, -1).max(-1).values
        off = torch.where(cnt == 0, 0, first)
        if bad is not None:
            holes = ((cnt != 0) & (last - first + 1 != cnt)).any()
            left = ((cnt != 0) & (first != 0)).any()
            bad |= (holes.to(bad.dtype) | left.to(bad.dtype) * 2).view(1)
    src = (ar[None, :] + off[:, None]) % T
    ids = input_ids.gather(1, src)
    nonpad = input_ids != pad_token_id if pad_token_id is not None else torch.ones_like(input_ids, dtype=torch.bool)
    lastnp = (ar * nonpad).argmax(-1)
    return ids, (lastnp - off) % T
