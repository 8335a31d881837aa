"""Fused large-vocabulary softmax cross-entropy (K6)."""
from __future__ import annotations

import os

from ._lib import _require

# GPT-2's return_logits=False path through linear_cross_entropy (A/B switch: NBD_FUSED_XENT=0)
FUSED_XENT = os.environ.get("NBD_FUSED_XENT", "1") != "0"


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
            dlogits = logits if ctx.inplace else torch.empty_strided(logits.shape, logits.stride(), dtype=logits.dtype,
                                                                             device=logits.device)
            torch.ops.nbd.xent_bwd(logits, target, lse, scale, ctx.ignore_index, dlogits)
            return dlogits, None, None, None, None

    class _LinearCrossEntropy(torch.autograd.Function):
        """loss(h·Wᵀ, target) with the loss forward and backward in ONE pass over the logits
        (``nbd::xent_fused``: the row stays in registers between the logsumexp and the in-place
        gradient write).  grad_out is applied to the two small GEMM operands in backward, never to
        the [N, V] gradient."""

        @staticmethod
        def forward(ctx, h2, w, target, ignore_index, reduction, vocab, fuse_dgrad):
            # vocabulary padded to a multiple of VOCAB_ALIGN for the three GEMMs (hipBLASLt: GPT-2's
            # 50257 -> 50304 takes the LM head from 2.18 to 1.75 ms per step, profiles/lmhead_r2.txt):
            # zero weight rows give exactly-zero pad logits, the loss reads only the first V columns
            # (row stride Vp), so the pad columns stay 0 as gradients and dW's pad rows are 0.
            # A model whose table is already padded (GPT2: rows [vocab, Vp) kept at zero) passes
            # `vocab` < w.shape[0] and nothing is copied; otherwise the padded copy is made here.
            V = vocab if vocab > 0 else w.shape[0]
            if V < w.shape[0]:
                Vp = w.shape[0]
            else:
                Vp = -(-V // VOCAB_ALIGN) * VOCAB_ALIGN if V >= VOCAB_PAD_MIN else V
            if Vp != w.shape[0]:
                wp = torch.empty(Vp, w.shape[1], dtype=w.dtype, device=w.device)
                wp[:V].copy_(w)
                wp[V:].zero_()
            else:
                wp = w
                # the table is cold here (the step's activations evicted it since the last
                # step): the last HIP GEMM launch before this one warms it into the MALL
                # (csrc/kernels/gemm.hip "next-weight warm-up"; docs/FINDINGS.md §23)
                if LM_HEAD_WARM_BYTES > 0 and wp.is_cuda and hasattr(torch.ops.nbd, "gemm_warm_hint"):
                    torch.ops.nbd.gemm_warm_hint(wp, False, LM_HEAD_WARM_BYTES)
            if reduction == "mean":  # 1 / #(non-ignored rows), one launch (inf -> nan loss if none)
                scale = torch.ops.nbd.xent_mean_scale(target, ignore_index)
            else:
                scale = torch.ones(1, dtype=torch.float32, device=h2.device)
            N = h2.shape[0]
            chunk = LM_HEAD_CHUNK if 0 < LM_HEAD_CHUNK < N else N
            dh = None
            plan = head_plan(h2, wp)
            if any(plan.values()):
                chunk = N  # (row chunks are a hipBLASLt experiment)
            if chunk == N:
                logits_p = _hip_logits(h2, wp) if plan["fwd"] else torch.mm(h2, wp.t())
                loss_rows, _ = torch.ops.nbd.xent_fused(logits_p[:, :V] if Vp != V else logits_p, target,
                                                        ignore_index, scale)
            else:
                # row chunks: each chunk's logits are written by its GEMM, turned into dlogits in
                # place by xent_fused and (fuse_dgrad) read by the input-gradient GEMM while they
                # are still in the MALL, instead of three HBM round trips of the whole [N, Vp]
                logits_p = torch.empty(N, Vp, dtype=h2.dtype, device=h2.device)
                loss_rows = torch.empty(N, dtype=torch.float32, device=h2.device)
                if fuse_dgrad:
                    dh = torch.empty_like(h2)
                for r0 in range(0, N, chunk):
                    r1 = min(N, r0 + chunk)
                    lc = logits_p[r0:r1]
                    torch.mm(h2[r0:r1], wp.t(), out=lc)
                    lr, _ = torch.ops.nbd.xent_fused(lc[:, :V] if Vp != V else lc, target[r0:r1], ignore_index,
                                                     scale)
                    loss_rows[r0:r1] = lr
                    if dh is not None:
                        torch.mm(lc, wp, out=dh[r0:r1])
            # logits now hold d(loss)/d(logits) for grad_out = 1 (and dh = dlogits·W, if fused)
            ctx.save_for_backward(h2, wp, logits_p, w, dh)
            ctx.plan = plan
            ctx.rows = w.shape[0]
            ctx.copied = wp is not w
            return torch.ops.nbd.xent_loss_total(loss_rows, scale)  # Σ rows · scale, one launch

        @staticmethod
        def backward(ctx, grad):
            from . import graddst

            h2, wp, dlogits, w, dh_fused = ctx.saved_tensors
            need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
            dh = hg = None
            if need_h:
                dh = dh_fused if dh_fused is not None else (
                    _hip_dgrad(dlogits, wp) if ctx.plan["dgrad"] else torch.mm(dlogits, wp))
            # the incoming gradient (1 after loss.backward()) scales dh and the weight gradient's
            # operand: one launch for both (dh in place, hg = h2·g), by the fp32 scalar as it arrives
            if need_h and need_w and dh.is_contiguous() and dh.numel() % 8 == 0 and h2.numel() % 8 == 0:
                hg = torch.ops.nbd.scale_pair_(dh, h2, grad.float().reshape(1))
            else:
                g = grad.to(h2.dtype)
                if need_h:
                    dh = dh.mul_(g)
                if need_w:
                    hg = h2 * g
            dw = None
            if need_w:
                dst, acc = graddst.claim(w) if not ctx.copied else (None, False)
                if dst is not None:  # straight into the DDP bucket slice (graddst.py)
                    if ctx.plan["wgrad"]:
                        _hip_wgrad(dlogits, hg, out=dst, accum=acc)
                    elif acc:
                        dst.addmm_(dlogits.t(), hg)
                    else:
                        torch.mm(dlogits.t(), hg, out=dst)
                    dw = graddst.hand_back(w, dst, acc)
                else:
                    dw = (_hip_wgrad(dlogits, hg) if ctx.plan["wgrad"] else torch.mm(dlogits.t(), hg))[:ctx.rows]
            return dh, dw, None, None, None, None, None

    _XentFn = (_FusedCrossEntropy, _LinearCrossEntropy)
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
    return _xent_fn()[0].apply(logits, target.contiguous().long(), int(ignore_index), reduction, bool(inplace_backward))


FUSED_MAX_VOCAB = 256 * 8 * 32  # xent_fused keeps a row in registers: 256 lanes x 32 chunks x 8
# LM-head GEMMs run on a vocabulary padded to this multiple (only from VOCAB_PAD_MIN up: the
# [V, C] weight copy costs one pass over it); the padded width must stay <= FUSED_MAX_VOCAB + 14
VOCAB_ALIGN = max(1, int(os.environ.get("NBD_VOCAB_ALIGN", "128")))  # 1 = no padding (A/B)
VOCAB_PAD_MIN = 4096
# how much of the LM-head table the HIP GEMM launch before the head warms into the MALL
# (opt-in, NBD_LM_HEAD_WARM_MB=96: measured no faster on the GPT-2 step,
# profiles/lmhead_warm_ab_r3.txt — hipBLASLt's head is not first-touch bound the way the
# short-K HIP GEMMs are)
LM_HEAD_WARM_BYTES = int(float(os.environ.get("NBD_LM_HEAD_WARM_MB", "0")) * (1 << 20))
# rows per LM-head chunk (0 = one [N, Vp] GEMM): GEMM -> in-place loss gradient -> input-gradient
# GEMM per chunk, so a chunk's logits are re-read from the 256 MB MALL rather than from HBM
LM_HEAD_CHUNK = int(os.environ.get("NBD_LMHEAD_CHUNK", "0"))
# The head's three products on the hand-written MFMA kernels (NBD_LMHEAD_HIP=0: hipBLASLt) — the
# 256x256 phase-interleaved kernel (gemm256.hip) wherever tokens, padded vocabulary and width are
# multiples of 256 (GPT2 then pads its table to a multiple of 512, so the input gradient splits 8
# ways along the vocabulary: 3 whole rounds of 256 workgroups), else the 128x128 8-wave kernel;
# the weight gradient is accumulated straight into a DDP bucket slice when one is claimed.  On the
# GPT-2 small step within 0.7-1.2 % of the library head (docs/FINDINGS.md §33), with no library
# GEMM left in the step.
LM_HEAD_HIP = os.environ.get("NBD_LMHEAD_HIP", "auto") != "0"
# Which of the three products run hand-written when LM_HEAD_HIP is on.  NBD_LMHEAD_HIP=1: all
# three; "auto" (default): the plan the GPT-2 small step measured fastest (interleaved A/B of every
# plan in the graphed step, one box: profiles/lmhead_plan_ab_r6a.txt, lmhead_plan_ab_r6b.txt) — the
# weight gradient on the 256x256 kernel (whole rounds + a token-split tail: 10.36-10.40 ms, tied
# with all-hipBLASLt 10.36-10.39), the forward and input gradient on hipBLASLt (hand-written: +0.10
# and +0.15 ms in the step, though the isolated kernels swap places from box to box:
# profiles/lmhead_products_r6.txt); or a list such as "fwd+wgrad".
_HEAD_SPEC = os.environ.get("NBD_LMHEAD_HIP", "auto")
HEAD_PRODUCTS = ({"fwd": False, "dgrad": False, "wgrad": True} if _HEAD_SPEC == "auto" else
                 {p: _HEAD_SPEC not in ("0",) and (_HEAD_SPEC == "1" or p in _HEAD_SPEC.replace("+", ",").split(","))
                  for p in ("fwd", "dgrad", "wgrad")})


def table_pad() -> int:
    """Row padding of an LM-head table for this process's plan: 512 when the input gradient is
    hand-written (split 8 ways into whole K-tiles), 256 when the forward or the weight gradient is
    (256x256 tiles over the vocabulary), else 128 (hipBLASLt's alignment)."""
    if not LM_HEAD_HIP:
        return 128
    if HEAD_PRODUCTS.get("dgrad"):
        return 512
    return 256 if HEAD_PRODUCTS.get("fwd") or HEAD_PRODUCTS.get("wgrad") else 128


def _use_hip(product: str) -> bool:
    return LM_HEAD_HIP and HEAD_PRODUCTS.get(product, False)
# the 256x256 kernel (for the forward with non-temporal C stores, variant 6: the 823 MB of GPT-2
# logits outgrow every cache on their way out — 660 -> 611 us isolated; the weight gradient, a
# 77 MB output, measured 643 vs 651 us with them: plain stores), the 128x128 8-wave kernel
_T256_NT, _T256, _T128 = 88256256, 86256256, 82128128


def _hip_ok(h2, wp) -> bool:
    import torch

    N, C = h2.shape
    return (LM_HEAD_HIP and h2.is_cuda and h2.dtype == torch.bfloat16 and wp.dtype == torch.bfloat16
            and N % 128 == 0 and wp.shape[0] % 128 == 0 and C % 128 == 0)


def head_plan(h2, wp) -> dict:
    """{fwd, dgrad, wgrad}: True where that product of the head runs hand-written."""
    ok = _hip_ok(h2, wp)
    return {p: ok and _use_hip(p) for p in ("fwd", "dgrad", "wgrad")}


def _big(*dims) -> bool:
    return all(d % 256 == 0 for d in dims)


def _hip_logits(h2, wp):
    """logits [N, Vp] = h2·wpᵀ on the hand-written kernels."""
    import torch

    N, Vp = h2.shape[0], wp.shape[0]
    out = torch.empty(N, Vp, dtype=h2.dtype, device=h2.device)
    torch.ops.nbd.gemm(h2, wp, out, False, False, None, 0, None, None, 1, _T256_NT if _big(N, Vp) else _T128)
    return out


def _hip_dgrad(dlogits, wp):
    """dh [N, C] = dlogits·wp (wp read as [K = Vp][C]), split along the vocabulary: the most splits
    up to 8 that divide it into whole K-tiles (N·C/256² tiles x splits workgroups)."""
    import torch

    N, (Vp, C) = dlogits.shape[0], wp.shape
    steps = Vp // 64
    S = next(s for s in (8, 6, 4, 3, 2, 1) if steps % s == 0)
    dh = torch.empty(N, C, dtype=dlogits.dtype, device=dlogits.device)
    torch.ops.nbd.gemm(dlogits, wp, dh, False, True, None, 0, None, None, S, _T256 if _big(N, C) else _T128)
    return dh


_CUS = []


def _cus(dev) -> int:
    if not _CUS:
        import torch

        _CUS.append(int(torch.cuda.get_device_properties(dev).multi_processor_count))
    return _CUS[0]


def _hip_wgrad(dlogits, hg, out=None, accum=False):
    """dW [Vp, C] = dlogitsᵀ·hg (both read as [K = tokens][...]) into ``out`` (+= with accum: the
    128x128 kernel, the one with an accumulating epilogue).  On the 256x256 kernel the vocabulary
    rows are cut in two launches so that no round of one-workgroup-per-CU tiles runs part-empty:
    whole rounds unsplit, the remaining tile rows split along the tokens to fill one more round
    (GPT-2: 594 tiles = 2.3 rounds of 256 CUs -> 510 tiles + 84 tiles x 2 splits; a single
    launch pays a third, 30 %-full round)."""
    import torch

    Vp, C = dlogits.shape[1], hg.shape[1]
    if out is None:
        out = torch.empty(Vp, C, dtype=hg.dtype, device=hg.device)
    if accum or not _big(Vp, C):
        torch.ops.nbd.gemm(dlogits, hg, out, True, True, None, 0, None, None, 1, _T128, 1 if accum else 0)
        return out
    cus, tn, rows = _cus(hg.device), C // 256, Vp // 256
    r1 = min(rows, (rows * tn // cus) * cus // tn)  # tile rows in whole rounds
    r2 = rows - r1
    S = 1
    while r2 and r2 * tn * S * 2 <= cus and (dlogits.shape[0] // 64) % (S * 2) == 0:
        S *= 2
    if r1 == 0 or r2 == 0 or S == 1:
        torch.ops.nbd.gemm(dlogits, hg, out, True, True, None, 0, None, None, 1, _T256, 0)
        return out
    c1 = r1 * 256
    torch.ops.nbd.gemm(dlogits[:, :c1], hg, out[:c1], True, True, None, 0, None, None, 1, _T256, 0)
    torch.ops.nbd.gemm(dlogits[:, c1:], hg, out[c1:], True, True, None, 0, None, None, S, _T256, 0)
    return out


def linear_cross_entropy(h, weight, target, ignore_index: int = -100, reduction: str = "mean", vocab: int = -1):
    """``cross_entropy(h @ weight.T, target)`` for an LM head (``h`` [..., C], ``weight`` [V, C]) —
    the loss's forward and backward fused into one pass over the logits on the GPU path (bf16/fp16,
    V ≤ 65,536: one read and one in-place write of the [N, V] logits instead of two reads and a
    write), the GEMMs on the hand-written MFMA kernels (``NBD_LMHEAD_HIP=0``: hipBLASLt).  The
    logits are not returned.  ``vocab`` < ``weight.shape[0]``:
    the table's rows past ``vocab`` are zero padding (GPT2 keeps its tied table padded to a
    multiple of 512; 128 with the library head) — the loss covers the first ``vocab`` classes
    only."""
    import torch
    import torch.nn.functional as F

    if reduction not in ("mean", "sum"):
        raise ValueError("linear_cross_entropy: reduction must be 'mean' or 'sum'")
    h2 = h.reshape(-1, h.shape[-1])
    tgt = target.reshape(-1)
    V = vocab if 0 < vocab < weight.shape[0] else weight.shape[0]
    if not (h.is_cuda and h.dtype in (torch.bfloat16, torch.float16) and weight.dtype == h.dtype
            and weight.shape[0] <= FUSED_MAX_VOCAB and not torch.is_autocast_enabled()):
        logits = F.linear(h2, weight)
        if V < weight.shape[0]:
            logits = logits[:, :V]
        return F.cross_entropy(logits.float(), tgt, ignore_index=ignore_index, reduction=reduction)
    _require()
    fuse_dgrad = torch.is_grad_enabled() and h.requires_grad
    return _xent_fn()[1].apply(h2 if h2.is_contiguous() else h2.contiguous(), weight, tgt.contiguous().long(),
                               int(ignore_index), reduction, int(V), fuse_dgrad)
