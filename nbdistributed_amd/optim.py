"""Flat-buffer optimizers for ``parallel.DistributedDataParallel(flat_params=True)``.

``FlatAdamW`` keeps fp32 master weights and moments in the DDP bucket layout and performs each
bucket's update with one fused HIP kernel (``nbd::adamw_flat``) that reads the all-reduced
gradient bucket directly — no unflatten, no per-parameter kernels, no fp32→bf16 weight casts in
the forward (the model runs in bf16; the master copy keeps fp32 precision).  Semantics match
``torch.optim.AdamW`` (decoupled weight decay, bias correction).

With ``DistributedDataParallel(..., shard=True)`` (ZeRO-2) the state covers only this rank's
slice of each bucket (``b.lo .. b.lo + b.shard``): the kernel reads the reduce-scattered gradient
slice, updates that slice of the bf16 parameters, and an async all-gather per bucket (waited at
the next DDP forward, or ``ddp.wait_params()``) rebuilds the full parameters on every rank.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import ops


# NBD_ADAMW_MULTI=0: one adamw_flat call per bucket (A/B of the one-call update)
_MULTI = os.environ.get("NBD_ADAMW_MULTI", "1") != "0"
# default of FlatAdamW(overlap=None): update each bucket during backward (NBD_ADAMW_OVERLAP=1)
_OVERLAP = os.environ.get("NBD_ADAMW_OVERLAP", "0") == "1"


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


class FlatAdamW(torch.optim.Optimizer):
    """A ``torch.optim.Optimizer`` (so LR schedulers and hooks work) whose state lives per DDP
    bucket: ``flat_state[i]`` = fp32 master / exp_avg / exp_avg_sq of bucket i.  One param group
    (the bucket kernels apply one lr / weight decay to the whole model)."""

    def __init__(self, ddp, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, capturable: bool = False, overlap: Optional[bool] = None):
        """``capturable=True``: the step counter and lr live in device memory (``step_t``,
        ``lr_t``) so the update can be captured in a HIP graph and replayed
        (:class:`nbdistributed_amd.graphs.GraphedStep` calls :meth:`sync_hyper` before each
        replay to push the current ``param_groups[0]['lr']``).

        ``overlap=True`` (unsharded, eager): each bucket is updated on a side stream as soon as
        its gradient is final during backward — at world size 1 when DDP finalises it, at world
        size > 1 when its all-reduce has landed (the update stream waits for the bucket's event
        on DDP's communication stream) — so the memory-bound update runs under the rest of the
        backward and the remaining collectives; ``step()`` then only completes the bookkeeping.
        It pays where the eager step is host-bound (small models: the GPU idles between
        launches), not where the GPU is busy (GPT-2 small: 1.7 % slower) and not inside a HIP
        graph (skipped there).  Call ``step()`` once after every synchronising backward (the
        update happens in that backward).  ``None``: ``NBD_ADAMW_OVERLAP=1`` turns it on."""
        if not getattr(ddp, "flat_params", False) or ddp.grad_mode != "bucket":
            raise ValueError("FlatAdamW needs DistributedDataParallel(..., flat_params=True, grad_mode='bucket')")
        super().__init__(list(ddp.params), dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.ddp = ddp
        self.step_count = 0
        self._clip_coef = None
        self.capturable = capturable
        dev = ddp.buckets[0].param_flat.device
        self.step_t = torch.zeros(1, dtype=torch.float32, device=dev) if capturable else None
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float32, device=dev) if capturable else None
        self.flat_state: List[Dict[str, torch.Tensor]] = []
        self.sharded = bool(getattr(ddp, "shard", False))
        self._multi = None  # (grads, params, masters, exp_avgs, exp_avg_sqs) of the one-call update
        if overlap is None:
            overlap = _OVERLAP
        self.overlap = bool(overlap) and not self.sharded and dev.type == "cuda"
        self._updated: List[int] = []  # buckets updated during the current backward (overlap)
        if self.overlap:
            self._opt_stream = torch.cuda.Stream(device=dev)
            ddp._on_bucket_ready = self._update_bucket
        for b in ddp.buckets:
            master = self._param_slice(b).detach().float().clone()
            self.flat_state.append({"master": master, "exp_avg": torch.zeros_like(master),
                                    "exp_avg_sq": torch.zeros_like(master)})

    def _joined_grads(self) -> bool:
        """No bucket's gradient is still waited on per bucket (``wait_grad`` would be a no-op)."""
        return getattr(self.ddp, "_joined", True) or getattr(self.ddp, "wait_grad", None) is None

    def _param_slice(self, b):
        return b.param_flat[b.lo:b.lo + b.shard] if self.sharded else b.param_flat

    def _grad(self, b):
        return b.grad_shard if self.sharded else b.buffer

    # ------------------------------------------------------------------ overlap (update in backward)
    @torch.no_grad()
    def _update_bucket(self, b) -> None:
        """DDP callback (``_on_bucket_ready``): bucket ``b``'s gradient is final — update it on the
        side stream now (inside backward; joined back at the end of backward)."""
        if _capturing():
            # not inside a HIP graph: the side-stream branches made the graphed SmolLM2 step 11 %
            # slower (profiles/adamw_overlap_ab_r3.txt); step() updates the captured step
            return
        if self._clip_coef is not None:
            raise RuntimeError("FlatAdamW(overlap=True) updates during backward: clip_grad_norm_ cannot apply")
        dev = b.param_flat.device
        cur = torch.cuda.current_stream(dev)
        if not self._updated:  # first bucket of this backward: the step's bookkeeping
            self.step_count += 1
            if self.capturable:
                self._opt_stream.wait_stream(cur)
                with torch.cuda.stream(self._opt_stream):
                    self.step_t.add_(1.0)
                    if not _capturing():
                        self.lr_t.fill_(float(self.param_groups[0]["lr"]))
            torch.autograd.Variable._execution_engine.queue_callback(self._join)
        done = getattr(b, "done", None)
        if getattr(self.ddp, "_side", False) and getattr(self.ddp, "_per_bucket_wait", False) and done is not None:
            # the bucket was finished on DDP's comm stream: its all-reduce (world > 1) and any
            # post-division have landed once this event has
            self._opt_stream.wait_event(done)
        self._opt_stream.wait_stream(cur)
        g = self.param_groups[0]
        st = self.flat_state[b.index]
        b1, b2 = g["betas"]
        with torch.cuda.stream(self._opt_stream):
            ops.adamw_flat(self._grad(b), self._param_slice(b), st["master"], st["exp_avg"], st["exp_avg_sq"], g["lr"],
                           b1, b2, g["eps"], g["weight_decay"], max(self.step_count, 1), step_t=self.step_t,
                           lr_t=self.lr_t)
        self._updated.append(b.index)

    def _join(self) -> None:
        torch.cuda.current_stream(self._opt_stream.device).wait_stream(self._opt_stream)

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if self.overlap and self._updated:
            # every bucket was updated during backward (DDP finalises each one, unused ones too)
            self._updated = []
            return loss
        g = self.param_groups[0]
        self.step_count += 1
        b1, b2 = g["betas"]
        if self.capturable:
            self.step_t.add_(1.0)
            if not _capturing():
                self.lr_t.fill_(float(g["lr"]))
        if (_MULTI and not self.sharded and self.ddp.buckets[0].param_flat.is_cuda
                and (self._joined_grads() or not getattr(self.ddp, "_collectives", False))):
            # all updates from one call.  (At world 1 there is no collective for a per-bucket wait
            # to overlap with: one join of the side stream, if any, then every bucket.)
            if not self._joined_grads():
                self.ddp.wait_grads()
            if self._multi is None:
                self._multi = ([self._grad(b) for b in self.ddp.buckets], [b.param_flat for b in self.ddp.buckets],
                               [st["master"] for st in self.flat_state], [st["exp_avg"] for st in self.flat_state],
                               [st["exp_avg_sq"] for st in self.flat_state])
            torch.ops.nbd.adamw_flat_multi(*self._multi, float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                           float(g["weight_decay"]), max(self.step_count, 1), 1.0, self._clip_coef,
                                           self.step_t, self.lr_t)
            self._clip_coef = None
            return loss
        pairs = list(zip(self.ddp.buckets, self.flat_state))
        if self.sharded:
            # a previous step's gathers still reading our slices must finish before the update
            # rewrites them (step() twice without a forward in between)
            self.ddp.wait_params()
        wait = getattr(self.ddp, "wait_grad", None)
        for b, st in pairs:  # bucket order = the order their collectives were issued
            if wait is not None:
                wait(b)
            ops.adamw_flat(self._grad(b), self._param_slice(b), st["master"], st["exp_avg"], st["exp_avg_sq"], g["lr"],
                           b1, b2, g["eps"], g["weight_decay"], max(self.step_count, 1), grad_scale_t=self._clip_coef,
                           step_t=self.step_t, lr_t=self.lr_t)
            if self.sharded and self.ddp._collectives:  # rebuild the full bucket from every rank's updated slice
                b.gather_work = dist.all_gather_into_tensor(b.param_flat, self._param_slice(b), group=self.ddp.pg,
                                                            async_op=True)
        if self.sharded and _capturing():
            self.ddp.wait_params()  # a captured step must join its collectives before it ends
        self._clip_coef = None
        return loss

    def sync_hyper(self) -> None:
        """Push the host-side lr (LR schedulers) into ``lr_t`` — call outside graph capture."""
        if self.capturable:
            self.lr_t.fill_(float(self.param_groups[0]["lr"]))

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float, eps: float = 1e-6) -> torch.Tensor:
        """``torch.nn.utils.clip_grad_norm_`` for bucket-resident gradients: the global L2 norm
        comes from the one-pass summary kernel (``ops.tensor_summary_raw``, float64 partials) over
        each averaged bucket; the clip coefficient stays on the device and is applied inside the
        next ``step()`` — no host synchronisation.  Returns the total norm (device tensor)."""
        if self.overlap:
            # the buckets were already updated during backward, unclipped: refuse loudly, and
            # leave no coefficient behind for a later step
            self._clip_coef = None
            raise RuntimeError("FlatAdamW(overlap=True) applies each bucket's update during backward, before "
                               "clip_grad_norm_ can run; construct it with overlap=False to clip gradients")
        sq = None
        if hasattr(self.ddp, "wait_grads"):
            self.ddp.wait_grads()
        for b in self.ddp.buckets:
            n = ops.tensor_summary_raw(self._grad(b))[4]
            sq = n * n if sq is None else sq + n * n
        if self.sharded:  # the slices partition the gradient: sum the squares over the ranks
            dist.all_reduce(sq, group=self.ddp.pg)
        total = sq.sqrt().float()
        self._clip_coef = torch.clamp(max_norm / (total + eps), max=1.0).reshape(1).contiguous()
        return total

    def zero_grad(self, set_to_none: bool = True) -> None:
        for p in self.ddp.params:
            p.grad = None

    def state_dict(self) -> Dict[str, Any]:
        """Per-bucket fp32 state; with a sharded DDP, this rank's slices only (``shard`` records
        rank and world: load it on the same rank of a same-size world)."""
        step = int(self.step_t.item()) if self.capturable else self.step_count
        sd = {"step": step, "param_groups": [{k: v for k, v in self.param_groups[0].items() if k != "params"}],
              "buckets": [{k: v for k, v in st.items()} for st in self.flat_state]}
        if self.sharded:
            sd["shard"] = {"rank": self.ddp.rank, "world": self.ddp.world}
        return sd

    @torch.no_grad()
    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        want = {"rank": self.ddp.rank, "world": self.ddp.world} if self.sharded else None
        if sd.get("shard") != want:
            raise ValueError(f"FlatAdamW.load_state_dict: state is for shard {sd.get('shard')}, this optimizer is {want}")
        if self.sharded:
            self.ddp.wait_params()
        self.step_count = int(sd["step"])
        if self.capturable:
            self.step_t.fill_(float(self.step_count))
        self.param_groups[0].update(sd["param_groups"][0])
        for st, src in zip(self.flat_state, sd["buckets"]):
            for k in st:
                st[k].copy_(src[k])
        for b, st in zip(self.ddp.buckets, self.flat_state):
            self._param_slice(b).copy_(st["master"].to(b.param_flat.dtype))
            if self.sharded and self.ddp._collectives:
                dist.all_gather_into_tensor(b.param_flat, self._param_slice(b), group=self.ddp.pg)


# ---------------------------------------------------------------------------------------------
# torch.optim.AdamW with torch's own per-parameter state, one HIP launch per <= 128 parameters
# (``nbd::adamw_tensors``, csrc/kernels/optim.hip) — what ``models.native()`` installs on the
# notebook's own AdamW (NBD_NATIVE_NBD_ADAMW=0 keeps torch's fused step).

_FALLBACK_KEYS = ("amsgrad", "maximize", "capturable", "differentiable")


def _fast_adamw_ok(opt) -> bool:
    """Every condition under which the HIP step computes torch's update (else torch's step
    runs): plain hyper-parameters, no step hooks, no graph capture, contiguous fp32 parameters /
    gradients all on ONE GPU (the kernel takes one device's tensor table), fused-style (device,
    fp32) step counts in any existing state.  The update then equals torch's within rounding, not
    bitwise: the kernel forms the bias corrections from the device step count in fp32 (powf),
    torch's fused AdamW in double, and the fp32 operations are ordered differently — parameters
    and moments agree to ~1e-6 relative (tests/test_gpu_swap_semantics.py)."""
    from torch.optim import optimizer as _topt

    if (getattr(opt, "_optimizer_step_pre_hooks", None) or getattr(opt, "_optimizer_step_post_hooks", None)
            or getattr(_topt, "_global_optimizer_pre_hooks", None) or getattr(_topt, "_global_optimizer_post_hooks", None)):
        return False
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return False
    dev = None
    for group in opt.param_groups:
        if any(group.get(k) for k in _FALLBACK_KEYS) or torch.is_tensor(group["lr"]):
            return False
        if any(torch.is_tensor(b) for b in group["betas"]):
            return False
        for p in group["params"]:
            g = p.grad
            if g is None:
                continue
            if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and g.dtype == torch.float32
                    and not g.is_sparse and g.is_contiguous() and g.device == p.device):
                return False
            if dev is None:
                dev = p.device
            elif p.device != dev:  # a model split across GPUs: torch's step
                return False
            st = opt.state.get(p)
            if st:
                s_ = st.get("step")
                if not (torch.is_tensor(s_) and s_.is_cuda and s_.dtype == torch.float32 and s_.numel() == 1
                        and s_.device == p.device and st["exp_avg"].device == p.device
                        and st["exp_avg"].is_contiguous() and st["exp_avg_sq"].is_contiguous()):
                    return False
    return True


def _fast_adamw_step(self, closure=None, **kwargs):
    """``torch.optim.AdamW.step`` (decoupled weight decay, bias-corrected moments, torch's state
    layout) as ``nbd::adamw_tensors`` launches; torch's own step whenever ``_fast_adamw_ok``
    says the two might differ (or extra arguments such as a GradScaler's are passed)."""
    if kwargs or not _fast_adamw_ok(self):
        return type(self).step(self, closure, **kwargs)
    loss = None
    if closure is not None:
        with torch.enable_grad():
            loss = closure()
    with torch.no_grad():
        for group in self.param_groups:
            ps, gs, ms, vs, ss = [], [], [], [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:  # as torch's fused AdamW initialises it
                    st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                ps.append(p)
                gs.append(p.grad)
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
                ss.append(st["step"])
            if not ps:
                continue
            torch._foreach_add_(ss, 1.0)
            b1, b2 = group["betas"]
            torch.ops.nbd.adamw_tensors(ps, gs, ms, vs, ss, float(group["lr"]), float(b1), float(b2),
                                        float(group["eps"]), float(group["weight_decay"]))
    return loss


def install_fast_adamw(opt) -> bool:
    """Give this ``torch.optim.AdamW`` instance the HIP step (a bound method on the instance, so
    LR schedulers and ``accelerate`` wrap it as they wrap torch's).  Returns False (nothing
    changed) for other classes or without the native library."""
    if type(opt) is not torch.optim.AdamW or not ops.native_available():
        return False
    import types

    opt.step = types.MethodType(_fast_adamw_step, opt)
    opt._nbd_fast_step = True
    return True
