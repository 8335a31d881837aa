"""Data parallelism for notebook cells: bucketed gradient all-reduce overlapped with backward.

Reference: the reference has no parallelism of its own — its notebook wraps the model with HF
accelerate, i.e. torch DDP (notebook exec 32/35: ``accelerator.prepare`` /
``accelerator.backward``).  ``DistributedDataParallel`` here is a drop-in for that pattern,
designed for MI355X + RCCL over xGMI:

* gradients are grouped into buckets in reverse registration order (≈ backward order); the
  bucket cap defaults to 64 MiB of wire bytes — large enough that each RCCL all-reduce runs in
  its bandwidth regime on a point-to-point xGMI ring (per-link bound), with a small
  first bucket (4 MiB) so communication starts early in backward;
* when the last gradient of a bucket is accumulated (``register_post_accumulate_grad_hook``),
  the bucket is launched on a dedicated HIP stream (normal priority — see __init__): one fused HIP kernel
  (``nbd::bucket_flatten``) gathers the grads into the bucket while casting to the wire dtype
  (fp32 -> bf16 halves the xGMI bytes) and pre-dividing by the world size; RCCL all-reduces the
  bucket; a second fused kernel (``nbd::bucket_unflatten``) scatters back, casting to the grads'
  dtype — all overlapped with the rest of backward on the compute stream;
* buckets are launched strictly in bucket order on every rank (a bucket that becomes ready early
  waits for its predecessors), so ranks always issue the same collective sequence;
* parameters that got no gradient this step (unused branches) are flattened as zeros at the end
  of backward so no rank ever waits on a missing bucket;
* ``no_sync()`` for gradient accumulation, buffers broadcast from rank 0 in forward, parameters
  broadcast from rank 0 at construction (coalesced through the same flatten kernel);
* ``shard=True`` (ZeRO stage 2, with ``flat_params`` + ``grad_mode="bucket"`` and
  ``nbdistributed_amd.optim.FlatAdamW``): each bucket is REDUCE-SCATTERED instead of all-reduced —
  rank r keeps only the averaged gradient of its 1/world slice (``b.grad_shard``), the fp32
  master weights and moments exist only for that slice (optimizer memory / world), the update
  runs on 1/world of the parameters, and the updated bf16 slices are ALL-GATHERED back into the
  parameter buckets, one async gather per bucket right after its update (so they overlap the
  remaining bucket updates), all waited device-side at the next forward.  Same bytes on the
  wire as the all-reduce (RCCL's ring all-reduce IS a reduce-scatter + all-gather), 1/world of
  the optimizer work and state.

Gradients as bucket views (``grad_views``, on by default on the GPU when a bucket's dtype is its
parameters' dtype): every parameter's bucket slice is registered as its gradient's home
(``ops.graddst``).  The framework's backward nodes — the C++ Linear / MLP nodes (weight and bias
gradients out of the GEMM epilogues, ``csrc/kernels/autograd.hip``), the LM head and the tied
token embedding — write straight into it, and ``p.grad`` *is* the slice: no flatten copy before
the all-reduce (which then averages with ``ReduceOp.AVG``) and no unflatten after it.  Plain
``nn.Linear`` layers of the wrapped module are routed through the same C++ node
(``fused_linear``).  Under ``no_sync()`` micro-batches accumulate in place: the GEMMs add into
the slice in their epilogue (beta = 1) and the remaining gradients are pre-reduced into the
bucket by K3 (``ops.prereduce_into_bucket``, fp32 accumulate) — no per-parameter autograd adds,
and the last micro-batch's bucket is the whole local gradient.

Also provides DDP communication hooks for stock ``torch.nn.parallel.DistributedDataParallel``
(``bf16_compress_hook``) built on the same fused kernels.
"""
from __future__ import annotations

import contextlib
import os
import types
import weakref
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch
import torch.distributed as dist

from .. import ops

# NBD_FAULT_DDP_GRAD_SCALE (tests only): rank 0 scales each bucket by this before its collective
_FAULT_GRAD_SCALE = float(os.environ.get("NBD_FAULT_DDP_GRAD_SCALE", "1") or "1")


@dataclass
class _Bucket:
    index: int
    params: List[torch.nn.Parameter]
    offsets: List[int]
    numel: int
    buffer: Optional[torch.Tensor] = None
    pending: int = 0
    ready: bool = False
    launched: bool = False
    work: Any = None
    grads: List[torch.Tensor] = field(default_factory=list)
    param_flat: Optional[torch.Tensor] = None  # flat_params: the parameters live here (views)
    # shard=True: this rank's slice [lo, lo + shard) of the bucket, its averaged gradient, and
    # the in-flight all-gather of the updated parameter slices (set by FlatAdamW.step)
    shard: int = 0
    lo: int = 0
    grad_shard: Optional[torch.Tensor] = None
    gather_work: Any = None
    done: Any = None  # side-stream mode: event recorded after this bucket's collective
    views: Optional[List[torch.Tensor]] = None  # grad_views: each parameter's gradient home
    partial: bool = False  # no_sync: the bucket holds locally accumulated (unscaled) gradients
    rest_grads: List[torch.Tensor] = field(default_factory=list)  # gradients not written in place
    rest_offsets: List[int] = field(default_factory=list)
    post_div: bool = False  # averaged after the collective (no ReduceOp.AVG on this backend)


class _Done:
    """A collective that had nothing to do (world size 1)."""

    def wait(self, timeout=None) -> bool:
        return True

    def is_completed(self) -> bool:
        return True


_DONE = _Done()


class DistributedDataParallel(torch.nn.Module):
    def __init__(self, module: torch.nn.Module, process_group=None, bucket_cap_mb: float = 64.0,
                 first_bucket_mb: float = 4.0, comm_dtype: Optional[torch.dtype] = None,
                 broadcast_buffers: bool = True, init_sync: bool = True, align: int = 64,
                 flat_params: bool = False, grad_mode: str = "unflatten", shard: bool = False,
                 grad_views: Optional[bool] = None, fused_linear: Optional[bool] = None,
                 accumulate: str = "bucket", force_collectives: Optional[bool] = None,
                 cpp_hooks: Optional[bool] = None):
        """``flat_params``: re-home each bucket's parameters into one contiguous buffer (the
        nn.Parameters become views) so a flat optimizer (``nbdistributed_amd.optim.FlatAdamW``)
        can update a whole bucket in one pass.  ``grad_mode="bucket"``: leave the averaged
        gradients in the bucket buffers (no unflatten, ``p.grad`` released after the flatten) —
        only for optimizers that read the buckets (FlatAdamW).  ``shard=True``: ZeRO-2 —
        reduce-scatter the buckets, optimizer state and update on this rank's slice only (module
        docstring); needs ``flat_params=True, grad_mode="bucket"``.  ``grad_views`` (default: on
        for GPU modules): gradients live in their bucket slices (module docstring);
        ``fused_linear`` (default: = grad_views): route ``nn.Linear`` layers through the C++
        Linear node so their gradients are written in place too.  ``accumulate``: where
        ``no_sync()`` micro-batches accumulate — ``"bucket"`` (K3 pre-reduce into the bucket,
        ``p.grad`` released; same-dtype buckets) or ``"grad"`` (in ``p.grad``, torch's semantics).
        ``force_collectives`` (default: ``NBD_DDP_FORCE_COLLECTIVES=1``): issue the real
        collectives even at world size 1 — every code path of a multi-GPU run (per-bucket
        flushes, side-stream collectives and events, in-place reduce-scatter / all-gather, RCCL
        inside a captured graph) then runs, and can be timed and profiled, on one GPU.
        ``cpp_hooks`` (default: on for GPU modules, ``NBD_DDP_CPP_HOOKS=0`` turns it off): count
        bucket readiness in C++ hooks (``csrc/kernels/ddp_hooks.cpp``) instead of one Python hook
        per parameter."""
        super().__init__()
        self._token = object()  # ownership of registrations / patches shared with newer DDPs
        self.module = module
        self.pg = process_group if process_group is not None else dist.group.WORLD
        self.world = dist.get_world_size(self.pg)
        if force_collectives is None:
            force_collectives = os.environ.get("NBD_DDP_FORCE_COLLECTIVES", "0") == "1"
        # the multi-rank code path: collectives issued (always at world > 1; forced at world 1)
        self._collectives = self.world > 1 or bool(force_collectives)
        self.broadcast_buffers = broadcast_buffers
        self.params = [p for p in module.parameters() if p.requires_grad]
        if not self.params:
            raise ValueError("module has no trainable parameters")
        self.device = self.params[0].device
        self.cuda = self.device.type == "cuda"
        self.comm_dtype = comm_dtype or self.params[0].dtype
        if grad_mode not in ("unflatten", "bucket"):
            raise ValueError("grad_mode must be 'unflatten' or 'bucket'")
        self.grad_mode = grad_mode
        self.flat_params = flat_params
        if shard and not (flat_params and grad_mode == "bucket"):
            raise ValueError("shard=True needs flat_params=True and grad_mode='bucket' (with FlatAdamW)")
        self.shard = shard
        if accumulate not in ("bucket", "grad"):
            raise ValueError("accumulate must be 'bucket' or 'grad'")
        self.accumulate = accumulate
        self._sync_pass = True
        self.rank = dist.get_rank(self.pg)
        self._require_sync = True
        self._in_backward = False
        self._capturing = False
        self._side = False
        self._next_launch = 0
        # normal | high | none.  A high-priority stream measured 2.2x slower end to end on
        # MI355X (GPT-2 small DDP step 55 ms vs 25.5 ms, benchmarks/ddp_compare.py).
        mode = os.environ.get("NBD_DDP_COMM_STREAM", "normal")
        if not self.cuda or mode == "none":
            self.comm_stream = None
        else:
            self.comm_stream = torch.cuda.Stream(device=self.device, priority=-1 if mode == "high" else 0)
        self.buckets = self._plan(bucket_cap_mb, first_bucket_mb, align)
        self._bucket_of: Dict[int, _Bucket] = {}
        for b in self.buckets:
            if shard:  # equal, aligned slices: pad the bucket to a multiple of world x align
                q = self.world * align
                b.numel = (b.numel + q - 1) // q * q
                b.shard = b.numel // self.world
                b.lo = self.rank * b.shard
            b.buffer = torch.zeros(b.numel, dtype=self.comm_dtype, device=self.device)
            if shard:
                # this rank's slice of the bucket itself: the reduce-scatter runs in place
                # (recv = send + rank·count), no second buffer, and at world 1 it is the whole
                # bucket with nothing to send
                b.grad_shard = b.buffer[b.lo:b.lo + b.shard]
            for p in b.params:
                self._bucket_of[id(p)] = b
        if flat_params:
            self._rehome_params()
        # grad_mode="bucket" on the side stream: the optimizer waits for each bucket's own
        # collective (an event per bucket) instead of the whole comm stream, so the first
        # buckets' updates overlap the last buckets' all-reduces — at world > 1 the last bucket
        # (the tied embedding / LM head, finished only when backward ends) is never overlapped
        # by backward itself
        self._per_bucket_wait = self.comm_stream is not None and grad_mode == "bucket"
        self._joined = True
        if self._per_bucket_wait:
            for b in self.buckets:
                b.done = torch.cuda.Event()

        # gradients as bucket views (module docstring): same-dtype buckets only (a cast needs a copy)
        if grad_views is None:
            grad_views = self.cuda
        self.grad_views = bool(grad_views) and self.cuda
        self._avg_ok = self.cuda and dist.get_backend(self.pg) in ("nccl", "rccl")
        self._n_views = 0
        if self.grad_views:
            from ..ops import graddst

            for b in self.buckets:
                if any(p.dtype != b.buffer.dtype for p in b.params):
                    continue
                b.views = [b.buffer[o:o + p.numel()].view_as(p) for p, o in zip(b.params, b.offsets)]
                for p, v in zip(b.params, b.views):
                    graddst.register(p, v)
                    _GRAD_OWNER[id(p)] = self._token
                self._n_views += len(b.params)
        self._patched: List[torch.nn.Module] = []
        if (self.grad_views if fused_linear is None else fused_linear) and self._n_views:
            self._patch_linears()
        # weight-gradient split-K reduces into the slices are queued and issued in one launch per
        # flush (before a bucket's collective, at the end of backward) — ops.graddst.defer_enable
        # (process-wide switch; NBD_GRAD_DEFER=0 turns it off for A/B runs).  Every DDP with slices
        # flushes, whoever enabled it.
        self._on_bucket_ready = None  # FlatAdamW(overlap=True): update a bucket as soon as it is final
        self._defer = bool(self._n_views)
        if self._defer:
            from ..ops import graddst

            graddst.defer_enable(os.environ.get("NBD_GRAD_DEFER", "1") != "0")

        # the hooks reach this object through a weak reference, so a DDP that the notebook drops
        # (re-running the cell that wraps the same module) is collected; its finalizer removes
        # the hooks, its gradient-destination registrations and its patched forwards — unless a
        # newer DDP on the same module has taken them over (ownership token)
        wself = weakref.ref(self)
        self._hooks = []
        self._hook_handle = None
        self._hook_buckets = [self._bucket_of[id(p)].index for p in self.params]
        if cpp_hooks is None:
            cpp_hooks = self.cuda and os.environ.get("NBD_DDP_CPP_HOOKS", "1") != "0"
        if cpp_hooks and ops.native_available():
            # bucket readiness counted in C++ (csrc/kernels/ddp_hooks.cpp): Python is entered
            # once at the first gradient of a pass and once per completed bucket, not once per
            # parameter (the eager step is host-bound)
            def _on_bucket(i, _w=wself):
                s = _w()
                if s is not None:
                    s._bucket_event(i)

            self._hook_cb = _on_bucket
            self._hook_handle = int(torch.ops.nbd.ddp_hooks_install(self.params, self._hook_buckets, id(_on_bucket)))
        else:
            def _hook(p, _w=wself):
                s = _w()
                if s is not None:
                    s._grad_ready(p)

            self._hooks = [p.register_post_accumulate_grad_hook(_hook) for p in self.params]
        self._finalizer = weakref.finalize(self, _release, self._token, self._hooks, list(self._patched),
                                           [p for b in self.buckets if b.views is not None for p in b.params],
                                           self._hook_handle, list(self.params))
        if init_sync and self._collectives:
            self._broadcast_tensors([p.data for p in module.parameters()])
            self._broadcast_tensors(list(module.buffers()))
        self.stats = {"buckets": len(self.buckets), "bucket_numels": [b.numel for b in self.buckets],
                      "comm_dtype": str(self.comm_dtype), "grad_views": self._n_views,
                      "fused_linears": len(self._patched)}

    # ------------------------------------------------------------------ gradients in place
    def _patch_linears(self) -> None:
        """Route every ``nn.Linear`` whose parameters have bucket views through the C++ Linear
        autograd node (``torch.ops.nbd.linear_ag``), which writes dW / db into the views."""
        from ..ops import gemm as _gemm

        viewed = {id(p) for b in self.buckets if b.views is not None for p in b.params}
        for m in self.module.modules():
            if type(m) is not torch.nn.Linear or id(m.weight) not in viewed:
                continue
            if m.bias is not None and id(m.bias) not in viewed:
                continue
            m.forward = types.MethodType(_fused_linear_forward, m)
            m._nbd_ddp_owner = self._token
            self._patched.append(m)
        if self._patched:
            _gemm.native_available_or_raise()

    def unpatch(self) -> None:
        """Undo ``fused_linear`` and the gradient-destination registrations (those still owned
        by this DDP); also runs when the DDP object is garbage-collected."""
        params = [p for b in self.buckets if b.views is not None for p in b.params]
        _release(self._token, [], self._patched, params)  # (the bucket hooks stay: DDP still counts)
        self._patched = []
        for b in self.buckets:
            b.views = None
        self._n_views = 0

    # ------------------------------------------------------------------ planning
    def _plan(self, cap_mb: float, first_mb: float, align: int) -> List[_Bucket]:
        esz = torch.tensor([], dtype=self.comm_dtype).element_size()
        buckets: List[_Bucket] = []
        cur: List[torch.nn.Parameter] = []
        cur_bytes = 0
        limit = first_mb * 2 ** 20
        for p in reversed(self.params):
            nbytes = p.numel() * esz
            if cur and cur_bytes + nbytes > limit:
                buckets.append(self._make_bucket(len(buckets), cur, align))
                cur, cur_bytes = [], 0
                limit = cap_mb * 2 ** 20
            cur.append(p)
            cur_bytes += nbytes
        if cur:
            buckets.append(self._make_bucket(len(buckets), cur, align))
        return buckets

    @staticmethod
    def _make_bucket(i: int, params: List[torch.nn.Parameter], align: int) -> _Bucket:
        offs, total = ops.plan_offsets([p.numel() for p in params], align)
        return _Bucket(index=i, params=list(params), offsets=offs, numel=total)

    def _rehome_params(self) -> None:
        for b in self.buckets:
            dts = {p.dtype for p in b.params}
            if len(dts) != 1:
                raise ValueError(f"flat_params needs one dtype per bucket, got {dts}")
            flat = torch.zeros(b.numel, dtype=dts.pop(), device=self.device)
            with torch.no_grad():
                for p, o in zip(b.params, b.offsets):
                    n = p.numel()
                    flat[o:o + n].copy_(p.data.reshape(-1))
                    p.data = flat[o:o + n].view_as(p)
            b.param_flat = flat

    # ------------------------------------------------------------------ ZeRO parameter gathers
    @staticmethod
    def _wait_gathers(buckets) -> None:
        for b in buckets:
            if b.gather_work is not None:
                b.gather_work.wait()  # RCCL: the current stream waits on the collective (device side)
                b.gather_work = None

    def wait_params(self) -> None:
        """Make the current stream wait until every parameter all-gather of a sharded step has
        landed (``shard=True``; forward does this itself — call it before reading the
        parameters directly)."""
        self._wait_gathers(self.buckets)

    def wait_grad(self, b: _Bucket) -> None:
        """Make the current stream wait until bucket ``b``'s averaged gradient is in place
        (``b.buffer`` / ``b.grad_shard``; a no-op unless the side stream defers the join)."""
        if not self._joined and b.done is not None:
            torch.cuda.current_stream(self.device).wait_event(b.done)

    def wait_grads(self) -> None:
        """Make the current stream wait for every bucket's gradient collective."""
        if not self._joined:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)
            self._joined = True

    def _reduce(self, b: _Bucket, avg: bool = False):
        if not self._collectives:
            # nothing to exchange (and for ZeRO the slice is the whole bucket).  Not even a no-op
            # launch: RCCL runs a one-rank ReduceOp.AVG as a full pre-multiply pass over the bucket
            # (oneRankReduce<FuncPreMulSum>: 190 µs per 48 MB bucket, profiles/gpt2_graph_prof_r3*.md)
            return _DONE
        # (forced at world 1: the average over one rank is the sum — RCCL would run AVG as a
        # separate pre-multiply pass over the bucket there, an artefact no N-GPU run has)
        op = dist.ReduceOp.AVG if avg and self.world > 1 else dist.ReduceOp.SUM
        if _FAULT_GRAD_SCALE != 1.0 and self.rank == 0:
            # fault injection (tests only): a broken gradient hook — rank 0 contributes a scaled
            # bucket, so the averaged gradient is wrong by a small factor and nothing else fails
            # (what nbdistributed_amd.checks' DDP-parity check must catch)
            b.buffer.mul_(_FAULT_GRAD_SCALE)
        if self.shard:  # ZeRO-2: this rank keeps the averaged gradient of its slice only
            return dist.reduce_scatter_tensor(b.grad_shard, b.buffer, op=op, group=self.pg, async_op=True)
        return dist.all_reduce(b.buffer, op=op, group=self.pg, async_op=True)

    # ------------------------------------------------------------------ forward
    def forward(self, *args, **kwargs):
        if self._in_backward and torch._C._current_graph_task_id() == -1:
            # a backward that raised never reached _finalize: this forward starts a new pass
            self._in_backward = False
            for b in self.buckets:
                b.work, b.grads, b.rest_grads, b.rest_offsets = None, [], [], []
        if self._hook_handle is not None and torch.is_grad_enabled():
            # a new pass (also after a backward that raised); hooks a user registered since
            # replaced ours: wrap theirs again
            self._rearm()
            if torch.ops.nbd.ddp_hooks_intact(self._hook_handle, self.params) != len(self.params):
                torch.ops.nbd.ddp_hooks_reattach(self._hook_handle, self.params, self._hook_buckets)
        if self._n_views:
            from ..ops import graddst

            graddst.new_pass()  # each gradient home may be handed out once per backward
        if self.shard:
            # the updated parameter slices of the last step must be back on every rank.  (Per
            # module pre-forward waits would let the first layers start earlier, but the models'
            # fused paths read weights without calling their modules' forward, so the hooks
            # would not fire: all buckets are waited here.)
            self._wait_gathers(self.buckets)
        if self._require_sync and self.broadcast_buffers and self._collectives:
            bufs = [b for b in self.module.buffers() if b.is_floating_point() or b.dtype in (torch.int64, torch.int32)]
            if bufs:
                self._broadcast_tensors(bufs)
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._require_sync
        self._require_sync = False
        try:
            yield
        finally:
            self._require_sync = prev

    # ------------------------------------------------------------------ backward hooks
    def _start_backward(self) -> None:
        self._in_backward = True
        self._sync_pass = self._require_sync
        self._next_launch = 0
        # Under HIP-graph capture the collectives are issued from the capturing stream itself
        # (ProcessGroupNCCL's own stream becomes a parallel branch of the graph) and every wait
        # is deferred to the end of backward: forking RCCL work off a second user stream inside
        # a capture crashes hipStreamEndCapture on this stack (benchmarks/graph_probe.py "side").
        self._capturing = self.cuda and torch.cuda.is_current_stream_capturing()
        self._side = self.comm_stream is not None and not self._capturing
        self._joined = True  # (re)set by _finalize; under capture every wait stays in the graph
        for b in self.buckets:
            b.pending = len(b.params)
            b.ready = b.launched = False
            b.work = None
        torch.autograd.Variable._execution_engine.queue_callback(self._finalize)

    def _bucket_event(self, i: int) -> None:
        """C++ hook callback: ``i = -1`` first gradient of a pass, else bucket ``i`` complete."""
        if not self._in_backward:
            self._start_backward()
        if i < 0:
            return
        b = self.buckets[i]
        b.pending = 0
        b.ready = True
        if self._sync_pass:
            self._launch_ready()
        else:
            self._prereduce_local(b)

    def _grad_ready(self, p: torch.nn.Parameter) -> None:
        if not self._in_backward:
            self._start_backward()
        b = self._bucket_of[id(p)]
        b.pending -= 1
        if b.pending == 0:
            b.ready = True
            if self._sync_pass:
                self._launch_ready()
            else:
                self._prereduce_local(b)

    def _split_in_place(self, b: _Bucket):
        """(#gradients already in their bucket slice, indices of the other parameters)."""
        n_in, rest = 0, []
        for i, p in enumerate(b.params):
            g = p.grad
            if b.views is not None and g is not None and g.data_ptr() == b.views[i].data_ptr():
                n_in += 1
            else:
                rest.append(i)
        return n_in, rest

    def _local_home(self, b: _Bucket) -> bool:
        """no_sync micro-batches accumulate in this bucket (K3) rather than in ``p.grad``: when its
        dtype is the parameters' own (no precision lost against autograd's accumulation)."""
        return self.accumulate == "bucket" and all(p.dtype == b.buffer.dtype for p in b.params)

    def _prereduce_local(self, b: _Bucket) -> None:
        """no_sync micro-batch: fold this bucket's new gradients into the bucket.

        Bucket with gradient views: after every micro-batch each ``p.grad`` IS its slice, so the
        next micro-batch accumulates in place (the GEMM epilogues claim the slice with
        ``acc=True``; autograd's AccumulateGrad adds into a defined ``.grad`` in place).  A
        gradient that still arrives elsewhere — a weight used twice in one pass, whose
        contributions the engine sums out of place — was computed as ``old .grad + new``, i.e.
        it already contains the slice: it OVERWRITES the slice (adding it would count the earlier
        micro-batches twice).  Bucket without views: the new gradients are summed into the bucket
        (K3, fp32 accumulate) and released."""
        if not self._local_home(b):
            return  # plain autograd accumulation into p.grad (torch semantics)
        _, rest = self._split_in_place(b)
        arrived = [i for i in rest if b.params[i].grad is not None]
        if not b.partial:
            # the first micro-batch defines the bucket: zero the slices of parameters that got no
            # gradient, overwrite the others (in-place gradients were written by their GEMMs)
            for i in rest:
                if b.params[i].grad is None:
                    o = b.offsets[i]
                    b.buffer[o:o + b.params[i].numel()].zero_()
        overwrite = not b.partial or b.views is not None
        if arrived:
            gs, offs = [b.params[i].grad for i in arrived], [b.offsets[i] for i in arrived]
            if overwrite:
                ops.bucket_flatten(gs, b.buffer, offs)
            else:
                ops.prereduce_into_bucket(gs, b.buffer, offs)
        if b.views is not None:
            for p, v in zip(b.params, b.views):
                p.grad = v  # the running sum: later micro-batches accumulate into it in place
        else:
            for i in arrived:
                b.params[i].grad = None
        b.partial = True

    def _launch_ready(self) -> None:
        while self._next_launch < len(self.buckets) and self.buckets[self._next_launch].ready:
            self._launch(self.buckets[self._next_launch])
            self._next_launch += 1

    def _bucket_grads(self, b: _Bucket) -> List[torch.Tensor]:
        grads = []
        for p in b.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            grads.append(p.grad)
        return grads

    def _flush_deferred(self) -> None:
        if self._defer:
            from ..ops import graddst

            graddst.defer_flush()

    def _launch(self, b: _Bucket) -> None:
        if self._collectives or self._on_bucket_ready is not None:
            self._flush_deferred()  # the collective / the update reads the slices: their reduces go first
        n_in, rest = self._split_in_place(b)
        if n_in == 0 and not b.partial:
            self._launch_flat(b)
            return
        # some gradients are already in their slices (bucket views), or the bucket holds the
        # no_sync micro-batches' local sum: the rest are pre-reduced into the bucket unscaled and
        # the collective averages (ReduceOp.AVG; a divide after it where the backend has no AVG)
        grads = []
        for i in rest:
            p = b.params[i]
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            grads.append(p.grad)
        offs = [b.offsets[i] for i in rest]
        b.rest_grads, b.rest_offsets = grads, offs
        avg = self._avg_ok
        b.post_div = not avg and self._collectives
        unflatten = self.grad_mode == "unflatten"

        # a partial bucket with views: every arrival was computed on top of its slice (see
        # _prereduce_local) and replaces it; without views the arrivals are new and add up
        acc_rest = b.partial and b.views is None

        def pre():
            if grads:
                ops.bucket_flatten(grads, b.buffer, offs, scale=1.0, accumulate=acc_rest)

        def post():
            if b.post_div:
                (b.grad_shard if self.shard else b.buffer).div_(self.world)
            if unflatten and grads:
                ops.bucket_unflatten(b.buffer, grads, offs)

        if self.cuda and self._capturing:
            pre()
            b.work = self._reduce(b, avg)  # waited (and post-processed) in _finalize
        elif self.cuda and not self._side:
            pre()
            self._reduce(b, avg).wait()
            post()
            b.work = None
        elif self.cuda:
            cur = torch.cuda.current_stream(self.device)
            self.comm_stream.wait_stream(cur)
            with torch.cuda.stream(self.comm_stream):
                pre()
                self._reduce(b, avg).wait()
                post()
                if self._per_bucket_wait:
                    b.done.record(self.comm_stream)
            for g in grads:
                g.record_stream(self.comm_stream)
        else:
            pre()
            b.work = self._reduce(b, avg)
        b.partial = False
        if not unflatten:
            for p in b.params:
                p.grad = None
            if not self.cuda:
                b.rest_grads = []
        b.launched = True
        if self._on_bucket_ready is not None:
            self._on_bucket_ready(b)

    def _launch_flat(self, b: _Bucket) -> None:
        """No gradient in place: flatten (pre-divided by the world size) -> all-reduce SUM ->
        unflatten."""
        grads = self._bucket_grads(b)
        b.grads = grads
        b.rest_grads, b.rest_offsets, b.post_div = [], [], False
        scale = 1.0 / self.world
        unflatten = self.grad_mode == "unflatten"
        if self.cuda and self._capturing:
            ops.bucket_flatten(grads, b.buffer, b.offsets, scale=scale)
            b.work = self._reduce(b)  # waited in _finalize
        elif self.cuda and not self._side:
            ops.bucket_flatten(grads, b.buffer, b.offsets, scale=scale)
            b.work = self._reduce(b)
            b.work.wait()
            if unflatten:
                ops.bucket_unflatten(b.buffer, grads, b.offsets)
            b.work = None
        elif self.cuda:
            cur = torch.cuda.current_stream(self.device)
            self.comm_stream.wait_stream(cur)  # the grads were produced on the compute stream
            with torch.cuda.stream(self.comm_stream):
                ops.bucket_flatten(grads, b.buffer, b.offsets, scale=scale)
                b.work = self._reduce(b)
                b.work.wait()  # device-side: the comm stream waits for RCCL's stream
                if unflatten:
                    ops.bucket_unflatten(b.buffer, grads, b.offsets)
                if self._per_bucket_wait:
                    b.done.record(self.comm_stream)
            for g in grads:
                g.record_stream(self.comm_stream)
        else:
            ops.bucket_flatten(grads, b.buffer, b.offsets, scale=scale)
            b.work = self._reduce(b)
        if not unflatten:
            # the averaged gradients live in b.buffer; release the per-parameter grads now
            # (the caching allocator will not reuse them before the comm stream is done)
            for p in b.params:
                p.grad = None
            if not self.cuda:
                b.grads = []
        b.launched = True
        if self._on_bucket_ready is not None:
            self._on_bucket_ready(b)

    def _finalize(self) -> None:
        self._flush_deferred()
        if not self._sync_pass:  # no_sync micro-batch: buckets hold the local sums, nothing to send
            if self._hook_handle is not None and not all(b.ready for b in self.buckets):
                for b, n in zip(self.buckets, torch.ops.nbd.ddp_hooks_pending(self._hook_handle)):
                    b.pending = int(n)
            for b in self.buckets:
                if not b.ready and b.pending < len(b.params):
                    self._prereduce_local(b)  # (some parameters of it got no gradient)
            self._in_backward = False
            self._rearm()
            return
        # buckets whose params got no gradient this step (unused parameters): zeros
        for b in self.buckets:
            if not b.ready:
                b.ready = True
        self._launch_ready()
        if self.cuda and self._side and self._per_bucket_wait:
            self._joined = False  # consumers wait per bucket: wait_grad(b) / wait_grads()
        elif self.cuda and self._side:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)
        else:
            for b in self.buckets:
                if b.work is not None:
                    b.work.wait()
                    if b.post_div:
                        (b.grad_shard if self.shard else b.buffer).div_(self.world)
                    if self.grad_mode == "unflatten":
                        if b.grads:
                            ops.bucket_unflatten(b.buffer, b.grads, b.offsets)
                        elif b.rest_grads:
                            ops.bucket_unflatten(b.buffer, b.rest_grads, b.rest_offsets)
        for b in self.buckets:
            b.grads = []
            b.rest_grads, b.rest_offsets = [], []
            b.work = None
        self._in_backward = False
        self._rearm()

    def _rearm(self) -> None:
        if self._hook_handle is not None:
            torch.ops.nbd.ddp_hooks_rearm(self._hook_handle)

    # ------------------------------------------------------------------ broadcast
    def _broadcast_tensors(self, tensors: List[torch.Tensor]) -> None:
        broadcast_tensors(tensors, src=0, group=self.pg)


# id(param) -> token of the DDP whose bucket slice is its registered gradient home
_GRAD_OWNER: Dict[int, object] = {}


def _release(token, hooks, patched, params, hook_handle=None, all_params=()) -> None:
    """Undo one DDP's hooks, patched ``nn.Linear`` forwards and gradient-destination
    registrations, leaving alone whatever a newer DDP on the same module has taken over."""
    for h in hooks:
        h.remove()
    if hook_handle is not None:
        try:
            torch.ops.nbd.ddp_hooks_remove(hook_handle, list(all_params))
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
    for m in patched:
        if m.__dict__.get("_nbd_ddp_owner") is token:
            m.__dict__.pop("forward", None)
            m.__dict__.pop("_nbd_ddp_owner", None)
    mine = [p for p in params if _GRAD_OWNER.get(id(p)) is token]
    if mine:
        try:
            from ..ops import graddst

            for p in mine:
                graddst.register(p, None)
                _GRAD_OWNER.pop(id(p), None)
        except Exception:  # noqa: BLE001 - interpreter shutdown: the registry dies with the process
            pass


def _fused_linear_forward(self, x):
    """``nn.Linear.forward`` through the C++ Linear node (``torch.ops.nbd.linear_ag``): same
    math (bf16: the HIP GEMMs; fp32 / fp16: the library GEMMs), with dW / db written straight into
    the DDP bucket slices (``ops.graddst``).  Autocast and CPU inputs keep the stock path."""
    if not x.is_cuda or torch.is_autocast_enabled() or x.dtype != self.weight.dtype:
        return torch.nn.functional.linear(x, self.weight, self.bias)
    from ..ops import gemm as _gemm

    return _gemm.linear_any(x, self.weight, self.bias)


def broadcast_tensors(tensors: List[torch.Tensor], src: int = 0, group=None, coalesce_max_bytes: int = 4 << 20) -> None:
    """In-place broadcast of ``tensors`` from ``src`` (a rank of ``group``).

    Tensors smaller than ``coalesce_max_bytes`` are latency-bound one by one (one RCCL launch and
    ring traversal each — the README pattern ``for p in model.parameters(): dist.broadcast(...)``,
    reference ``README.md:115-125``); they are packed per dtype by one fused HIP kernel
    (``nbd::bucket_flatten``) into one buffer, sent as ONE broadcast and scattered back by
    ``nbd::bucket_unflatten``.  Larger contiguous tensors are bandwidth-bound and go out directly
    in place (no copies)."""
    pg = group if group is not None else dist.group.WORLD
    gsrc = src if pg is dist.group.WORLD else dist.get_global_rank(pg, src)
    groups: Dict[torch.dtype, List[torch.Tensor]] = {}
    for t in tensors:
        big = t.numel() * t.element_size() >= coalesce_max_bytes and t.is_contiguous()
        if big or t.dtype not in (torch.float32, torch.bfloat16, torch.float16):
            dist.broadcast(t, src=gsrc, group=pg)
        else:
            groups.setdefault(t.dtype, []).append(t)
    for dt, ts in groups.items():
        if len(ts) == 1 and ts[0].is_contiguous():
            dist.broadcast(ts[0], src=gsrc, group=pg)
            continue
        flat = [t if t.is_contiguous() else t.contiguous() for t in ts]
        buf, offs = ops.bucket_flatten(flat, dtype=dt)
        dist.broadcast(buf, src=gsrc, group=pg)
        ops.bucket_unflatten(buf, flat, offs)
        for t, f in zip(ts, flat):
            if t.data_ptr() != f.data_ptr():
                t.copy_(f)


def broadcast_params(module: torch.nn.Module, src: int = 0, group=None, buffers: bool = True) -> None:
    """Make every rank's ``module`` parameters (and buffers) equal to rank ``src``'s — the
    ``%%rank[0]`` build-then-broadcast pattern in one call."""
    with torch.no_grad():
        ts = [p.data for p in module.parameters()]
        if buffers:
            ts += list(module.buffers())
        broadcast_tensors(ts, src=src, group=group)


# ---------------------------------------------------------------------- comm hooks for torch DDP
def bf16_compress_hook(process_group, bucket):
    """Fused replacement for torch's bf16_compress_hook: one HIP kernel casts fp32 -> bf16 and
    pre-divides, RCCL all-reduces the bf16 bucket, one HIP kernel casts back into the fp32
    bucket (torch's version runs three eager kernels plus a copy)."""
    group = process_group if process_group is not None else dist.group.WORLD
    world = dist.get_world_size(group)
    buf = bucket.buffer()
    comp = torch.empty(buf.numel(), dtype=torch.bfloat16, device=buf.device)
    ops.bucket_flatten([buf], comp, [0], scale=1.0 / world)
    fut = dist.all_reduce(comp, group=group, async_op=True).get_future()

    def _decompress(f):
        ops.bucket_unflatten(comp, [buf], [0])
        return buf

    return fut.then(_decompress)


def allreduce_hook(process_group, bucket):
    """Plain averaging all-reduce with the pre-divide fused into one HIP pass."""
    group = process_group if process_group is not None else dist.group.WORLD
    world = dist.get_world_size(group)
    buf = bucket.buffer()
    ops.bucket_unflatten(buf, [buf], [0], scale=1.0 / world)  # in-place scale (same-dtype copy)
    fut = dist.all_reduce(buf, group=group, async_op=True).get_future()
    return fut.then(lambda f: f.value()[0])
