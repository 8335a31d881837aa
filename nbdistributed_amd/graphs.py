"""HIP graphs for whole training steps — the MI355X answer to launch-bound cells.

A small-batch step of a deep model is thousands of short kernels (SmolLM2-135M at batch 16 x 128:
≈4,600 launches, GPU busy 25 ms of a 40 ms eager step: ``profiles/notebook_prof_r1.md``).
:class:`GraphedStep` records one step — forward, backward, the DDP bucket pipeline (flatten
kernels, RCCL all-reduce on the side stream, stream joins) and the optimizer — into a HIP graph
once, then replays it: one launch per step, no Python or per-kernel launch cost.

Requirements (checked by construction, as for any CUDA/HIP graph):
* static shapes; inputs are copied into the graph's static tensors on each call;
* no host synchronisation inside the step (``.item()``, ``print(tensor)``, data-dependent
  Python control flow);
* optimizers that keep step/lr on the device: ``FlatAdamW(..., capturable=True)`` or
  ``torch.optim.AdamW(..., capturable=True)``; ``sync_hyper()`` (FlatAdamW) is called before
  each replay so LR schedulers keep working.
"""
from __future__ import annotations

import contextlib
from typing import Any, Callable, Iterable, Sequence

import torch


def _clone_static(x):
    if isinstance(x, torch.Tensor):
        return x.detach().clone()
    return x


def _copy_into(dst, src):
    if isinstance(dst, torch.Tensor):
        if src.shape != dst.shape or src.dtype != dst.dtype:
            raise ValueError(f"GraphedStep: input {tuple(src.shape)}/{src.dtype} does not match the captured "
                             f"{tuple(dst.shape)}/{dst.dtype}")
        dst.copy_(src, non_blocking=True)
    elif dst is not src and dst != src:
        raise ValueError("GraphedStep: non-tensor arguments are baked into the graph and must not change")


# checks attached to the capture in progress (note_capture_check): objects with before_replay()
# and after_replay(), e.g. the Llama fused path's attention-mask check (models/llama.py)
_CAPTURE_CHECKS: list = []


def note_capture_check(check) -> None:
    """Called by a model op whose host-side check cannot run inside a stream capture: the check
    then runs around every replay of the graph being captured (``GraphedStep``)."""
    _CAPTURE_CHECKS.append(check)


def _drain_collective_watchdog(poll_s: float = 0.35) -> None:
    """ProcessGroupNCCL's watchdog thread polls the events of outstanding collectives (every
    ~100 ms) and retires completed ones.  Warm-up collectives still on its list when capture
    starts get their (recycled) events queried mid-capture, which aborts the process
    ("operation not permitted when stream is capturing" / "... on an event last recorded in a
    capturing stream").  After a device sync every warm-up collective is complete; give the
    watchdog a few polling periods to drop them.  Collectives issued during capture are never
    put on its list."""
    import time

    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        time.sleep(poll_s)


def _take_warm_refs():
    """Tensors aliasing every storage that GEMM launches captured since the last call warm up
    (``torch.ops.nbd.gemm_warm_take_refs``); empty without the native extension."""
    try:
        from .ops import _lib

        if not _lib.native_available():
            return []
        return list(torch.ops.nbd.gemm_warm_take_refs())
    except (AttributeError, RuntimeError):
        return []


@contextlib.contextmanager
def _suspend_block_graphs():
    """The per-block graphs of the eager Llama step (ops.block_graphs) off while a whole step is
    warmed up and captured: inside the capture the blocks are part of the outer graph anyway, and
    block graphs made during the warm-up would only hold static memory nobody replays."""
    prev = None
    try:
        from .ops import _lib

        if _lib._loaded:
            prev = bool(torch.ops.nbd.llama_block_graphs_suspend(True))
    except (AttributeError, RuntimeError):
        prev = None
    try:
        yield
    finally:
        if prev is not None:
            torch.ops.nbd.llama_block_graphs_suspend(prev)


def _capture(graph, body, pool=None) -> None:
    """``body()`` captured into ``graph`` on a fresh stream; whatever happens, the caller's stream
    and the device's default RNG come back usable.  (``torch.cuda.graph`` leaves its capture
    stream current when ``capture_end`` raises — e.g. ``hipErrorStreamCaptureUnjoined`` from a
    collective whose side-stream work was not joined — and skips the RNG's capture epilogue, so
    ``torch.manual_seed`` and every later random op on the thread failed.  A failed capture here
    costs only this graph.)"""
    import gc

    torch.cuda.synchronize()
    gc.collect()
    gen = torch.cuda.default_generators[torch.cuda.current_device()]
    rng = gen.clone_state()  # (not capturing: put back if the capture fails half way)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        graph.capture_begin(pool=pool, capture_error_mode="thread_local")
        try:
            try:
                body()
            except BaseException:
                try:
                    graph.capture_end()
                except Exception:  # noqa: BLE001 - the body's error is the one to report
                    pass
                raise
            graph.capture_end()
        except BaseException:
            gen.graphsafe_set_state(rng)
            raise
    torch.cuda.current_stream().wait_stream(stream)


class GraphedStep:
    """``step = GraphedStep(fn, example_args, optimizers=[opt])``; ``out = step(*args)``.

    ``fn(*args)`` runs ``warmup`` times eagerly on a side stream (allocator and library
    warm-up, DDP bucket state), is captured once, and every call replays the graph after
    copying ``args`` into the static inputs.  Returns the captured output tensors (overwritten
    by the next replay — clone what you keep).
    """

    def __init__(self, fn: Callable[..., Any], example_args: Sequence[Any], warmup: int = 3,
                 optimizers: Iterable[Any] = (), pool=None):
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedStep needs a GPU")
        self.fn = fn
        self.optimizers = list(optimizers)
        self.static_args = [_clone_static(a) for a in example_args]
        self.replays = 0
        with _suspend_block_graphs():
            self._warm_and_capture(fn, warmup, pool)

    def _warm_and_capture(self, fn, warmup, pool) -> None:
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self._sync_hyper()
                fn(*self.static_args)
        cur.wait_stream(side)
        torch.cuda.synchronize()
        _drain_collective_watchdog()
        self.graph = torch.cuda.CUDAGraph()
        self._sync_hyper()
        # thread_local: only this thread's calls are checked during capture — ProcessGroupNCCL's
        # watchdog thread keeps querying its events meanwhile, which "global" mode turns into a
        # hipErrorStreamCaptureUnsupported abort (seen intermittently on this stack)
        _take_warm_refs()  # (drop references left by an earlier capture that nobody took)
        del _CAPTURE_CHECKS[:]
        try:
            _capture(self.graph, lambda: setattr(self, "static_out", fn(*self.static_args)), pool)
            self._checks = list(_CAPTURE_CHECKS)
        finally:
            del _CAPTURE_CHECKS[:]
        # the captured GEMMs' next-weight warm-up reads (csrc/kernels/gemm.hip, namespace warm)
        # are frozen pointers into those weights' storages: hold them as long as the graph
        self._warm_refs = _take_warm_refs()
        torch.cuda.synchronize()

    def _sync_hyper(self) -> None:
        for o in self.optimizers:
            sync = getattr(o, "sync_hyper", None)
            if sync is not None:
                sync()

    def __call__(self, *args):
        if len(args) != len(self.static_args):
            raise ValueError(f"GraphedStep: expected {len(self.static_args)} arguments, got {len(args)}")
        dsts, srcs = [], []
        for dst, src in zip(self.static_args, args):
            if isinstance(dst, torch.Tensor) and isinstance(src, torch.Tensor) and src.device == dst.device:
                if src.shape != dst.shape or src.dtype != dst.dtype:
                    _copy_into(dst, src)  # (raises with the mismatch)
                if src.data_ptr() != dst.data_ptr():
                    dsts.append(dst)
                    srcs.append(src)
            else:
                _copy_into(dst, src)
        if dsts:  # the step's device inputs in one multi-tensor launch, not one copy each
            torch._foreach_copy_(dsts, srcs, non_blocking=True)
        self._sync_hyper()
        for c in self._checks:
            c.before_replay()
        self.graph.replay()
        self.replays += 1
        for c in self._checks:
            c.after_replay()
        return self.static_out


__all__ = ["GraphedStep"]
