"""Benchmarks driven exactly like a notebook: every measured step is a ``%%distributed`` cell.

Headline metric (BASELINE.json): ``%%distributed`` cell p50 round trip (ms) and all_reduce bus
bandwidth (GB/s) at 1/2/4/8 MI355X.  The reference's own number is 111.6 ms per trivial cell on
2 GPUs (``00_accelerate.ipynb:1127``; 100 ms display-poll quantum, ``magic.py:1092-1094``).

Phases (all through Session.execute → native transport → worker exec → response):

1. ``cell``      — W warm-up + K timed trivial cells, bracketed by ``%sync`` (barrier +
                   ``torch.cuda.synchronize`` on every rank); coordinator wall clock, which is
                   the max over ranks by construction (a cell ends when the last rank replies).
2. ``allreduce`` — one cell times ``iters`` in-place all_reduces of a 1 GiB bf16 buffer with HIP
                   events on every rank (config 2); max over ranks; nccl-tests formulas
                   algbw = bytes/t, busbw = algbw·2(n−1)/n (undefined at n = 1 → null).
3. ``sweep``     — optional 1 KiB … 1 GiB curve.
"""
from __future__ import annotations

import os
import statistics
import sys
import time
from typing import Any, Dict, List, Optional

BASELINE_CELL_P50_MS = 111.6
METRIC = "all_reduce bus GB/s + %%distributed cell p50 round-trip (ms) at 1/2/4/8 MI355X"

AR_SETUP = """
import time as _t
def _nbd_sync():
    if device.type == 'cuda':
        torch.cuda.synchronize()

def _nbd_barrier():
    _nbd_sync()
    dist.barrier(device_ids=[device.index]) if device.type == 'cuda' else dist.barrier()
    _nbd_sync()

def _nbd_ar_time(numel, dtype, iters, warm):
    x = torch.zeros(numel, dtype=dtype, device=device)
    for _ in range(warm):
        dist.all_reduce(x)
    _nbd_barrier()
    if device.type == 'cuda':
        s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            dist.all_reduce(x)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / iters
    else:
        t = _t.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x)
        ms = (_t.perf_counter() - t) / iters * 1e3
    del x
    return ms

def _nbd_ar_check():
    y = torch.full((1024,), float(rank + 1), dtype=torch.bfloat16, device=device)
    dist.all_reduce(y)
    want = world_size * (world_size + 1) / 2
    return bool((y.float() == want).all().item())
"""


DDP_SETUP = """
import time as _t
from nbdistributed_amd.models import GPT2, GPT2Config, linear_4096
from nbdistributed_amd.parallel import DistributedDataParallel as _NbdDDP
from nbdistributed_amd.optim import FlatAdamW as _FlatAdamW
from torch.nn.parallel import DistributedDataParallel as _TorchDDP

def _nbd_time_steps(step, steps, warm, per_step=False):
    # per_step: a HIP event after every timed step (graph replays), so a slow arm shows whether
    # its first replays or its steady state are slow
    for _ in range(warm):
        step()
    _nbd_barrier()
    evs = None
    if per_step and device.type == "cuda":
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        evs[0].record()
    t = _t.perf_counter()
    for i in range(steps):
        out = step()
        if evs is not None:
            evs[i + 1].record()
    _nbd_sync()
    ms = (_t.perf_counter() - t) / steps * 1e3
    if evs is None:
        return ms, float(out)
    d = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
    rest = sorted(d[3:]) or sorted(d)
    return ms, float(out), {"replay_ms_first3": [round(x, 4) for x in d[:3]],
                            "replay_ms_median": round(rest[len(rest) // 2], 4), "replay_ms_max": round(max(d), 4)}

def _nbd_wrap(m, impl, **kw):
    if impl == "nbd":
        return _NbdDDP(m, **kw)
    return _TorchDDP(m, device_ids=[device.index] if device.type == "cuda" else None, bucket_cap_mb=25)

def _nbd_gpt2_bench(steps, warm, B, T, impl, config="small", force=False, lmhead_lib=False, lmhead_hip=False):
    # force: the multi-rank DDP code path even at world size 1 (real collectives per bucket)
    # lmhead_lib: the LM head's three GEMMs on hipBLASLt (NBD_LMHEAD_HIP=0), the table padded to a
    # multiple of 128 as the library wants; lmhead_hip: all three on the hand-written kernels
    # (NBD_LMHEAD_HIP=1); neither: the default per-product plan (ops.loss.HEAD_PRODUCTS)
    if impl == "flatgraph" and device.type != "cuda":
        impl = "flat"   # HIP graphs need a GPU
    import nbdistributed_amd.ops.loss as _lm
    prev_hip, prev_products = _lm.LM_HEAD_HIP, _lm.HEAD_PRODUCTS
    if lmhead_lib:
        _lm.LM_HEAD_HIP = False
    if lmhead_hip:
        _lm.LM_HEAD_HIP, _lm.HEAD_PRODUCTS = True, {"fwd": True, "dgrad": True, "wgrad": True}
    try:
        # the table padded as each plan wants it (ops.loss.table_pad): 128 for the library, 512 with
        # the hand-written input gradient, the default plan's own otherwise
        return _nbd_gpt2_bench_body(steps, warm, B, T, impl, config, force,
                                    128 if lmhead_lib else 512 if lmhead_hip else 0)
    finally:
        _lm.LM_HEAD_HIP, _lm.HEAD_PRODUCTS = prev_hip, prev_products

def _nbd_gpt2_bench_body(steps, warm, B, T, impl, config, force, vocab_pad):
    # vocab_pad: the table's padding multiple (0: GPT2Config's default)
    torch.manual_seed(0)
    cfg = getattr(GPT2Config, config)()
    if vocab_pad:
        cfg.vocab_pad = vocab_pad
    m = GPT2(cfg).to(device)
    amp = impl not in ("flat", "flatgraph", "zero")
    if not amp:   # bf16 params in the DDP buckets + fp32 master/moments in FlatAdamW
        m = m.to(torch.bfloat16)
        model = _NbdDDP(m, flat_params=True, grad_mode="bucket", shard=impl == "zero",
                        force_collectives=bool(force))
        opt = _FlatAdamW(model, lr=3e-4, capturable=impl == "flatgraph")
    else:
        model = _nbd_wrap(m, impl, comm_dtype=torch.bfloat16)
        opt = torch.optim.AdamW(m.parameters(), lr=3e-4, fused=device.type == "cuda")
    x = torch.randint(0, m.config.vocab_size, (B, T), device=device)
    def step(inp=x):
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=amp):
            _, loss = model(inp, inp, return_logits=False)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss.detach()
    run = step
    if impl == "flatgraph":   # the whole step (fwd, bwd, bucket all-reduces, AdamW) as one HIP graph
        from nbdistributed_amd.graphs import GraphedStep
        g = GraphedStep(step, (x,), warmup=3, optimizers=[opt])
        run = lambda: g(x)
    res = _nbd_time_steps(run, steps, warm, per_step=impl == "flatgraph")
    del model, opt, m, x, run
    if device.type == "cuda":
        torch.cuda.empty_cache()
    return res

def _nbd_linear_bench(steps, warm, rows, impl, dim=4096, bf16=False):
    # bf16: the same step on a bf16 Linear (nbd: flat bf16 parameters in the DDP buckets, the
    # forward / input gradient / weight gradient + bias row sums on the HIP GEMMs, the weight
    # gradient written into its bucket slice; torch: DDP over the bf16 module, hipBLASLt)
    torch.manual_seed(0)
    dt = torch.bfloat16 if bf16 and device.type == "cuda" else torch.float32
    m = torch.nn.Linear(dim, dim).to(device, dt)
    model = _nbd_wrap(m, impl, **({"flat_params": True, "grad_mode": "bucket"} if bf16 and impl == "nbd" else {}))
    opt = torch.optim.SGD(m.parameters(), lr=1e-3)
    x = torch.randn(rows, dim, device=device).to(dt)
    def step():
        loss = model(x).square().mean()
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss.detach()
    ms, loss = _nbd_time_steps(step, steps, warm)
    del model, opt, m, x
    if device.type == "cuda":
        torch.cuda.empty_cache()
    return ms, loss
"""


def _echo(d) -> str:
    return d.get("echo") or d["output"].strip().splitlines()[-1]  # echo = the last expression only


def _max_over_ranks(res) -> float:
    return max(float(_echo(res.results[r]).strip("()").split(",")[0]) for r in res.ranks)


def _replay_detail(res) -> Optional[Dict[str, Any]]:
    """The per-replay HIP-event record (``_nbd_time_steps(per_step=True)``) of the slowest rank,
    or None (eager arms, CPU)."""
    import ast

    best = None
    for r in res.ranks:
        try:
            t = ast.literal_eval(_echo(res.results[r]))
        except (ValueError, SyntaxError):
            continue
        if isinstance(t, tuple) and len(t) >= 3 and isinstance(t[2], dict) and (best is None or t[0] > best[0]):
            best = (t[0], dict(t[2], rank=r))
    return None if best is None else best[1]


def _err(e: BaseException) -> str:
    if hasattr(e, "result") and e.args:  # DistributedExecutionError: its str() holds every traceback
        return f"{type(e).__name__}: {e.args[0]}"[:800]
    return f"{type(e).__name__}: {e}"[:800]


def _rank_tracebacks(e: BaseException) -> Optional[Dict[str, str]]:
    """Per-rank tail of the first exception of a failed cell (ranks that died: why), so an arm
    that can only fail at N > 1 is diagnosable from the result line alone."""
    res = getattr(e, "result", None)
    if res is None:
        return None
    out = {}
    for r, info in sorted(getattr(res, "errors", {}).items()):
        tb = (info.get("traceback") or "").rstrip() or str(info.get("error"))
        out[str(r)] = tb[-700:]
    for r, why in sorted(getattr(res, "dead", {}).items()):
        out[str(r)] = f"died: {why}"
    return out or None


def _record_error(dst: Dict[str, Any], key: str, e: BaseException) -> None:
    dst[key] = _err(e)
    tbs = _rank_tracebacks(e)
    if tbs:
        dst[key + "_rank_tracebacks"] = tbs


_ARM_T0 = [time.monotonic()]  # run_all's start: arm start offsets are relative to it


def _arm_start(out: Dict[str, Any], arm: str) -> None:
    out.setdefault("arm_start_s", {})[arm] = round(time.monotonic() - _ARM_T0[0], 2)
    _log(f"  arm {arm} starts")  # (a progress line per arm: long multi-rank arms are not silent)


def _graph_arms(n: int) -> bool:
    """Graphed arms at this world size: always at N = 1; at N > 1 unless NBD_BENCH_GRAPH_MULTI=0
    (RCCL inside the captured step is exercised at world 1 with real collectives, the
    ``collective_path`` arms; the graphed arms run after the eager ones and results are kept
    arm by arm, so a capture problem at N > 1 cannot cost the measured numbers)."""
    return n == 1 or os.environ.get("NBD_BENCH_GRAPH_MULTI", "1") != "0"


def bench_ddp(session, steps: int = 20, warmup: int = 5, B: int = 8, T: int = 1024, compare_torch: bool = True,
              linear_rows: int = 8192, config: str = "small", linear_dim: int = 4096,
              force_collectives: bool = True, out: Optional[Dict[str, Any]] = None, tick=None,
              graph: Optional[bool] = None) -> Dict[str, Any]:
    """BASELINE configs 4 and 5 as notebook cells: DDP steps timed inside each worker (max over
    ranks).  ``graph`` (default: ``_graph_arms``) runs the whole-step graph arm here; run_all
    defers it at N > 1 (``bench_ddp_graph``) until every eager arm is measured.  GPT-2 small, synthetic tokens.  Primary number: bf16 parameters living in the DDP
    buckets, fp32 master weights and moments in ``FlatAdamW`` (fused HIP AdamW per bucket).  Also
    reported: fp32 params + bf16 autocast + torch fused AdamW through nbd DDP (``amp_*``) and
    through torch DDP (``torch_ddp_*``).  ``out`` is filled arm by arm (``tick()`` after each), so
    a later arm that fails or times out leaves the earlier ones measured."""
    n = session.world_size
    out = {} if out is None else out
    tick = tick or (lambda: None)
    session.execute(AR_SETUP, render=False)
    session.execute(DDP_SETUP, render=False)
    out.update({"model": f"gpt2-{config}", "per_gpu_batch": B, "seq_len": T, "global_batch": B * n, "steps": steps,
                "warmup": warmup})
    # primary: bf16 params re-homed into the DDP buckets + FlatAdamW (fp32 master/moments, one
    # fused HIP kernel per bucket reading the all-reduced bucket); secondary: fp32 params +
    # autocast + torch fused AdamW through nbd DDP (bf16 wire)
    _arm_start(out, "flat")
    r = session.execute(f"_nbd_gpt2_bench({steps}, {warmup}, {B}, {T}, 'flat', {config!r})", render=False)
    ms = _max_over_ranks(r)
    toks = n * B * T / (ms / 1e3)
    out.update(recipe="bf16 params + fp32 master weights/moments (FlatAdamW), bf16 grad all_reduce",
               ms_per_step=ms, tokens_per_s=toks, tokens_per_s_per_gpu=toks / n)
    if config == "small":  # 6·N·tokens FLOPs over the 2.5 PFLOP/s dense bf16 peak per GPU
        out["mfu"] = 6 * 124_439_808 * toks / (2.5e15 * n)
    tick()
    try:  # ZeRO-2: reduce-scattered gradients, optimizer on this rank's slice, parameter all-gather
        _arm_start(out, "zero2")
        r = session.execute(f"_nbd_gpt2_bench({steps}, {warmup}, {B}, {T}, 'zero', {config!r})", render=False)
        zms = _max_over_ranks(r)
        out.update(zero2_ms_per_step=zms, zero2_tokens_per_s=n * B * T / (zms / 1e3),
                   zero2_recipe="as the primary recipe with DistributedDataParallel(shard=True) (ZeRO-2)")
    except Exception as e:  # noqa: BLE001 - recorded, the other recipes still run
        _record_error(out, "zero2_error", e)
        if isinstance(e, TimeoutError):
            raise
    tick()
    r = session.execute(f"_nbd_gpt2_bench({steps}, {warmup}, {B}, {T}, 'nbd', {config!r})", render=False)
    ams = _max_over_ranks(r)
    out.update(amp_ms_per_step=ams, amp_tokens_per_s=n * B * T / (ams / 1e3))
    if compare_torch:
        r = session.execute(f"_nbd_gpt2_bench({steps}, {warmup}, {B}, {T}, 'torch', {config!r})", render=False)
        tms = _max_over_ranks(r)
        # like for like: both fp32 params + bf16 autocast + torch fused AdamW, only the DDP differs
        out.update(torch_ddp_ms_per_step=tms, torch_ddp_tokens_per_s=n * B * T / (tms / 1e3),
                   speedup_vs_torch_ddp=tms / ams,
                   speedup_vs_torch_ddp_note="amp_ms_per_step vs torch_ddp_ms_per_step (same recipe)",
                   recipe_speedup_vs_torch_ddp=tms / ms)
    tick()
    r = session.execute(f"_nbd_linear_bench({steps}, {warmup}, {linear_rows}, 'nbd', {linear_dim})", render=False)
    lin = {"rows": linear_rows, "dim": linear_dim, "ms_per_step": _max_over_ranks(r)}
    out["linear4096"] = lin
    if compare_torch:
        r = session.execute(f"_nbd_linear_bench({steps}, {warmup}, {linear_rows}, 'torch', {linear_dim})", render=False)
        lin["torch_ddp_ms_per_step"] = _max_over_ranks(r)
    lin["recipe"] = "fp32 Linear (the reference README's module as written), SGD; both arms' GEMMs on hipBLASLt"
    # the same step in bf16: the module on the HIP GEMMs (no library GEMM) against torch DDP on hipBLASLt
    r = session.execute(f"_nbd_linear_bench({steps}, {warmup}, {linear_rows}, 'nbd', {linear_dim}, bf16=True)",
                        render=False)
    lb = {"ms_per_step": _max_over_ranks(r),
          "recipe": "bf16 Linear, SGD; nbd: flat bf16 params in DDP buckets, HIP GEMMs (bias add and bias-gradient "
                    "row sums fused, weight gradient written into its bucket slice); torch: DDP, hipBLASLt"}
    if compare_torch:
        r = session.execute(f"_nbd_linear_bench({steps}, {warmup}, {linear_rows}, 'torch', {linear_dim}, bf16=True)",
                            render=False)
        lb["torch_ddp_ms_per_step"] = _max_over_ranks(r)
        lb["speedup_vs_torch_ddp"] = lb["torch_ddp_ms_per_step"] / lb["ms_per_step"]
    lin["bf16"] = lb
    tick()
    if _graph_arms(n) if graph is None else graph:
        bench_ddp_graph(session, out, steps, warmup, B, T, config)
        tick()
    if n == 1 and force_collectives:
        # the world > 1 code path on this one GPU: every bucket's all-reduce (reduce-scatter +
        # all-gather for ZeRO-2) issued on RCCL from the DDP side stream / inside the graph, with
        # the per-bucket flushes and events of a multi-GPU run — what an N-GPU rank executes
        cp: Dict[str, Any] = {"note": "NBD_DDP_FORCE_COLLECTIVES semantics at world size 1: real RCCL "
                                      "collectives per bucket (a one-rank ring moves no bytes)"}
        out["collective_path"] = cp
        for key, impl in (("ms_per_step", "flat"), ("graph_ms_per_step", "flatgraph"), ("zero2_ms_per_step", "zero")):
            try:
                _arm_start(cp, key)
                r = session.execute(f"_nbd_gpt2_bench({steps}, {warmup}, {B}, {T}, {impl!r}, {config!r}, force=True)",
                                    render=False)
                cp[key] = _max_over_ranks(r)
                rd = _replay_detail(r)
                if rd:
                    cp[key.replace("ms_per_step", "replays")] = rd
            except Exception as e:  # noqa: BLE001 - recorded, the other arms still run
                _record_error(cp, key.replace("ms_per_step", "error"), e)
                if isinstance(e, TimeoutError):
                    raise
            tick()
        if "ms_per_step" in cp:
            cp["vs_no_collectives"] = cp["ms_per_step"] / ms
    return out


def bench_ddp_graph(session, out: Dict[str, Any], steps: int = 20, warmup: int = 5, B: int = 8, T: int = 1024,
                    config: str = "small") -> None:
    """The GPT-2 DDP step as one HIP graph (GraphedStep) into ``out`` (bench_ddp's dict)."""
    n = session.world_size
    try:
        _arm_start(out, "graph")
        r = session.execute(f"_nbd_gpt2_bench({steps}, {warmup}, {B}, {T}, 'flatgraph', {config!r})", render=False)
        gms = _max_over_ranks(r)
        out.update(graph_ms_per_step=gms, graph_tokens_per_s=n * B * T / (gms / 1e3),
                   graph_recipe="as the primary recipe, whole step captured in one HIP graph (GraphedStep)")
        rd = _replay_detail(r)
        if rd:
            out["graph_replays"] = rd
    except Exception as e:  # noqa: BLE001
        _record_error(out, "graph_error", e)
        if isinstance(e, TimeoutError):
            raise
    if "graph_error" in out:
        # a failed capture can leave a backend's own streams capturing (gloo's, in the one-GPU
        # N = 2 rehearsal): a second capture in the same workers would only fail the same way
        out["graph_lmhead_lib_error"] = "skipped: the graph arm failed"
    elif bool(session.ready.get(0, {}).get("cuda_available")):
        # the same graphed step with the LM head's three GEMMs all on hipBLASLt, and all on the
        # hand-written kernels, for comparison with the default per-product plan
        # (ops.loss.HEAD_PRODUCTS: weight gradient hand-written, forward / input gradient library)
        out["graph_lmhead_plan"] = "per-product (ops.loss.HEAD_PRODUCTS): " + session.execute(
            "import nbdistributed_amd.ops.loss as _lm2; str(_lm2.HEAD_PRODUCTS if _lm2.LM_HEAD_HIP else 'library')",
            render=False).results[0].get("echo", "")
        for key, kw, recipe in (("graph_lmhead_lib", "lmhead_lib=True",
                                 "as graph, the LM head's forward / input- / weight-gradient GEMMs all on hipBLASLt "
                                 "(NBD_LMHEAD_HIP=0)"),
                                ("graph_lmhead_hip", "lmhead_hip=True",
                                 "as graph, the LM head's three GEMMs all on the hand-written 256x256 kernel "
                                 "(NBD_LMHEAD_HIP=1: no library GEMM in the step)")):
            try:
                _arm_start(out, key)
                r = session.execute(f"_nbd_gpt2_bench({steps}, {warmup}, {B}, {T}, 'flatgraph', {config!r}, {kw})",
                                    render=False)
                out[key + "_ms_per_step"] = _max_over_ranks(r)
                out[key + "_recipe"] = recipe
                rd = _replay_detail(r)
                if rd:
                    out[key + "_replays"] = rd
            except Exception as e:  # noqa: BLE001
                _record_error(out, key + "_error", e)
                if isinstance(e, TimeoutError):
                    raise


def _log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _pct(xs: List[float], q: float) -> float:
    s = sorted(xs)
    if not s:
        return float("nan")
    k = min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))
    return s[k]


def bench_cells(session, steps: int, warmup: int, code: str = "1 + 1") -> Dict[str, Any]:
    for _ in range(warmup):
        session.execute(code, render=False)
    session.sync()
    lat = []
    t0 = time.perf_counter()
    for _ in range(steps):
        t = time.perf_counter()
        session.execute(code, render=False)
        lat.append(time.perf_counter() - t)
    session.sync()
    total = time.perf_counter() - t0
    ms = [x * 1e3 for x in lat]
    return {"p50_ms": statistics.median(ms), "p90_ms": _pct(ms, 0.9), "p99_ms": _pct(ms, 0.99), "min_ms": min(ms),
            "mean_ms": statistics.fmean(ms), "max_ms": max(ms), "steps": steps, "total_s": total}


def bench_cells_magic(session, steps: int, warmup: int, code: str = "1 + 1") -> Dict[str, Any]:
    """The trivial cell through the whole notebook path with default settings: a headless
    IPython-shaped shell runs the raw cell through the input transformers (auto mode rewrites it
    to ``%%distributed``), dispatches the cell magic, which runs it with the per-cell namespace
    delta on rank 0 (``ide_sync``, default on) and the per-rank renderer, and applies the delta
    as local proxies — what the reference's 111.6 ms covers (``magic.py:1042-1129``: poll loop,
    display, namespace sync).  Rendered text goes to a counting sink instead of a notebook
    frontend."""
    from .utils.fakeshell import HeadlessShell

    shell = HeadlessShell()
    rendered = [0]

    def sink(text: str) -> None:
        rendered[0] += len(text)

    prev_write = session.write
    session.write = sink
    try:
        core = shell.load_extension(session=session, writer=sink)
        core.enable_auto()
        for _ in range(warmup):
            r = shell.run_cell(code)
            if not r.success:
                raise RuntimeError(f"magic-path cell failed: {r.error_in_exec!r}")
        session.sync()
        lat = []
        for _ in range(steps):
            t = time.perf_counter()
            shell.run_cell(code)
            lat.append(time.perf_counter() - t)
        session.sync()
        core.disable_auto()
    finally:
        session.write = prev_write
    ms = [x * 1e3 for x in lat]
    return {"p50_ms": statistics.median(ms), "p90_ms": _pct(ms, 0.9), "min_ms": min(ms),
            "mean_ms": statistics.fmean(ms), "steps": steps, "ide_sync": core.ide_sync,
            "rendered_bytes": rendered[0]}


IPYTHON_PY = "/opt/conda/bin/python3.9"  # IPython 7.29, no torch: a kernel that never imports torch

IPYTHON_KERNEL = """
import io, json, statistics, sys, time
sys.path.insert(0, {root!r})
from IPython.core.interactiveshell import InteractiveShell
sh = InteractiveShell.instance()
sh.run_cell("%load_ext nbdistributed_amd")
res = {{}}
for n in {ranks!r}:
    r = sh.run_cell("%dist_init -n " + str(n) + " --backend gloo --python {py}")
    assert r.error_in_exec is None, r.error_in_exec
    real = sys.stdout
    for code, key in (("1 + 1", "auto"), ("%%distributed\\n1 + 1", "explicit"), ("%%rank [0]\\n1 + 1", "rank0")):
        lat = []
        for i in range({warm} + {steps}):
            sys.stdout = io.StringIO()     # the renderer's output, as a frontend would receive it
            t = time.perf_counter()
            r = sh.run_cell(code, store_history=True)
            dt = time.perf_counter() - t
            sys.stdout = real
            assert r.error_in_exec is None, r.error_in_exec
            if i >= {warm}:
                lat.append(dt * 1e3)
        lat.sort()
        res.setdefault(str(n), {{}})[key] = {{"p50_ms": statistics.median(lat), "p90_ms": lat[int(0.9 * (len(lat) - 1))],
                                           "min_ms": lat[0], "steps": len(lat)}}
    sh.run_cell("%dist_shutdown")
print("RESULT " + json.dumps(res))
"""


def bench_cells_ipython(ranks: List[int], steps: int = 200, warmup: int = 20, timeout_s: float = 300.0,
                        worker_python: Optional[str] = None) -> Dict[str, Any]:
    """The trivial cell through a REAL IPython ``InteractiveShell.run_cell`` (input transformers,
    auto mode -> ``%%distributed``, cell-magic dispatch, run-cell events, history) on the
    torch-less IPython interpreter, with CPU/gloo workers of the PyTorch interpreter — the control
    plane as a Jupyter kernel drives it (the GPU plays no part in a trivial cell's round trip).
    Returns {ranks: {auto|explicit|rank0: {p50_ms, ...}}}; raises if no IPython is installed."""
    import json as _json
    import subprocess
    import textwrap

    if not os.path.exists(IPYTHON_PY):
        raise FileNotFoundError(f"no IPython interpreter at {IPYTHON_PY}")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent(IPYTHON_KERNEL.format(root=root, ranks=list(ranks), py=worker_python or sys.executable,
                                                 warm=warmup, steps=steps))
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "PYTHONHOME")}
    p = subprocess.run([IPYTHON_PY, "-c", code], capture_output=True, text=True, env=env, timeout=timeout_s)
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
    if p.returncode != 0 or not line:
        raise RuntimeError(f"real-IPython cell bench failed ({p.returncode}): {(p.stdout + p.stderr)[-600:]}")
    return _json.loads(line[0][7:])


WORLD_CHECK = "(dist.get_world_size(), dist.get_backend(), rank)"


def bench_world(session) -> Dict[str, Any]:
    """What every worker's process group says: proves that RCCL saw N ranks in an N-GPU run."""
    res = session.execute(WORLD_CHECK, render=False)
    per = {}
    for r in res.ranks:
        d = res.results[r]
        out = (d.get("echo") or d.get("output") or "").strip().splitlines()[-1]
        ws, be, rk = out.strip("()").split(",")
        per[r] = {"world_size": int(ws), "backend": be.strip().strip("'\""), "rank": int(rk)}
    return {"per_rank": per, "world_sizes": sorted({v["world_size"] for v in per.values()}),
            "backends": sorted({v["backend"] for v in per.values()})}


def bench_allreduce(session, nbytes: int = 1 << 30, dtype: str = "bfloat16", iters: int = 20, warm: int = 5) -> Dict[str, Any]:
    n = session.world_size
    elem = 2 if dtype in ("bfloat16", "float16") else 4
    numel = nbytes // elem
    session.execute(AR_SETUP, render=False)
    ok = session.execute("_nbd_ar_check()", render=False)
    correct = all(ok.results[r].get("output") == "True" for r in ok.ranks)
    t = time.perf_counter()
    res = session.execute(f"_nbd_ar_time({numel}, torch.{dtype}, {iters}, {warm})", render=False)
    cell_s = time.perf_counter() - t
    per_rank = {r: float(res.results[r]["output"]) for r in res.ranks}
    t_ms = max(per_rank.values())
    # at n = 1 an all_reduce moves nothing (≈10 µs whatever the size): no bandwidth to report
    algbw = nbytes / (t_ms * 1e-3) / 1e9 if n > 1 else None
    busbw = algbw * 2 * (n - 1) / n if n > 1 else None
    return {"bytes": nbytes, "dtype": dtype, "iters": iters, "time_ms": t_ms, "per_rank_ms": per_rank,
            "algbw_GBps": algbw, "busbw_GBps": busbw, "cell_s": cell_s, "correct": correct}


def bench_sweep(session, dtype: str = "bfloat16", max_bytes: int = 1 << 30, min_bytes: int = 1024) -> List[Dict[str, Any]]:
    out = []
    b = min_bytes
    while b <= max_bytes:
        iters = 50 if b <= (16 << 20) else 20
        r = bench_allreduce(session, b, dtype, iters=iters, warm=5)
        out.append({"bytes": r["bytes"], "time_ms": round(r["time_ms"], 5),
                    "algbw_GBps": None if r["algbw_GBps"] is None else round(r["algbw_GBps"], 2),
                    "busbw_GBps": None if r["busbw_GBps"] is None else round(r["busbw_GBps"], 2)})
        b *= 4
    return out


NOTEBOOK_SETUP = """
def _nbd_notebook_bench(steps, warm, bs=16, seq=128, mode="reference", small=False, force=False):
    # the reference notebook's training loop (00_accelerate.ipynb exec 22-35): SmolLM2-135M
    # sequence classifier, AdamW lr 2e-5 + linear warmup, bs 16/rank, max_length 128, through
    # accelerate -> DDP.  Random init + synthetic MRPC-shaped batches (no network here).
    import gc
    from torch.utils.data import DataLoader, TensorDataset
    from transformers import get_linear_schedule_with_warmup
    from nbdistributed_amd.models import smollm2_135m_classifier, synthetic_mrpc
    torch.manual_seed(42)
    over = dict(num_hidden_layers=2, hidden_size=64, intermediate_size=128, num_attention_heads=4,
                num_key_value_heads=2, vocab_size=512) if small else {}
    n = bs * world_size * (steps + warm + 2)
    ids, mask, labels = synthetic_mrpc(n=n, seq_len=seq, vocab=over.get("vocab_size", 49152))
    model = smollm2_135m_classifier(**over)
    if mode in ("reference", "reference_native"):  # the notebook's loop: accelerate-prepared torch DDP
        from accelerate import Accelerator
        if mode == "reference_native":  # + the one-line swap: native Llama, fp32 master, bf16 compute
            from nbdistributed_amd.models import native
            model = native(model.to(device))
        acc = Accelerator(cpu=device.type == "cpu")
        opt = torch.optim.AdamW(model.parameters(), lr=2e-5)
        dl = DataLoader(TensorDataset(ids, mask, labels), batch_size=bs, shuffle=True)
        sched = get_linear_schedule_with_warmup(opt, 100, 3 * len(dl))
        model, opt, dl, sched = acc.prepare(model, opt, dl, sched)
        it = iter(dl)
        def step():
            x, m, y = next(it)
            out = model(input_ids=x, attention_mask=m, labels=y)
            acc.backward(out.loss)
            opt.step(); sched.step(); opt.zero_grad()
            return out.loss.detach()
    else:  # nbd: native Llama (HIP kernels), bf16 params in DDP buckets + FlatAdamW (fp32 master)
        from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification
        del model
        lc = LlamaConfig.smollm2_135m(**({k: v for k, v in over.items()} if small else {}))
        model = _NbdDDP(LlamaForSequenceClassification(lc).to(
            device, torch.bfloat16 if device.type == "cuda" else torch.float32), flat_params=True, grad_mode="bucket",
            force_collectives=bool(force))
        graph = mode == "nbd_graph"
        blockg = mode == "nbd_block_graphs" and device.type == "cuda"
        if blockg:  # eager, each decoder block's forward replayed from its own HIP graph
            from nbdistributed_amd import ops as _ops
            _prev_bg = _ops.block_graphs(1)
        # eager: each bucket updated during backward (FlatAdamW(overlap=True): this step is
        # host-bound, the GPU has room for the update; with collectives as soon as the bucket's
        # all-reduce has landed; never inside a graph)
        # (block graphs: the update after backward — measured faster than the side-stream overlap
        # with them, docs/FINDINGS.md §30)
        opt = _FlatAdamW(model, lr=2e-5, capturable=graph, overlap=not graph and not blockg)
        sched = get_linear_schedule_with_warmup(opt, 100, 3 * (n // (bs * world_size)))
        sl = slice(rank * (n // world_size), (rank + 1) * (n // world_size))
        ids, mask, labels = ids[sl].to(device), mask[sl].to(device), labels[sl].to(device)
        pos = [0]
        def train(x, mk, y):
            loss = model(x, mk, y)[0]
            loss.backward()
            opt.step(); opt.zero_grad()
            return loss.detach()
        run = train
        if graph:   # the whole step (fwd, bwd, bucket all-reduce, optimizer) as one HIP graph
            from nbdistributed_amd.graphs import GraphedStep
            run = GraphedStep(train, (ids[:bs], mask[:bs], labels[:bs]), warmup=3, optimizers=[opt])
        def step():
            i = pos[0] % (ids.shape[0] - bs); pos[0] += bs
            out = run(ids[i:i + bs], mask[i:i + bs], labels[i:i + bs])
            sched.step()
            return out
    try:
        res = _nbd_time_steps(step, steps, warm, per_step=mode in ("nbd_graph", "nbd_block_graphs"))
    finally:
        if mode == "nbd_block_graphs" and device.type == "cuda":
            _ops.block_graphs(_prev_bg)
    del model, opt
    gc.collect()
    if device.type == "cuda":
        torch.cuda.empty_cache()
    return res
"""

REFERENCE_NOTEBOOK_MS_PER_STEP = 126.6  # 1 epoch = 14.56 s / 115 steps, 2 GPUs


NOTEBOOK_RECIPES = {"reference": "HF model, fp32, accelerate DDP, torch AdamW (the notebook's recipe)",
                    "reference_native": "the notebook's accelerate loop unchanged except model = nbd.models.native(model): "
                                        "native Llama, fp32 master weights + torch AdamW (fused: native()'s default), bf16 "
                                        "compute on the fused HIP path, per-block forward graphs (native()'s default)",
                    "nbd": "native Llama (HIP kernels, one autograd node per block), bf16 params + fp32 master "
                            "(FlatAdamW, buckets updated during backward at world 1), nbd DDP",
                    "nbd_block_graphs": "as nbd (eager), each decoder block's forward replayed from its own HIP graph "
                                        "(ops.block_graphs(1)); FlatAdamW update after backward (no overlap)",
                    "nbd_graph": "as nbd, whole step captured in one HIP graph (GraphedStep)"}


def bench_notebook(session, steps: int = 20, warmup: int = 5, small: bool = False,
                   force_collectives: bool = True, out: Optional[Dict[str, Any]] = None, tick=None,
                   graph: Optional[bool] = None) -> Dict[str, Any]:
    """The reference's own measured workload (SmolLM2-135M-cls fine-tune, 126.6
    ms/step, ≈252 samples/s on 2 GPUs) as notebook cells, max over ranks."""
    n = session.world_size
    out = {} if out is None else out
    tick = tick or (lambda: None)
    session.execute(AR_SETUP, render=False)
    session.execute(DDP_SETUP, render=False)
    session.execute(NOTEBOOK_SETUP, render=False)
    out.update({"model": "SmolLM2-135M sequence classifier (random init)", "per_gpu_batch": 16,
                "seq_len": 128, "data": "synthetic MRPC-shaped",
                "reference_ms_per_step": REFERENCE_NOTEBOOK_MS_PER_STEP,
                "reference_samples_per_s": 32 / (REFERENCE_NOTEBOOK_MS_PER_STEP / 1e3)})
    modes = ["reference", "reference_native", "nbd"]
    if n == 1:  # (the per-block graph arm: an eager-step variant, timed where the GPU is ours alone)
        modes.append("nbd_block_graphs")
    if _graph_arms(n) if graph is None else graph:  # last of the main arms (bench_ddp's _graph_arms note)
        modes.append("nbd_graph")
    _notebook_arms(session, out, modes, steps, warmup, small, tick)
    if n == 1 and force_collectives:  # the N-GPU code path on one GPU (see bench_ddp)
        for mode, base in (("nbd_collective_path", "nbd"), ("nbd_graph_collective_path", "nbd_graph")):
            if "ms_per_step" not in out.get(base, {}):
                continue
            try:
                _arm_start(out, mode)
                r = session.execute(f"_nbd_notebook_bench({steps}, {warmup}, mode={base!r}, small={small}, force=True)",
                                    render=False)
                ms = _max_over_ranks(r)
                out[mode] = {"ms_per_step": ms, "vs_no_collectives": ms / out[base]["ms_per_step"],
                             "recipe": NOTEBOOK_RECIPES[base] + "; real RCCL collectives per bucket (forced at world size 1)"}
                rd = _replay_detail(r)
                if rd:
                    out[mode]["replays"] = rd
            except Exception as e:  # noqa: BLE001
                out[mode] = {}
                _record_error(out[mode], "error", e)
                if isinstance(e, TimeoutError):
                    raise
            tick()
    _notebook_summary(out)
    return out


def _notebook_arms(session, out: Dict[str, Any], modes: List[str], steps: int, warmup: int, small: bool,
                   tick) -> None:
    n = session.world_size
    for mode in modes:
        try:
            _arm_start(out, mode)
            r = session.execute(f"_nbd_notebook_bench({steps}, {warmup}, mode={mode!r}, small={small})", render=False)
        except Exception as e:  # noqa: BLE001 - recorded, the other arms still run
            out[mode] = {}
            _record_error(out[mode], "error", e)
            if isinstance(e, TimeoutError):
                raise
            continue
        ms = _max_over_ranks(r)
        _log(f"  notebook {mode}: {ms:.2f} ms/step")
        out[mode] = {"ms_per_step": ms, "samples_per_s": n * 16 / (ms / 1e3), "recipe": NOTEBOOK_RECIPES[mode]}
        rd = _replay_detail(r)
        if rd:
            out[mode]["replays"] = rd
        tick()


def bench_notebook_graph(session, out: Dict[str, Any], steps: int = 20, warmup: int = 5, small: bool = False,
                         tick=None) -> Dict[str, Any]:
    """The notebook step as one HIP graph into ``out`` (bench_notebook's dict): run_all's last
    phase at N > 1, after every eager arm."""
    _notebook_arms(session, out, ["nbd_graph"], steps, warmup, small, tick or (lambda: None))
    _notebook_summary(out)
    return out


def _notebook_summary(out: Dict[str, Any]) -> None:
    # same-recipe comparisons only: the fp32 HF arm and the bf16 native arms differ in precision
    # and model implementation, so no cross-recipe "speedup" is printed
    out["reference_vs_native_note"] = ("'reference' = HF fp32 model through accelerate (the notebook as written); "
                                       "'reference_native' = the same loop with the one-line model swap (bf16 compute, "
                                       "fp32 master weights: the recipe of Accelerator(mixed_precision='bf16')); "
                                       "'nbd*' = native bf16 Llama + FlatAdamW (bf16 params, fp32 master in the optimizer)")
    if "ms_per_step" in out.get("reference", {}) and "ms_per_step" in out.get("reference_native", {}):
        out["reference_native_speedup_same_loop"] = out["reference"]["ms_per_step"] / out["reference_native"]["ms_per_step"]
    # the eager loop against the whole-step graph (same recipe): plain, and with block/stack graphs
    g = out.get("nbd_graph", {}).get("ms_per_step")
    if g:
        for k in ("nbd", "nbd_block_graphs"):
            if "ms_per_step" in out.get(k, {}):
                out[f"{k}_vs_graph"] = out[k]["ms_per_step"] / g


BCAST_BUILD = """
model = torch.nn.Linear({dim}, {dim}, device=device)   # %%rank[0]: only rank 0 builds (random init)
"""

BCAST_RECV = """
model = torch.nn.Linear({dim}, {dim}, device="meta").to_empty(device=device)  # receivers: storage only
"""

BCAST_CELL = """
def _nbd_bcast_bench(iters, warm, coalesced):
    from nbdistributed_amd.parallel import broadcast_params
    def one():
        if coalesced:
            broadcast_params(model, src=0)
        else:
            for p in model.parameters():      # the reference README pattern (README.md:115-125)
                dist.broadcast(p.data, src=0)
    for _ in range(warm):
        one()
    _nbd_barrier()
    t = _t.perf_counter()
    for _ in range(iters):
        one()
    _nbd_sync()
    return (_t.perf_counter() - t) / iters * 1e3
"""


def bench_rank_broadcast(session, dim: int = 4096, iters: int = 20, warm: int = 3) -> Dict[str, Any]:
    """BASELINE config 3: ``%%rank[0]`` builds ``nn.Linear(dim, dim)``, then a ``%%distributed``
    cell broadcasts its parameters to every rank (per-parameter loop as in the reference README,
    and the coalesced ``broadcast_params``).  Reports the cell round-trips and in-worker times."""
    n = session.world_size
    session.execute(AR_SETUP, render=False)
    session.execute("import time as _t", render=False)
    t = time.perf_counter()
    session.execute(BCAST_BUILD.format(dim=dim), ranks=[0], render=False)
    build_ms = (time.perf_counter() - t) * 1e3
    if n > 1:
        session.execute(BCAST_RECV.format(dim=dim), ranks=list(range(1, n)), render=False)
    session.execute(BCAST_CELL, render=False)
    t = time.perf_counter()
    session.execute("for p in model.parameters():\n    dist.broadcast(p.data, src=0)\n_nbd_sync()", render=False)
    first_cell_ms = (time.perf_counter() - t) * 1e3
    chk = session.execute("w = model.weight.detach().float(); t = torch.stack([w.sum(), w.square().sum()])\n"
                          "ref = t.clone(); dist.broadcast(ref, src=0); bool(torch.equal(t, ref))", render=False)
    correct = all(chk.results[r].get("output") == "True" for r in chk.ranks)
    per_param = _max_over_ranks(session.execute(f"_nbd_bcast_bench({iters}, {warm}, False)", render=False))
    coalesced = _max_over_ranks(session.execute(f"_nbd_bcast_bench({iters}, {warm}, True)", render=False))
    nbytes = (dim * dim + dim) * 4
    session.execute("del model", render=False)
    bw = (lambda ms: nbytes / (ms * 1e-3) / 1e9) if n > 1 else (lambda ms: None)  # n = 1: a no-op
    return {"dim": dim, "bytes": nbytes, "build_cell_ms": build_ms, "broadcast_cell_ms": first_cell_ms,
            "per_param_ms": per_param, "coalesced_ms": coalesced,
            "per_param_GBps": bw(per_param), "coalesced_GBps": bw(coalesced), "correct": correct}


def _phase(session, out: Dict[str, Any], name: str, fn, timeout_s: float, deadline: Optional[float] = None,
           min_s: float = 0.0) -> None:
    """Run one optional benchmark phase; failures are recorded in ``out[name]`` instead of
    losing the whole result line.  A timeout means ranks are stuck (e.g. inside a collective):
    interrupt them (out-of-band SIGINT; the worker watchdog aborts the RCCL communicator) and
    skip the remaining phases.  ``deadline`` (time.monotonic()): the bench's global budget —
    a phase that would start with less than ``min_s`` left is skipped, and no request of a
    running phase waits past it (``Session.deadline``)."""
    if out.get("aborted"):
        out[name] = {"skipped": "an earlier phase timed out"}
        return
    if deadline is not None and deadline - time.monotonic() < min_s:
        out[name] = {"skipped": "bench deadline reached"}
        _log(f"phase {name} skipped: bench deadline")
        return
    prev = session.default_timeout
    session.default_timeout = timeout_s
    try:
        out[name] = fn()
    except Exception as e:  # noqa: BLE001 - recorded in the result line
        part = out.get(name)
        if not (isinstance(part, dict) and part):  # arms measured before the failure stay
            part = out[name] = {}
        _record_error(part, "error", e)
        _log(f"phase {name} failed: {type(e).__name__}: {str(e)[:300]}")
        if isinstance(e, TimeoutError):
            out["aborted"] = name
            try:
                dl = getattr(session, "deadline", None)
                if dl is not None:
                    session.deadline = None  # the interrupt itself must not be cut short
                session.interrupt()
                time.sleep(session.cfg.interrupt_abort_s + 5.0)
            except Exception:  # noqa: BLE001
                pass
    finally:
        session.default_timeout = prev


# The driver allows bench.py 600 s in all (torchrun start, imports and RCCL init included): the
# phases share a global budget well inside it, and the result is checkpointed after each phase
DEFAULT_DEADLINE_S = float(os.environ.get("NBD_BENCH_DEADLINE_S", "420"))
# all-reduce size cap when the workers have no GPU (gloo on the CPU: plumbing, not bandwidth)
CPU_AR_BYTES = int(os.environ.get("NBD_BENCH_CPU_AR_BYTES", str(1 << 20)))


def run_all(session, steps: int, warmup: int, allreduce: bool = True, sweep: bool = False,
            ar_bytes: int = 1 << 30, ddp: bool = True, ddp_steps: int = 20, bcast: bool = True,
            notebook: bool = True, phase_timeout_s: float = 300.0, deadline_s: Optional[float] = None,
            checkpoint=None, checks: bool = True) -> Dict[str, Any]:
    """All phases under one global deadline (``deadline_s`` from now, default
    ``NBD_BENCH_DEADLINE_S`` = 420 s); ``checkpoint(out)`` is called after every phase so the
    caller can persist what has been measured (bench.py writes it where rank 0 reads it, even if
    a later phase hangs)."""
    n = session.world_size
    _ARM_T0[0] = time.monotonic()
    deadline = time.monotonic() + (DEFAULT_DEADLINE_S if deadline_s is None else deadline_s)
    prev_deadline = getattr(session, "deadline", None)
    session.deadline = deadline

    def ckpt(out):
        if checkpoint is not None:
            try:
                checkpoint(out)
            except Exception as e:  # noqa: BLE001
                _log(f"checkpoint failed: {e}")

    try:
        _log(f"phase 1: {warmup}+{steps} trivial %%distributed cells on {n} rank(s)")
        cells = bench_cells(session, steps, warmup)
        _log(f"cell p50 {cells['p50_ms']:.3f} ms")
        out: Dict[str, Any] = {"cell": cells}
        ckpt(out)
        _phase(session, out, "world", lambda: bench_world(session), phase_timeout_s, deadline)
        _log(f"phase 1b: {warmup}+{steps} trivial cells through the magic path (auto mode, ide_sync, renderer)")
        _phase(session, out, "cell_magic", lambda: bench_cells_magic(session, steps, warmup), phase_timeout_s, deadline)
        if "p50_ms" in out["cell_magic"]:
            _log(f"magic-path cell p50 {out['cell_magic']['p50_ms']:.3f} ms")
        ckpt(out)
        if os.path.exists(IPYTHON_PY) and os.environ.get("NBD_BENCH_IPYTHON", "1") != "0":
            _log(f"phase 1c: trivial cells through a real IPython kernel ({n} gloo worker(s))")
            _phase(session, out, "cell_ipython",
                   lambda: bench_cells_ipython([n], steps=max(steps, 50), warmup=warmup,
                                               timeout_s=max(30.0, min(240.0, deadline - time.monotonic() - 5.0))),
                   phase_timeout_s, deadline, 30.0)
            ci = out["cell_ipython"].get(str(n), {}).get("auto") if isinstance(out["cell_ipython"], dict) else None
            if ci:
                _log(f"real-IPython cell p50 {ci['p50_ms']:.3f} ms")
            ckpt(out)
        hang = os.environ.get("NBD_BENCH_FAULT_HANG")
        if hang:  # fault injection (tests): a cell that outlives the budget must not cost the line
            _phase(session, out, "fault_hang",
                   lambda: session.execute(f"import time as _t; _t.sleep({float(hang)})", render=False) and {},
                   phase_timeout_s, deadline)
            ckpt(out)
        gpu = bool(session.ready.get(0, {}).get("cuda_available"))
        if not gpu:  # CPU/gloo (tests, a GPU-less host): the same cells on small buffers
            ar_bytes = min(ar_bytes, CPU_AR_BYTES)
        if allreduce:
            _log(f"phase 2: {ar_bytes / 2**20:.2f} MiB bf16 all_reduce")
            _phase(session, out, "allreduce", lambda: bench_allreduce(session, ar_bytes, iters=20 if gpu else 3,
                                                                      warm=5 if gpu else 1),
                   phase_timeout_s, deadline, 10.0)
            ar = out["allreduce"]
            if "time_ms" in ar:
                _log(f"all_reduce {ar['time_ms']:.3f} ms busbw {ar['busbw_GBps']}")
            ckpt(out)
        if sweep:
            _log("phase 3: all_reduce sweep")
            _phase(session, out, "sweep", lambda: bench_sweep(session, max_bytes=1 << 30 if gpu else CPU_AR_BYTES),
                   phase_timeout_s, deadline, 20.0)
            ckpt(out)
        if bcast and gpu:
            _log("phase 3b: %%rank[0] Linear(4096) build + broadcast (config 3)")
            _phase(session, out, "rank_broadcast", lambda: bench_rank_broadcast(session), phase_timeout_s, deadline, 10.0)
            rb = out["rank_broadcast"]
            if "per_param_ms" in rb:
                _log(f"broadcast per-param {rb['per_param_ms']:.3f} ms, coalesced {rb['coalesced_ms']:.3f} ms")
            ckpt(out)
        # at N > 1 the whole-step graph arms run last, after every eager arm of both workloads: a
        # capture that fails there (a collective's unjoined side-stream work, say) must not cost
        # the measured eager numbers of the later phases
        defer_graphs = n > 1 and _graph_arms(n)
        if ddp and gpu:
            _log("phase 4: DDP steps (GPT-2 small bf16 config 5, Linear 4096 config 4)")
            out["ddp"] = {}
            _phase(session, out, "ddp", lambda: bench_ddp(session, steps=ddp_steps, out=out["ddp"], tick=lambda: ckpt(out),
                                                          graph=False if defer_graphs else None),
                   phase_timeout_s, deadline, 60.0)
            d = out["ddp"]
            if "ms_per_step" in d:
                _log(f"gpt2 ddp {d['ms_per_step']:.2f} ms/step {d['tokens_per_s']:.0f} tok/s")
            ckpt(out)
        if notebook and gpu:
            _log("phase 5: reference notebook workload (SmolLM2-135M-cls, bs16, seq128)")
            out["notebook"] = {}
            _phase(session, out, "notebook",
                   lambda: bench_notebook(session, steps=ddp_steps, out=out["notebook"], tick=lambda: ckpt(out),
                                          graph=False if defer_graphs else None),
                   phase_timeout_s, deadline, 60.0)
            nb = out["notebook"]
            if "ms_per_step" in nb.get("reference", {}) and "ms_per_step" in nb.get("nbd", {}):
                _log(f"notebook fp32 {nb['reference']['ms_per_step']:.2f} ms/step, nbd {nb['nbd']['ms_per_step']:.2f}")
            ckpt(out)
        if defer_graphs and gpu and (ddp or notebook):
            _log("phase 6: whole-step HIP graph arms (GraphedStep)")
            if ddp and isinstance(out.get("ddp"), dict) and "ms_per_step" in out["ddp"]:
                _phase(session, out, "ddp_graph", lambda: bench_ddp_graph(session, out["ddp"], steps=ddp_steps),
                       phase_timeout_s, deadline, 60.0)
                ckpt(out)
            if notebook and isinstance(out.get("notebook"), dict):
                _phase(session, out, "notebook_graph",
                       lambda: bench_notebook_graph(session, out["notebook"], steps=ddp_steps, tick=lambda: ckpt(out))
                       and None, phase_timeout_s, deadline, 60.0)
                ckpt(out)
        if checks:
            # correctness of the data plane at this world size (nbdistributed_amd.checks): every
            # collective against closed-form values, nbd DDP against torch DDP, the recipe's
            # cross-rank sync, ZeRO-2, the graphed step, accelerate, %%rank + broadcast.  Last:
            # a check that hangs (aborting the phase) must not cost the measured numbers.
            _log(f"phase 7: data-plane correctness checks on {n} rank(s)")
            from .checks import run_checks

            # (150 s per cell at most: at N = 8 the whole phase takes seconds; a hang in it ends early)
            _phase(session, out, "checks", lambda: run_checks(session, log=_log), min(phase_timeout_s, 150.0),
                   deadline, 30.0)
            ck = out["checks"]
            _log("checks: " + ("all passed" if ck.get("passed") else
                               f"NOT PASSED {ck.get('failed') or ck.get('error') or ck.get('skipped')}"))
            ckpt(out)
        return out
    finally:
        session.deadline = prev_deadline


def error_line(error: str, n: int, steps: int, warmup: int) -> Dict[str, Any]:
    """The result line when nothing could be measured (e.g. the ranks never all joined): the
    contract keys with a null value and the reason."""
    return {"metric": METRIC, "value": None, "unit": "ms", "n_gpus": n, "steps": steps, "warmup": warmup,
            "ms_per_step": None, "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": "%%distributed trivial cell (1 + 1) + 1 GiB bf16 all_reduce cell via RCCL/xGMI",
                       "global_batch": None, "seq_len": None, "parallelism": f"dp{n}"},
            "error": error}


def result_line(res: Dict[str, Any], n: int, steps: int, warmup: int) -> Dict[str, Any]:
    cells = res["cell"]
    ar = res.get("allreduce") or {}
    line = {
        "metric": METRIC,
        "value": round(cells["p50_ms"], 4),
        "unit": "ms",
        "n_gpus": n,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(cells["mean_ms"], 4),
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": round(cells["p50_ms"] / BASELINE_CELL_P50_MS, 5),
        "dtype": "bf16",
        "data": "synthetic",
        "config": {"model": "%%distributed trivial cell (1 + 1) + 1 GiB bf16 all_reduce cell via RCCL/xGMI",
                   "global_batch": None, "seq_len": None, "parallelism": f"dp{n}"},
        "cell_p50_ms": round(cells["p50_ms"], 4),
        "cell_p90_ms": round(cells["p90_ms"], 4),
        "cell_min_ms": round(cells["min_ms"], 4),
        "baseline_cell_p50_ms": BASELINE_CELL_P50_MS,
        "speedup_vs_baseline": round(BASELINE_CELL_P50_MS / cells["p50_ms"], 1),
    }
    if ar and ("error" in ar or "skipped" in ar):
        line["allreduce_error"] = ar.get("error") or ar.get("skipped")
    elif ar:
        line["allreduce_bytes"] = ar["bytes"]
        line["allreduce_time_ms"] = round(ar["time_ms"], 4)
        line["allreduce_algbw_GBps"] = None if ar["algbw_GBps"] is None else round(ar["algbw_GBps"], 2)
        if n == 1:
            line["allreduce_note"] = "world size 1: the all_reduce is a no-op, no bandwidth is reported"
        line["allreduce_busbw_GBps"] = None if ar["busbw_GBps"] is None else round(ar["busbw_GBps"], 2)
        line["allreduce_correct"] = ar["correct"]
    sw = res.get("sweep")
    if isinstance(sw, list) and sw:
        line["allreduce_sweep"] = sw
        bus = [r["busbw_GBps"] for r in sw if r.get("busbw_GBps") is not None]
        if bus:
            line["allreduce_peak_busbw_GBps"] = round(max(bus), 2)
    elif isinstance(sw, dict):
        line["allreduce_sweep_error"] = sw.get("error") or sw.get("skipped")
    cm = res.get("cell_magic") or {}
    if "p50_ms" in cm:
        line["cell_magic_p50_ms"] = round(cm["p50_ms"], 4)
        line["cell_magic_p90_ms"] = round(cm["p90_ms"], 4)
        line["cell_magic_note"] = ("raw cell -> auto-mode transformer -> %%distributed magic with ide_sync="
                                   f"{cm.get('ide_sync')} namespace delta + renderer (default settings)")
    elif cm:
        line["cell_magic_error"] = cm.get("error") or cm.get("skipped")
    ci = res.get("cell_ipython") or {}
    if isinstance(ci, dict) and str(n) in ci:
        d = ci[str(n)]
        line["cell_ipython_p50_ms"] = round(d["auto"]["p50_ms"], 4)
        line["cell_ipython_explicit_p50_ms"] = round(d["explicit"]["p50_ms"], 4)
        line["cell_ipython_rank0_p50_ms"] = round(d["rank0"]["p50_ms"], 4)
        line["cell_ipython_note"] = ("plain cell through a real IPython 7.29 InteractiveShell.run_cell (auto mode, "
                                     "ide_sync, renderer; torch-less kernel) with CPU/gloo workers: the control "
                                     "plane as a Jupyter kernel drives it")
    elif ci and ("error" in ci or "skipped" in ci):
        line["cell_ipython_error"] = ci.get("error") or ci.get("skipped")
    ck = res.get("checks")
    if isinstance(ck, dict) and ck:
        if "passed" in ck:
            line["checks_passed"] = bool(ck["passed"])
            line["checks"] = ck
        elif "skipped" in ck:  # not run (bench deadline / an earlier phase aborted): no verdict
            line["checks_passed"] = None
            line["checks"] = {"passed": None, "skipped": ck["skipped"]}
        else:  # the phase itself failed (raised or timed out): not a pass
            line["checks_passed"] = False
            line["checks"] = {"passed": False, "error": ck.get("error")}
    wd = res.get("world") or {}
    if "per_rank" in wd:
        line["rccl_world_size"] = {str(r): v["world_size"] for r, v in wd["per_rank"].items()}
        line["process_group_backend"] = wd["backends"][0] if len(wd["backends"]) == 1 else wd["backends"]
    if res.get("aborted"):
        line["aborted_phase"] = res["aborted"]
    for k in ("ddp", "rank_broadcast", "notebook"):
        if k in res:
            line[k] = res[k]
    for k in ("ddp_graph", "notebook_graph"):  # run_all's deferred graph phase (N > 1): only a failure
        if isinstance(res.get(k), dict) and res[k]:
            line[k] = res[k]
    return line
