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

import statistics
import sys
import time
from typing import Any, Dict, List, Optional

BASELINE_CELL_P50_MS = 111.6
METRIC = "all_reduce bus GB/s + %%distributed cell p50 round-trip (ms) at 1/2/4/8 MI355X"

AR_SETUP = """
import time as _t
def _nbd_ar_time(numel, dtype, iters, warm):
    x = torch.zeros(numel, dtype=dtype, device=device)
    for _ in range(warm):
        dist.all_reduce(x)
    torch.cuda.synchronize()
    dist.barrier(device_ids=[device.index]) if device.type == 'cuda' else dist.barrier()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        dist.all_reduce(x)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    del x
    return ms

def _nbd_ar_check():
    y = torch.full((1024,), float(rank + 1), dtype=torch.bfloat16, device=device)
    dist.all_reduce(y)
    want = world_size * (world_size + 1) / 2
    return bool((y.float() == want).all().item())
"""


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
    algbw = nbytes / (t_ms * 1e-3) / 1e9
    busbw = algbw * 2 * (n - 1) / n if n > 1 else None
    return {"bytes": nbytes, "dtype": dtype, "iters": iters, "time_ms": t_ms, "per_rank_ms": per_rank,
            "algbw_GBps": algbw, "busbw_GBps": busbw, "cell_s": cell_s, "correct": correct}


def bench_sweep(session, dtype: str = "bfloat16", max_bytes: int = 1 << 30, min_bytes: int = 1024) -> List[Dict[str, Any]]:
    out = []
    b = min_bytes
    while b <= max_bytes:
        iters = 50 if b <= (16 << 20) else 20
        r = bench_allreduce(session, b, dtype, iters=iters, warm=5)
        out.append({k: r[k] for k in ("bytes", "time_ms", "algbw_GBps", "busbw_GBps")})
        b *= 4
    return out


def run_all(session, steps: int, warmup: int, allreduce: bool = True, sweep: bool = False,
            ar_bytes: int = 1 << 30) -> Dict[str, Any]:
    n = session.world_size
    _log(f"phase 1: {warmup}+{steps} trivial %%distributed cells on {n} rank(s)")
    cells = bench_cells(session, steps, warmup)
    _log(f"cell p50 {cells['p50_ms']:.3f} ms")
    out: Dict[str, Any] = {"cell": cells}
    gpu = bool(session.ready.get(0, {}).get("cuda_available"))
    if allreduce and gpu:
        _log(f"phase 2: {ar_bytes / 2**30:.2f} GiB bf16 all_reduce")
        out["allreduce"] = bench_allreduce(session, ar_bytes)
        _log(f"all_reduce {out['allreduce']['time_ms']:.3f} ms busbw {out['allreduce']['busbw_GBps']}")
    if sweep and gpu:
        _log("phase 3: all_reduce sweep")
        out["sweep"] = bench_sweep(session)
    return out


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
    if ar:
        line["allreduce_bytes"] = ar["bytes"]
        line["allreduce_time_ms"] = round(ar["time_ms"], 4)
        line["allreduce_algbw_GBps"] = round(ar["algbw_GBps"], 2)
        line["allreduce_busbw_GBps"] = None if ar["busbw_GBps"] is None else round(ar["busbw_GBps"], 2)
        line["allreduce_correct"] = ar["correct"]
    if res.get("sweep"):
        line["allreduce_sweep"] = res["sweep"]
    for k in ("ddp",):
        if k in res:
            line[k] = res[k]
    return line
