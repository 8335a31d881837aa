"""Data-plane correctness checks at any world size, run as notebook cells.

The reference's core use is collectives typed into ``%%distributed`` cells across real ranks
(``/root/reference/README.md:106-124``, ``src/nbdistributed/worker.py:151``) and the 2-GPU DDP
notebook (``00_accelerate.ipynb:1089``).  A timing run at N > 1 proves nothing about those: a
collective that returns wrong bytes, a DDP that averages the wrong thing, ranks that silently
desynchronise or a captured step that replays something else all still produce a number.  These
checks run in the workers exactly as a user's cells do and compare against closed-form values
or against an independent implementation:

* ``collectives`` — ``all_reduce`` / ``broadcast`` / ``all_gather_into_tensor`` /
  ``reduce_scatter_tensor`` / ``all_to_all_single`` / ``send``+``recv`` / ``batch_isend_irecv``,
  fp32 and bf16, a small and a large message (1 KiB and 64 MiB on GPUs), against closed-form
  expected values (small integers: exact in bf16, so the comparison is bitwise);
* ``ddp`` — nbd ``DistributedDataParallel`` vs ``torch.nn.parallel.DistributedDataParallel`` on
  the same fp32 GPT-2 (tiny), the same per-rank batches and SGD: per-step losses and the total
  parameter update after 5 steps;
* ``recipe_sync`` — the bench's own recipe (bf16 params in the DDP buckets, ``FlatAdamW`` fp32
  master): after 5 steps every rank holds bit-identical parameters;
* ``zero2`` — the same recipe with ``shard=True`` (reduce-scatter, sharded optimizer,
  all-gather) against the unsharded one;
* ``adamw_overlap`` (GPU) — the recipe with ``FlatAdamW(overlap=True)`` (each bucket updated on
  a side stream once its collective has landed) bit-identical to the update after backward;
* ``graph`` (GPU) — the recipe's whole step captured as one HIP graph (``GraphedStep``, RCCL
  collectives inside the graph) against the same steps run eagerly;
* ``accelerate`` — HF ``Accelerator()`` on the framework's process group (``"rccl"`` on GPUs):
  its world / rank / device, ``gather``, and a prepared DDP step that leaves the ranks in sync;
* ``rank_broadcast`` — ``%%rank [0]`` builds a Linear, a ``%%distributed`` cell broadcasts its
  parameters (BASELINE config 3), every rank then holds rank 0's bytes.

``run_checks`` returns ``{"passed": bool, "failed": [...], "results": {...}, "detail": {...}}``;
bench.py puts it in its JSON line and exits non-zero when anything failed.
"""
from __future__ import annotations

import ast
import time
from typing import Any, Callable, Dict, List, Optional

CHECK_SETUP = r'''
import copy as _copy
import contextlib as _ctx

def _nbd_clean(d):
    # repr-safe (ast.literal_eval on the coordinator): non-finite floats as strings
    if isinstance(d, dict):
        return {k: _nbd_clean(v) for k, v in d.items()}
    if isinstance(d, (list, tuple)):
        return [_nbd_clean(v) for v in d]
    if isinstance(d, float) and (d != d or d in (float("inf"), float("-inf"))):
        return str(d)
    return d

def _nbd_pat(n, dtype, k, scale=1, offset=0):
    # small integers (exact in bf16 up to 256): ((i % k) + 1 + offset) * scale
    return (((torch.arange(n, device=device) % k) + 1 + offset) * scale).to(dtype)

def _nbd_chk_collectives(sizes, dtypes):
    W, r = world_size, rank
    res, errs = {}, {}

    def run(key, fn):
        # one collective: a raise is recorded as a failure of that op only (the others still run)
        try:
            res[key] = bool(fn())
        except Exception as e:  # noqa: BLE001
            res[key] = False
            errs[key] = (type(e).__name__ + ": " + str(e))[:300]

    for dt in dtypes:
        dtype = getattr(torch, dt)
        esz = torch.tensor([], dtype=dtype).element_size()
        for nbytes in sizes:
            tag = dt + "_" + str(nbytes)
            n = max(64 * W, nbytes // esz // (8 * W) * (8 * W))   # elements, a multiple of 8 W
            c = n // W

            def all_reduce():  # SUM: Σ_r (r + 1) · p = W(W+1)/2 · p
                x = _nbd_pat(n, dtype, 5, r + 1)
                dist.all_reduce(x)
                return torch.equal(x, _nbd_pat(n, dtype, 5, W * (W + 1) // 2))

            def broadcast():  # from the last rank (a non-zero source)
                src = W - 1
                x = _nbd_pat(n, dtype, 7, 1, r) if r == src else torch.zeros(n, dtype=dtype, device=device)
                dist.broadcast(x, src=src)
                return torch.equal(x, _nbd_pat(n, dtype, 7, 1, src))

            def all_gather():  # chunk s = (s + 1) · p
                out = torch.empty(n, dtype=dtype, device=device)
                dist.all_gather_into_tensor(out, _nbd_pat(c, dtype, 3, r + 1))
                return torch.equal(out, torch.cat([_nbd_pat(c, dtype, 3, s + 1) for s in range(W)]))

            def reduce_scatter():  # SUM: this rank's chunk of W(W+1)/2 · p
                out = torch.empty(c, dtype=dtype, device=device)
                dist.reduce_scatter_tensor(out, _nbd_pat(n, dtype, 5, r + 1))
                return torch.equal(out, _nbd_pat(n, dtype, 5, W * (W + 1) // 2)[r * c:(r + 1) * c])

            def all_to_all():  # the chunk sent to rank j is r·W + j + 1; received chunk s = s·W + r + 1
                x = torch.cat([torch.full((c,), r * W + j + 1, dtype=dtype, device=device) for j in range(W)])
                out = torch.empty(n, dtype=dtype, device=device)
                dist.all_to_all_single(out, x)
                return torch.equal(out, torch.cat([torch.full((c,), s * W + r + 1, dtype=dtype, device=device)
                                                   for s in range(W)]))

            run("all_reduce_" + tag, all_reduce)
            run("broadcast_" + tag, broadcast)
            run("all_gather_" + tag, all_gather)
            run("reduce_scatter_" + tag, reduce_scatter)
            run("all_to_all_" + tag, all_to_all)
            if W > 1:   # point to point around the ring (even ranks send first: no deadlock)
                nxt, prv = (r + 1) % W, (r - 1) % W

                def send_recv():
                    s_ = _nbd_pat(n, dtype, 7, 1, r)
                    rb = torch.zeros(n, dtype=dtype, device=device)
                    if r % 2 == 0:
                        dist.send(s_, nxt); dist.recv(rb, prv)
                    else:
                        dist.recv(rb, prv); dist.send(s_, nxt)
                    return torch.equal(rb, _nbd_pat(n, dtype, 7, 1, prv))

                def batch_p2p():  # both directions at once
                    s_ = _nbd_pat(n, dtype, 7, 1, r)
                    fw = torch.zeros(n, dtype=dtype, device=device)
                    bw = torch.zeros(n, dtype=dtype, device=device)
                    ops_ = [dist.P2POp(dist.isend, s_, nxt), dist.P2POp(dist.irecv, fw, prv),
                            dist.P2POp(dist.isend, s_, prv), dist.P2POp(dist.irecv, bw, nxt)]
                    for q in dist.batch_isend_irecv(ops_):
                        q.wait()
                    return torch.equal(fw, _nbd_pat(n, dtype, 7, 1, prv)) and torch.equal(bw, _nbd_pat(n, dtype, 7, 1, nxt))

                run("send_recv_" + tag, send_recv)
                run("batch_isend_irecv_" + tag, batch_p2p)
    if device.type == "cuda":
        torch.cuda.synchronize()
    if errs:
        res["detail"] = {"collective_errors": errs}
    return res

def _nbd_same_on_all_ranks(t):
    # every rank holds the same bytes as rank 0 (bitwise)
    ref = t.detach().clone()
    dist.broadcast(ref, src=0)
    same = torch.tensor([1 if torch.equal(ref, t) else 0], device=t.device, dtype=torch.int32)
    dist.all_reduce(same, op=dist.ReduceOp.MIN)
    return bool(same.item() == 1)

def _nbd_tiny_gpt2(dtype):
    from nbdistributed_amd.models import GPT2, GPT2Config
    torch.manual_seed(1234)   # the same initial weights on every rank
    return GPT2(GPT2Config(vocab_size=512, n_positions=64, n_embd=128, n_layer=2, n_head=2)).to(device, dtype)

def _nbd_batches(steps, B=2, T=64):
    g = torch.Generator().manual_seed(4321 + rank)   # each rank its own data, as in DDP
    return [torch.randint(0, 512, (B, T), generator=g).to(device) for _ in range(steps)]

def _nbd_chk_ddp(steps=5, lr=0.05):
    # nbd DDP vs torch DDP: same fp32 model, batches and SGD; the losses step by step and the
    # total parameter update must agree (only the gradient averaging differs between them)
    from nbdistributed_amd.parallel import DistributedDataParallel as _N
    from torch.nn.parallel import DistributedDataParallel as _T
    base = _nbd_tiny_gpt2(torch.float32)
    p0 = [p.detach().clone() for p in base.parameters()]
    a = _N(_copy.deepcopy(base), bucket_cap_mb=0.25, first_bucket_mb=0.05)
    b = _T(_copy.deepcopy(base), device_ids=[device.index] if device.type == "cuda" else None, bucket_cap_mb=0.25)
    oa = torch.optim.SGD(a.module.parameters(), lr=lr)
    ob = torch.optim.SGD(b.module.parameters(), lr=lr)
    la, lb = [], []
    for x in _nbd_batches(steps):
        for m, o, l in ((a, oa, la), (b, ob, lb)):
            o.zero_grad(set_to_none=True)
            _, loss = m(x, x, return_logits=False)
            loss.backward()
            o.step()
            l.append(float(loss.detach()))
    loss_rel = max(abs(u - v) / max(1e-6, abs(v)) for u, v in zip(la, lb))
    du = torch.cat([(p.detach() - q).reshape(-1) for p, q in zip(a.module.parameters(), p0)])
    dv = torch.cat([(p.detach() - q).reshape(-1) for p, q in zip(b.module.parameters(), p0)])
    upd_rel = float((du - dv).abs().max() / dv.abs().max().clamp_min(1e-12))
    in_sync = _nbd_same_on_all_ranks(torch.cat([p.detach().reshape(-1) for p in a.module.parameters()]))
    del a, b, oa, ob, base
    return {"ddp_vs_torch": loss_rel < 1e-4 and upd_rel < 1e-3 and in_sync,
            "detail": {"loss_rel": loss_rel, "update_rel": upd_rel, "in_sync": in_sync, "losses": la[:2] + la[-1:]}}

def _nbd_recipe(shard, capturable=False, overlap=False):
    from nbdistributed_amd.parallel import DistributedDataParallel as _N
    from nbdistributed_amd.optim import FlatAdamW as _F
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    m = _N(_nbd_tiny_gpt2(dtype), flat_params=True, grad_mode="bucket", shard=shard,
           bucket_cap_mb=0.25, first_bucket_mb=0.05)
    return m, _F(m, lr=1e-3, capturable=capturable, overlap=overlap)

def _nbd_recipe_step(m, o, x):
    _, loss = m(x, x, return_logits=False)
    loss.backward()
    o.step()
    o.zero_grad(set_to_none=True)
    return loss.detach()

def _nbd_flat_params(m):
    if getattr(m, "shard", False):
        m.wait_params()
    return torch.cat([p.detach().float().reshape(-1) for p in m.module.parameters()])

def _nbd_chk_recipe(steps=5):
    # the bench recipe (bf16 bucket params + FlatAdamW) keeps every rank bit-identical; ZeRO-2
    # (reduce-scatter + sharded update + all-gather) trains like the unsharded recipe
    full, of = _nbd_recipe(False)
    zero, oz = _nbd_recipe(True)
    lf, lz = [], []
    for x in _nbd_batches(steps):
        lf.append(float(_nbd_recipe_step(full, of, x)))
        lz.append(float(_nbd_recipe_step(zero, oz, x)))
    pf, pz = _nbd_flat_params(full), _nbd_flat_params(zero)
    tol = 2e-2 if pf.dtype != torch.float32 and device.type == "cuda" else 1e-5
    err = float((pf - pz).abs().max() / pf.abs().max().clamp_min(1e-12))
    loss_rel = max(abs(u - v) / max(1e-6, abs(v)) for u, v in zip(lf, lz))
    sync_full = _nbd_same_on_all_ranks(pf)
    sync_zero = _nbd_same_on_all_ranks(pz)
    del zero, oz
    res = {"recipe_sync": sync_full, "zero2": err <= tol and loss_rel <= 1e-2 and sync_zero,
           "detail": {"zero2_param_rel": err, "zero2_loss_rel": loss_rel, "zero2_in_sync": sync_zero,
                      "losses": lf[:2] + lf[-1:]}}
    if device.type == "cuda":
        # FlatAdamW(overlap=True): each bucket updated on a side stream once its collective has
        # landed (DDP's per-bucket event), during backward — bit-identical to the update after it
        ov, oo = _nbd_recipe(False, overlap=True)
        lo = [float(_nbd_recipe_step(ov, oo, x)) for x in _nbd_batches(steps)]
        po = _nbd_flat_params(ov)
        res["adamw_overlap"] = bool(torch.equal(po, pf)) and lo == lf
        res["detail"]["adamw_overlap_param_maxdiff"] = float((po - pf).abs().max())
        del ov, oo
    del full, of
    return res

def _nbd_chk_graph(warm=3, replays=3):
    # the recipe's whole step as one HIP graph (RCCL collectives captured) vs the same steps eagerly
    from nbdistributed_amd.graphs import GraphedStep
    xs = _nbd_batches(1)
    x = xs[0]
    me, oe = _nbd_recipe(False)
    le = [float(_nbd_recipe_step(me, oe, x)) for _ in range(warm + replays)]
    mg, og = _nbd_recipe(False, capturable=True)
    g = GraphedStep(lambda inp: _nbd_recipe_step(mg, og, inp), (x,), warmup=warm, optimizers=[og])
    lg = [float(g(x)) for _ in range(replays)]
    torch.cuda.synchronize()
    pe, pg_ = _nbd_flat_params(me), _nbd_flat_params(mg)
    err = float((pe - pg_).abs().max() / pe.abs().max().clamp_min(1e-12))
    loss_rel = max(abs(u - v) / max(1e-6, abs(v)) for u, v in zip(le[warm:], lg))
    in_sync = _nbd_same_on_all_ranks(pg_)
    del g, me, mg, oe, og
    torch.cuda.empty_cache()
    return {"graph": err <= 2e-2 and loss_rel <= 1e-2 and in_sync,
            "detail": {"graph_param_rel": err, "graph_loss_rel": loss_rel, "graph_in_sync": in_sync}}

def _nbd_chk_accelerate():
    from accelerate import Accelerator
    from accelerate.utils import DistributedType as _DT
    acc = Accelerator(cpu=device.type == "cpu")
    st = acc.state
    want = (_DT.MULTI_GPU if device.type == "cuda" else _DT.MULTI_CPU) if world_size > 1 else None
    ok_state = st.num_processes == world_size and st.process_index == rank and (
        want is None or st.distributed_type == want)
    ok_dev = acc.device.type == device.type and (device.type != "cuda" or acc.device.index == device.index)
    g = acc.gather(torch.tensor([rank], device=acc.device))
    ok_gather = g.tolist() == list(range(world_size))
    torch.manual_seed(99)
    m = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.GELU(), torch.nn.Linear(64, 8)).to(acc.device)
    o = torch.optim.SGD(m.parameters(), lr=0.1)
    m, o = acc.prepare(m, o)
    gen = torch.Generator().manual_seed(7 + rank)
    for _ in range(3):
        x = torch.randn(16, 32, generator=gen).to(acc.device)
        loss = m(x).square().mean()
        acc.backward(loss)
        o.step()
        o.zero_grad()
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    ok_sync = _nbd_same_on_all_ranks(flat)
    backend = dist.get_backend()
    del m, o
    return {"accelerate": ok_state and ok_dev and ok_gather and ok_sync,
            "detail": {"distributed_type": str(st.distributed_type), "num_processes": st.num_processes,
                       "gather": ok_gather, "in_sync": ok_sync, "pg_backend": str(backend)}}
'''


def _echo(d: Dict[str, Any]) -> str:
    return (d.get("echo") or d.get("output") or "").strip().splitlines()[-1]


def _per_rank(res) -> Dict[int, Dict[str, Any]]:
    out = {}
    for r in res.ranks:
        out[r] = ast.literal_eval(_echo(res.results[r]))
    return out


def _merge(dst: Dict[str, Any], detail: Dict[str, Any], per: Dict[int, Dict[str, Any]]) -> List[str]:
    """AND every boolean key over ranks into dst; keep rank 0's (and any failing rank's) detail.
    Returns the merged keys."""
    keys = set()
    for d in per.values():
        keys.update(k for k, v in d.items() if isinstance(v, bool))
    for k in sorted(keys):
        dst[k] = all(bool(per[r].get(k, False)) for r in per)
    for r, d in sorted(per.items()):
        if "detail" in d and (r == 0 or not all(v for v in d.values() if isinstance(v, bool))):
            detail.setdefault(f"rank{r}", {}).update(d["detail"])
    return sorted(keys)


def _log_default(msg: str) -> None:
    import sys

    print(f"[checks {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def run_checks(session, gpu: Optional[bool] = None, big_bytes: Optional[int] = None, log: Callable = _log_default,
               only: Optional[List[str]] = None) -> Dict[str, Any]:
    """Run every check as cells on all ranks (see the module docstring).  ``gpu``: default from
    the workers' READY; ``big_bytes``: the large message (64 MiB on GPUs, 1 MiB on CPU/gloo);
    ``only``: a subset of {"collectives", "ddp", "recipe", "graph", "accelerate", "rank_broadcast"}."""
    if gpu is None:
        gpu = bool(session.ready.get(0, {}).get("cuda_available"))
    if big_bytes is None:
        big_bytes = (64 << 20) if gpu else (1 << 20)
    want = set(only or ("collectives", "ddp", "recipe", "graph", "accelerate", "rank_broadcast"))
    results: Dict[str, Any] = {}
    detail: Dict[str, Any] = {}
    errors: Dict[str, str] = {}
    t0 = time.monotonic()
    session.execute(CHECK_SETUP, render=False)

    def one(name: str, code: str) -> None:
        t = time.monotonic()
        keys: List[str] = []
        try:
            per = _per_rank(session.execute(f"_nbd_clean({code})", render=False))
            keys = _merge(results, detail, per)
        except Exception as e:  # noqa: BLE001 - a check that raises has failed
            results[name] = False
            errors[name] = f"{type(e).__name__}: {e}"[:800]
        detail.setdefault("seconds", {})[name] = round(time.monotonic() - t, 2)
        ok = name not in errors and bool(keys) and all(results[k] is True for k in keys)
        bad = [k for k in keys if results[k] is not True]
        log(f"  check {name}: " + ("ok" if ok else f"FAILED {bad or errors.get(name, '')}"[:300]))

    if "collectives" in want:
        one("collectives", f"_nbd_chk_collectives([1024, {int(big_bytes)}], ['float32', 'bfloat16'])")
    if "ddp" in want:
        one("ddp_vs_torch", "_nbd_chk_ddp()")
    if "recipe" in want:
        one("recipe", "_nbd_chk_recipe()")
    if "graph" in want and gpu:
        one("graph", "_nbd_chk_graph()")
    if "accelerate" in want:
        one("accelerate", "_nbd_chk_accelerate()")
    if "rank_broadcast" in want:
        t = time.monotonic()
        try:
            results["rank_broadcast"] = check_rank_broadcast(session, 1024 if gpu else 256)
        except Exception as e:  # noqa: BLE001
            results["rank_broadcast"] = False
            errors["rank_broadcast"] = f"{type(e).__name__}: {e}"[:800]
        detail.setdefault("seconds", {})["rank_broadcast"] = round(time.monotonic() - t, 2)
    failed = sorted(k for k, v in results.items() if v is not True)
    out = {"passed": not failed and not errors, "failed": failed, "results": results, "detail": detail,
           "world_size": session.world_size, "seconds": round(time.monotonic() - t0, 2)}
    if errors:
        out["errors"] = errors
    return out


def check_rank_broadcast(session, dim: int) -> bool:
    """``%%rank [0]`` builds ``nn.Linear(dim, dim)`` (random init on rank 0 only), the other ranks
    allocate storage, a ``%%distributed`` cell broadcasts the parameters: every rank then holds
    rank 0's bytes (BASELINE config 3, README.md:115-125)."""
    n = session.world_size
    session.execute(f"_nbd_rb = torch.nn.Linear({dim}, {dim}, device=device)", ranks=[0], render=False)
    if n > 1:
        session.execute(f"_nbd_rb = torch.nn.Linear({dim}, {dim}, device='meta').to_empty(device=device)",
                        ranks=list(range(1, n)), render=False)
    r = session.execute("for _p in _nbd_rb.parameters():\n    dist.broadcast(_p.data, src=0)\n"
                        "_ok = all(_nbd_same_on_all_ranks(_p.data) for _p in _nbd_rb.parameters())\n"
                        "del _nbd_rb\n_ok", render=False)
    return all(_echo(r.results[k]) == "True" for k in r.ranks)


__all__ = ["CHECK_SETUP", "run_checks", "check_rank_broadcast"]
