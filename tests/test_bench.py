"""The benchmark harness itself, multi-rank on CPU/gloo: the same cells the driver's 2/4/8-GPU
runs execute (all-reduce timing, DDP phases) and bench.py's JSON contract."""
import json
import os
import subprocess
import sys

import pytest

from nbdistributed_amd import benchmarking as B
from nbdistributed_amd.session import Session

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sess():
    s = Session(writer=lambda t: None)
    s.start(2, backend="gloo")
    yield s
    s.shutdown()


def test_allreduce_phase_multi_rank(sess):
    r = B.bench_allreduce(sess, nbytes=1 << 16, iters=3, warm=1)
    assert r["correct"] and r["busbw_GBps"] is not None and r["busbw_GBps"] > 0
    assert set(r["per_rank_ms"]) == {0, 1}


def test_ddp_phase_multi_rank(sess):
    r = B.bench_ddp(sess, steps=2, warmup=1, B=2, T=32, config="tiny", linear_rows=16, linear_dim=64)
    assert r["ms_per_step"] > 0 and r["tokens_per_s"] > 0 and r["global_batch"] == 4
    assert r["amp_ms_per_step"] > 0 and "FlatAdamW" in r["recipe"]
    assert r["torch_ddp_ms_per_step"] > 0 and r["linear4096"]["ms_per_step"] > 0
    lb = r["linear4096"]["bf16"]  # the bf16 arm (fp32 on the CPU): both implementations timed
    assert lb["ms_per_step"] > 0 and lb["torch_ddp_ms_per_step"] > 0 and lb["speedup_vs_torch_ddp"] > 0


def test_allreduce_sweep_multi_rank(sess):
    sw = B.bench_sweep(sess, max_bytes=1 << 14, min_bytes=1 << 10)
    assert [r["bytes"] for r in sw] == [1024, 4096, 16384] and all(r["busbw_GBps"] is not None for r in sw)
    cells = {"p50_ms": 1.0, "p90_ms": 1.0, "min_ms": 1.0, "mean_ms": 1.0}
    line = B.result_line({"cell": cells, "sweep": sw}, 2, 1, 1)
    assert line["allreduce_peak_busbw_GBps"] == max(r["busbw_GBps"] for r in sw)


def test_notebook_phase_multi_rank(sess):
    r = B.bench_notebook(sess, steps=2, warmup=1, small=True)
    for mode in ("reference", "nbd"):
        assert r[mode]["ms_per_step"] > 0 and r[mode]["samples_per_s"] > 0
    assert r["reference_ms_per_step"] == 126.6


def test_rank_broadcast_phase_multi_rank(sess):
    r = B.bench_rank_broadcast(sess, dim=128, iters=3, warm=1)
    assert r["correct"], r
    assert r["per_param_ms"] > 0 and r["coalesced_ms"] > 0 and r["bytes"] == (128 * 128 + 128) * 4


def test_cells_phase_and_result_line(sess):
    cells = B.bench_cells(sess, steps=10, warmup=2)
    line = B.result_line({"cell": cells}, 2, 10, 2)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in line
    assert line["metric"] == json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert line["higher_is_better"] is False and line["n_gpus"] == 2


def test_failed_phase_is_recorded_and_timeout_aborts_the_rest():
    class _Cfg:
        interrupt_abort_s = 0.0

    class _Sess:
        default_timeout = None
        cfg = _Cfg()
        interrupts = 0

        def interrupt(self):
            self.interrupts += 1

    def _timeout():
        raise TimeoutError("ranks stuck")

    s, out = _Sess(), {}
    B._phase(s, out, "a", lambda: 1 / 0, 5.0)
    B._phase(s, out, "b", _timeout, 5.0)
    B._phase(s, out, "c", lambda: {"ok": 1}, 5.0)
    assert "ZeroDivisionError" in out["a"]["error"] and out["aborted"] == "b"
    assert "skipped" in out["c"] and s.interrupts == 1 and s.default_timeout is None
    cells = {"p50_ms": 1.0, "p90_ms": 1.0, "min_ms": 1.0, "mean_ms": 1.0}
    line = B.result_line({"cell": cells, "allreduce": out["a"], "aborted": "b"}, 2, 1, 1)
    assert line["allreduce_error"].startswith("ZeroDivisionError") and line["aborted_phase"] == "b"


@pytest.mark.parametrize("n", [1, 2])
def test_bench_py_contract_cpu(n):
    if n == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "2"]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", "29655", os.path.join(ROOT, "bench.py"),
               "--gpus", str(n), "--steps", "20", "--warmup", "2"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd="/tmp")
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert res.returncode == 0 and len(lines) == 1, res.stdout[-2000:] + res.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 20 and d["value"] > 0 and d["config"]["parallelism"] == f"dp{n}"
    # the magic path (auto transformer + %%distributed + ide_sync delta + renderer) is timed too
    assert d["cell_magic_p50_ms"] > 0 and "ide_sync=True" in d["cell_magic_note"]
    # every worker reports the process group it sees
    assert d["rccl_world_size"] == {str(r): n for r in range(n)}
    assert d["launch"].startswith("self" if n == 1 else "attach")


def _selflaunch(n, env_extra=None, timeout=300, args=()):
    """``python bench.py --gpus N`` with no torchrun variables: bench.py starts its own N workers."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "TORCHELASTIC_RUN_ID")}
    env.update({"NBD_BENCH_IPYTHON": "0"}, **(env_extra or {}))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "10", "--warmup", "2",
           "--no-ddp", "--no-notebook", "--no-bcast", *args]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=env)
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    return res, lines


@pytest.mark.parametrize("n", [2, 4])
def test_bench_py_self_launch(n):
    """Without torchrun, ``--gpus N`` starts N workers itself (as ``%dist_init -n N``): every rank
    sees a world of N and the all-reduce cells report a bus bandwidth."""
    res, lines = _selflaunch(n)
    assert res.returncode == 0 and len(lines) == 1, res.stdout[-2000:] + res.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["value"] > 0 and d["config"]["parallelism"] == f"dp{n}"
    assert d["rccl_world_size"] == {str(r): n for r in range(n)}
    assert d["allreduce_busbw_GBps"] is not None and d["allreduce_busbw_GBps"] > 0 and d["allreduce_correct"]
    assert d["allreduce_peak_busbw_GBps"] > 0 and d["launch"].startswith("self")
    # every data-plane correctness check ran at this world size and passed
    ck = d["checks"]
    assert d["checks_passed"] is True and ck["passed"] and ck["world_size"] == n and not ck["failed"], ck
    for k in ("ddp_vs_torch", "recipe_sync", "zero2", "accelerate", "rank_broadcast"):
        assert ck["results"][k] is True, (k, ck)
    for op in ("all_reduce", "broadcast", "all_gather", "reduce_scatter", "all_to_all", "send_recv",
               "batch_isend_irecv"):
        for dt in ("float32", "bfloat16"):
            assert ck["results"][f"{op}_{dt}_1024"] is True, (op, dt, ck)


def test_bench_py_broken_ddp_hook_fails_the_run():
    """A deliberately broken gradient hook (rank 0 scales its buckets by 1.5 before the
    collective: ``NBD_FAULT_DDP_GRAD_SCALE``) trains without any error — only the DDP-parity
    check against torch DDP sees it, and the bench then exits non-zero."""
    res, lines = _selflaunch(2, env_extra={"NBD_FAULT_DDP_GRAD_SCALE": "1.5"}, args=("--no-sweep",))
    assert len(lines) == 1, res.stdout[-2000:] + res.stderr[-3000:]
    d = json.loads(lines[0])
    assert res.returncode == 5, (res.returncode, d.get("checks"))
    assert d["checks_passed"] is False and "ddp_vs_torch" in d["checks"]["failed"]
    assert d["checks"]["results"]["all_reduce_float32_1024"] is True  # the collectives themselves are fine


def test_bench_py_rank_that_never_joins_is_reported():
    """One rank never starts: the line (value null, "rendezvous: 1/2 ranks joined") is printed
    before the rendezvous limit runs out, with a non-zero exit status — never a silent hang."""
    res, lines = _selflaunch(2, {"NBD_FAULT_STALL_RANK": "1", "NBD_BENCH_RENDEZVOUS_S": "20"}, timeout=120)
    assert len(lines) == 1, res.stdout[-2000:] + res.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["value"] is None and d["error"] == "rendezvous: 1/2 ranks joined", d
    assert d["rendezvous"]["ready"] == 0 and res.returncode == 3


def test_bench_py_torchrun_rank_that_never_joins_is_reported():
    """The same under torchrun: rank 1 never connects, rank 0 is stuck in the RCCL/gloo rendezvous;
    rank 0 still prints the error line once its coordinator gives up."""
    env = dict(os.environ, NBD_FAULT_STALL_RANK="1", NBD_BENCH_RENDEZVOUS_S="15", NBD_BENCH_GRACE_S="3",
               NBD_BENCH_IPYTHON="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29657", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "5", "--warmup", "1"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd="/tmp", env=env)
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:] + res.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["value"] is None and d["error"].startswith("rendezvous: ") and d["error"].endswith("/2 ranks joined")
    assert res.returncode != 0


def test_world1_reports_no_bandwidth():
    """At world size 1 an all_reduce / broadcast is a no-op: no GB/s may be printed for it."""
    s = Session(writer=lambda t: None)
    s.start(1, backend="gloo")
    try:
        ar = B.bench_allreduce(s, nbytes=1 << 16, iters=3, warm=1)
        assert ar["correct"] and ar["algbw_GBps"] is None and ar["busbw_GBps"] is None
        sw = B.bench_sweep(s, max_bytes=1 << 12, min_bytes=1 << 10)
        assert all(r["algbw_GBps"] is None and r["busbw_GBps"] is None for r in sw)
        rb = B.bench_rank_broadcast(s, dim=64, iters=2, warm=1)
        assert rb["per_param_GBps"] is None and rb["coalesced_GBps"] is None
        cells = {"p50_ms": 1.0, "p90_ms": 1.0, "min_ms": 1.0, "mean_ms": 1.0}
        line = B.result_line({"cell": cells, "allreduce": ar, "sweep": sw}, 1, 1, 1)
        assert line["allreduce_algbw_GBps"] is None and line["allreduce_busbw_GBps"] is None
        assert "allreduce_peak_busbw_GBps" not in line and "no-op" in line["allreduce_note"]
        w = B.bench_world(s)
        assert w["world_sizes"] == [1]
    finally:
        s.shutdown()


def test_magic_path_cells(sess):
    r = B.bench_cells_magic(sess, steps=5, warmup=2)
    assert r["p50_ms"] > 0 and r["ide_sync"] is True and r["rendered_bytes"] > 0


def _run_bench(env_extra, timeout=240):
    env = dict(os.environ, NBD_BENCH_IPYTHON="0", **env_extra)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "5", "--warmup", "1"]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=env)
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    return res, lines


def test_bench_line_survives_a_phase_past_the_global_deadline():
    """A phase that hangs past the bench's global budget is interrupted and recorded; the JSON
    line (with the measured cell p50) is still printed, exactly once."""
    res, lines = _run_bench({"NBD_BENCH_FAULT_HANG": "600", "NBD_BENCH_DEADLINE_S": "25"})
    assert res.returncode == 0 and len(lines) == 1, res.stdout[-2000:] + res.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["aborted_phase"] == "fault_hang"


def test_bench_line_survives_the_hard_deadline():
    """Past the hard deadline rank 0 kills the coordinator and, still stuck in the cell, prints
    the checkpointed result itself."""
    res, lines = _run_bench({"NBD_BENCH_FAULT_HANG": "600", "NBD_BENCH_DEADLINE_S": "400",
                             "NBD_BENCH_HARD_S": "30", "NBD_BENCH_GRACE_S": "3"})
    # a partial line is printed, and the exit status says the run did not complete
    assert res.returncode == 3 and len(lines) == 1, res.stdout[-2000:] + res.stderr[-3000:]
    d = json.loads(lines[0])
    assert d["value"] > 0 and d["partial"] is True and d["partial_reason"] == "hard deadline"
