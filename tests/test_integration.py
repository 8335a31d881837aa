"""CPU/gloo multi-process integration: every magic through a notebook-shaped shell, with real
worker processes (BASELINE config 1 and the reference's notebook flow)."""
import os
import time

import pytest
import torch  # noqa: F401  (loaded in this "kernel": proxies become meta tensors)

from nbdistributed_amd.session import DistributedExecutionError, Session
from nbdistributed_amd.utils.fakeshell import HeadlessShell


class Capture:
    def __init__(self):
        self.buf = []

    def __call__(self, s):
        self.buf.append(s)

    def take(self):
        out = "".join(self.buf)
        self.buf.clear()
        return out


@pytest.fixture(scope="module")
def nb():
    """A 2-rank session driven like a notebook: %load_ext + %dist_init -n 2."""
    sh = HeadlessShell()
    core = sh.load_extension()
    cap = Capture()
    core.write = cap
    core.session.write = cap
    sh.run_cell("%dist_init -n 2 --backend gloo", raise_errors=True)
    assert core.session.active, cap.take()
    out = cap.take()
    assert "Successfully started 2 workers" in out
    yield sh, core, cap
    sh.run_cell("%dist_shutdown")


def test_first_cell_right_after_init_is_not_lost(nb):
    # reference D-2: the first message after %dist_init could be dropped (no READY handshake)
    sh, core, cap = nb
    r = sh.run_cell("first = rank * 10\nfirst")
    assert r.success
    out = cap.take()
    assert "🔹 Rank 0:" in out and "🔹 Rank 1:" in out and "10" in out


def test_baseline_config1_allreduce_on_gloo(nb):
    sh, core, cap = nb
    sh.run_cell("x = torch.ones(4)\ndist.all_reduce(x)\nx")
    out = cap.take()
    assert out.count("tensor([2., 2., 2., 2.])") == 2


def test_namespace_contract(nb):
    sh, core, cap = nb
    res = core.session.execute("(rank, world_size, __rank__, __world_size__, str(device), __name__, dist.get_backend())",
                               render=False)
    assert res.results[0]["output"] == "(0, 2, 0, 2, 'cpu', '__main__', 'gloo')"
    assert res.results[1]["output"] == "(1, 2, 1, 2, 'cpu', '__main__', 'gloo')"


def test_print_with_several_args_is_one_line(nb):
    # reference D-8: print(a, b, c) became 3 lines (one per write() chunk)
    sh, core, cap = nb
    sh.run_cell("print('a', 'b', 3)")
    out = cap.take()
    assert out.count("  a b 3\n") == 2


def test_stderr_and_c_level_output_are_streamed(nb):
    sh, core, cap = nb
    sh.run_cell("import sys, os\nprint('err line', file=sys.stderr)\nos.system('echo from-shell-$RANK')")
    out = cap.take()
    assert out.count("err line") == 2 and "from-shell-0" in out and "from-shell-1" in out


def test_stderr_flood_does_not_wedge(nb):
    # reference §5.3: 200 KB of stderr filled an undrained pipe and wedged the worker forever
    sh, core, cap = nb
    t = time.time()
    r = sh.run_cell("import sys\nsys.stderr.write('x' * 300_000 + '\\n')\nsys.stderr.flush()\n'alive'")
    assert r.success and time.time() - t < 20
    assert cap.take().count("'alive'") == 2


def test_rank_magic_both_forms_and_subset(nb):
    sh, core, cap = nb
    sh.run_cell("%%rank [0]\nsolo = 'r0'\nprint('only', rank)")
    out = cap.take()
    assert "only 0" in out and "only 1" not in out
    sh.run_cell("%%rank[1]\nprint('nospace', rank)")  # reference D-6: this form raised UsageError
    out = cap.take()
    assert "nospace 1" in out and "nospace 0" not in out
    res = core.session.execute("'solo' in dir()", render=False)
    assert res.results[0]["output"] == "True" and res.results[1]["output"] == "False"
    sh.run_cell("%%rank [0-1]\nprint('both', rank)")
    assert cap.take().count("both") == 2
    sh.run_cell("%%rank\nprint('x')")
    assert "Usage" in cap.take()


def test_selective_build_then_broadcast(nb):
    # BASELINE config 3 (CPU-sized): build on rank 0, broadcast params to all ranks
    sh, core, cap = nb
    sh.run_cell("torch.manual_seed(rank)\nmodel = torch.nn.Linear(64, 64)")
    sh.run_cell("%%rank [0]\nref_sum = float(sum(p.detach().sum() for p in model.parameters()))")
    sh.run_cell("for p in model.parameters():\n    dist.broadcast(p.data, src=0)\n"
                "s = torch.tensor([float(sum(p.sum() for p in model.parameters()))])\n"
                "g = [torch.zeros(1) for _ in range(world_size)]\ndist.all_gather(g, s)\n"
                "bool(torch.allclose(g[0], g[1]))")
    assert cap.take().count("  True\n") == 2


def test_errors_fail_the_cell_with_per_rank_tracebacks(nb):
    sh, core, cap = nb
    r = sh.run_cell("if rank == 1:\n    raise ValueError('only rank 1 fails')\n'fine'")
    assert isinstance(r.error_in_exec, DistributedExecutionError)
    res = r.error_in_exec.result
    assert list(res.errors) == [1] and res.results[0]["output"].endswith("'fine'")
    assert "only rank 1 fails" in "\n".join(r.error_in_exec._render_traceback_())


def test_ide_sync_proxies(nb):
    sh, core, cap = nb
    sh.run_cell("weights = torch.zeros(128, 256)\ncount = 7\ndef helper(a, b=2):\n    'doc'\n    return a\n")
    ns = sh.user_ns
    assert ns["count"] == 7
    assert ns["weights"].device.type == "meta" and tuple(ns["weights"].shape) == (128, 256)
    import inspect

    assert str(inspect.signature(ns["helper"])) == "(a, b=2)"
    ns["count"] = "mine"
    sh.run_cell("count = 8")
    assert ns["count"] == "mine"  # never clobbers a local definition
    sh.run_cell("%dist_sync_ide")
    assert "Synchronized" in cap.take()


def test_sync_status_debug_mode_timeline(nb, tmp_path):
    sh, core, cap = nb
    sh.run_cell("%sync")
    assert "✓ Synchronized 2 ranks" in cap.take()
    sh.run_cell("%dist_status")
    out = cap.take()
    assert "Rank 0: ✓ PID" in out and "Rank 1: ✓ PID" in out and "Status: Running" in out
    sh.run_cell("%dist_debug")
    out = cap.take()
    assert "Connected peers: 2" in out and "Control-plane round trip" in out
    sh.run_cell("%dist_mode --disable")
    assert "disabled" in cap.take()
    sh.run_cell("local_only = 1")
    assert sh.user_ns.get("local_only") == 1
    sh.run_cell("%dist_mode -e")
    assert "enabled" in cap.take()
    sh.run_cell("%timeline_debug")
    assert "Timeline:" in cap.take()
    p = tmp_path / "tl.json"
    sh.run_cell(f"%timeline_save {p}")
    assert p.exists() and (tmp_path / "tl.trace.json").exists()
    # opt-in notebook-metadata write (reference magic.py:163-283), once on demand
    import json

    nbp = tmp_path / "nb.ipynb"
    nbp.write_text(json.dumps({"cells": [], "metadata": {"kernelspec": {"name": "python3"}}, "nbformat": 4,
                               "nbformat_minor": 5}))
    cap.take()
    sh.run_cell(f"%timeline_save {tmp_path / 'tl2.json'} --ipynb {nbp}")
    assert "execution_timelines" in cap.take()
    meta = json.loads(nbp.read_text())["metadata"]
    assert meta["kernelspec"] == {"name": "python3"} and meta["execution_timelines"]
    rec = next(iter(meta["execution_timelines"].values()))
    assert {"cell_id", "kind", "duration_s", "per_rank"} <= set(rec)
    js = core.session.timeline.notebook_metadata_js()
    assert "Jupyter.notebook.metadata.execution_timelines" in js and rec["cell_id"] in js
    sh.run_cell("%timeline_clear")
    assert "Cleared" in cap.take()


def test_dist_check_magic(nb):
    """%dist_check verifies the data plane on the live ranks (nbdistributed_amd.checks)."""
    sh, core, cap = nb
    cap.take()
    r = sh.run_cell("%dist_check --only collectives,ddp,rank_broadcast")
    assert r.success
    out = cap.take()
    assert "data-plane checks passed on 2 rank(s)" in out, out


def test_pull_push(nb):
    sh, core, cap = nb
    sh.run_cell("arr = torch.arange(6.).reshape(2, 3) + rank")
    sh.run_cell("%dist_pull arr --rank 1 --as arr1")
    import torch

    assert torch.equal(sh.user_ns["arr1"], torch.arange(6.).reshape(2, 3) + 1)
    sh.user_ns["cfg"] = {"lr": 0.1}
    sh.run_cell("%dist_push cfg")
    res = core.session.execute("cfg['lr']", render=False)
    assert res.results[1]["output"] == "0.1"


def test_interrupt_running_python_cell(nb):
    sh, core, cap = nb
    import threading

    s = core.session
    threading.Timer(0.5, lambda: s.interrupt()).start()
    t = time.time()
    r = sh.run_cell("import time\nwhile True:\n    time.sleep(0.01)")
    assert time.time() - t < 10
    assert isinstance(r.error_in_exec, DistributedExecutionError)
    assert all(e.get("status") == "interrupted" for e in r.error_in_exec.result.errors.values())
    assert sh.run_cell("'still alive'").success  # workers survive the interrupt


def test_sigint_in_the_coordinator_while_it_drains_the_socket(nb):
    # the waiting main thread is the socket's leader: a real SIGINT is deferred to a batch
    # boundary (no reply lost), then raised; the workers are interrupted and the receive thread
    # takes over again afterwards
    import signal
    import threading

    sh, core, cap = nb
    s = core.session
    before = signal.getsignal(signal.SIGINT)
    threading.Timer(0.5, lambda: os.kill(os.getpid(), signal.SIGINT)).start()
    t = time.time()
    r = sh.run_cell("import time\nwhile True:\n    time.sleep(0.01)")
    assert time.time() - t < 15
    assert isinstance(r.error_in_exec, DistributedExecutionError)
    assert all(e.get("status") == "interrupted" for e in r.error_in_exec.result.errors.values())
    assert signal.getsignal(signal.SIGINT) is before
    assert s.comm._leader is None
    cap.take()
    # background output (no request waiting) reaches the output callback through the receive thread
    got = []
    s.comm.set_output_callback(lambda rank, text, stream: got.append(text))
    try:
        s.execute("import threading\nthreading.Timer(0.2, lambda: print('late-bg', flush=True)).start()", render=False)
        deadline = time.time() + 10
        while sum("late-bg" in g for g in got) < 2 and time.time() < deadline:
            time.sleep(0.05)
        assert sum("late-bg" in g for g in got) == 2
    finally:
        s.comm.set_output_callback(None)
    assert sh.run_cell("'still alive'").success


def test_concurrent_waiters_share_one_leader(nb):
    # several threads wait at once: one drains the socket, the others are completed by it
    import threading

    sh, core, cap = nb
    comm = core.session.comm
    out, errs = {}, []

    def go(i):
        try:
            res = comm.send_to_ranks([i % 2], "execute", f"__import__('time').sleep(0.05 * {i % 3}); {i} * 7", timeout=30)
            out[i] = res[i % 2]
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ths = [threading.Thread(target=go, args=(i,)) for i in range(6)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    assert not errs and len(out) == 6
    for i, d in out.items():
        assert str(i * 7) in str(d.get("output", d)), d
    assert comm._leader is None


def test_cell_latency_is_sub_millisecond_scale(nb):
    sh, core, cap = nb
    lat = []
    for _ in range(30):
        t = time.perf_counter()
        core.session.execute("1", render=False)
        lat.append(time.perf_counter() - t)
    lat.sort()
    assert lat[15] < 0.02  # reference: 111.6 ms


# ------------------------------------------------------------------ lifecycle / faults
def _alive(pid):
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False


def test_dist_shutdown_really_stops_workers():
    # reference D-1: %dist_shutdown left the workers running
    sh = HeadlessShell()
    core = sh.load_extension()
    core.write = core.session.write = Capture()
    sh.run_cell("%dist_init -n 2 --backend gloo", raise_errors=True)
    pids = [w.pid for w in core.session.pm.workers]
    assert all(_alive(p) for p in pids)
    sh.run_cell("%dist_shutdown")
    time.sleep(0.5)
    assert not any(_alive(p) for p in pids)
    assert not core.auto_mode


def test_rank_crash_mid_cell_fails_fast_with_partial_results():
    s = Session(writer=lambda t: None)
    s.start(2, backend="gloo")
    try:
        t = time.time()
        with pytest.raises(DistributedExecutionError) as ei:
            s.execute("import os, time\nif rank == 1:\n    os._exit(7)\ntime.sleep(0.2)\n'rank0 ok'")
        assert time.time() - t < 5
        res = ei.value.result
        assert 1 in res.dead and "exit code 7" in res.dead[1] or "connection lost" in res.dead[1]
        assert res.results[0]["output"] == "'rank0 ok'"
        # later cells fail fast on the dead rank instead of hanging
        t = time.time()
        r2 = s.execute("rank", raise_on_error=False)
        assert 1 in r2.dead and time.time() - t < 2
        assert r2.results[0]["output"] == "0"
        deadline = time.time() + 5  # the socket EOF can beat the process waiter
        while s.status()[1]["returncode"] is None and time.time() < deadline:
            time.sleep(0.05)
        st = s.status()
        assert st[1]["running"] is False and st[1]["returncode"] == 7
    finally:
        s.shutdown()


def test_dist_init_replaces_degraded_cluster():
    sh = HeadlessShell()
    core = sh.load_extension()
    cap = Capture()
    core.write = core.session.write = cap
    sh.run_cell("%dist_init -n 2 --backend gloo", raise_errors=True)
    sh.run_cell("%%rank [1]\nimport os\nos._exit(1)")
    cap.take()
    sh.run_cell("%dist_init -n 2 --backend gloo")
    out = cap.take()
    assert "Replacing a degraded session" in out and "Successfully started 2 workers" in out
    assert sh.run_cell("rank").success
    sh.run_cell("%dist_reset")
    assert "Reset complete" in cap.take()
    assert not core.session.active


def test_bootstrap_failure_is_reported():
    s = Session(writer=lambda t: None)
    with pytest.raises(RuntimeError, match="failed to start|exited"):
        s.start(1, backend="rccl")  # no GPU here: rank 0 must report why it cannot start
    assert not s.active


@pytest.mark.parametrize("n", [1, 4, 8])
def test_scale_world_sizes(n):
    s = Session(writer=lambda t: None)
    t0 = time.time()
    s.start(n, backend="gloo")
    try:
        init_s = time.time() - t0
        res = s.execute("x = torch.ones(8) * (rank + 1)\ndist.all_reduce(x)\nint(x[0])", render=False)
        want = str(n * (n + 1) // 2)
        assert all(res.results[r]["output"] == want for r in range(n))
        lat = []
        for _ in range(20):
            t = time.perf_counter()
            s.execute("1", render=False)
            lat.append(time.perf_counter() - t)
        lat.sort()
        assert lat[10] < 0.05, lat
        assert init_s < 120
    finally:
        s.shutdown()


def test_subset_collective_fails_fast_instead_of_hanging(nb):
    # reference: %%rank [0] + dist.all_reduce blocks forever
    sh, core, cap = nb
    t = time.time()
    r = sh.run_cell("%%rank [0]\nx = torch.ones(4)\ndist.all_reduce(x)")
    assert time.time() - t < 5
    err = r.error_in_exec.result.errors[0]
    assert err["ename"] == "SubsetCollectiveError" and "ranks [1] are not executing" in err["error"]
    r = sh.run_cell("%%rank [0]\nimport torch.distributed as D\nD.send(torch.ones(1), dst=1)")
    assert r.error_in_exec.result.errors[0]["ename"] == "SubsetCollectiveError"
    # subgroups of the executing ranks are fine; full-world cells are unaffected
    sh.run_cell("g01 = dist.new_group([0, 1])")
    assert sh.run_cell("%%rank [0-1]\ny = torch.ones(2)\ndist.all_reduce(y, group=g01)\nint(y[0])").success
    assert sh.run_cell("z = torch.ones(2)\ndist.all_reduce(z)\nint(z[0])").success
    assert cap.take().count("  2\n") == 4


def test_interrupt_kill_then_reinit():
    sh = HeadlessShell()
    core = sh.load_extension()
    cap = Capture()
    core.write = core.session.write = cap
    sh.run_cell("%dist_init -n 2 --backend gloo", raise_errors=True)
    sh.run_cell("%dist_interrupt --kill [1]")
    assert "Killed ranks 1" in cap.take()
    time.sleep(0.5)
    r = sh.run_cell("rank")
    assert 1 in r.error_in_exec.result.dead
    sh.run_cell("%dist_init -n 2 --backend gloo")
    assert "Replacing a degraded session" in cap.take()
    assert sh.run_cell("rank").success
    sh.run_cell("%dist_shutdown")


def test_checkpoint_save_and_load_roundtrip(nb, tmp_path):
    sh, core, cap = nb
    sh.run_cell("torch.manual_seed(7 + rank)\nnet = torch.nn.Linear(8, 4)\nopt = torch.optim.SGD(net.parameters(), lr=0.1)\n"
                "step = 41 + rank\nbuf = torch.arange(5.) * (rank + 1)\nw0 = net.weight.detach().clone()")
    sh.run_cell(f"%dist_checkpoint save {tmp_path}/ck net opt step buf")
    assert "Saved net, opt, step, buf on 2 ranks" in cap.take()
    sh.run_cell("with torch.no_grad():\n    net.weight.zero_()\nstep = 0\nbuf.zero_()")
    sh.run_cell(f"%dist_checkpoint load {tmp_path}/ck net opt step buf")
    assert "Loaded" in cap.take()
    res = core.session.execute("(bool(torch.equal(net.weight, w0)), step, buf.tolist())", render=False)
    assert res.results[0]["output"] == "(True, 41, [0.0, 1.0, 2.0, 3.0, 4.0])"
    assert res.results[1]["output"] == "(True, 42, [0.0, 2.0, 4.0, 6.0, 8.0])"


def test_collective_primitives_from_cells(nb):
    # everything a user-written TP/SP/EP/PP cell needs works from cells
    sh, core, cap = nb
    code = (
        "out = []\n"
        "t = torch.tensor([float(rank)])\n"
        "g = [torch.zeros(1) for _ in range(world_size)]\ndist.all_gather(g, t)\nout.append([x.item() for x in g])\n"
        "b = torch.tensor([rank * 10.])\ndist.broadcast(b, src=1)\nout.append(b.item())\n"
        "r = torch.tensor([1.])\ndist.reduce(r, dst=0)\nout.append(r.item() if rank == 0 else None)\n"
        "if rank == 0:\n    dist.send(torch.tensor([5.]), dst=1)\nelse:\n    q = torch.zeros(1); dist.recv(q, src=0); out.append(q.item())\n"
        "ops = [dist.P2POp(dist.isend, torch.tensor([float(rank)]), (rank + 1) % 2), dist.P2POp(dist.irecv, rr := torch.zeros(1), (rank + 1) % 2)]\n"
        "[w.wait() for w in dist.batch_isend_irecv(ops)]\nout.append(rr.item())\n"
        "objs = [None, None]\ndist.all_gather_object(objs, {'r': rank})\nout.append(objs)\n"
        "out"
    )
    res = core.session.execute(code, render=False)
    assert res.results[0]["output"] == "[[0.0, 1.0], 10.0, 2.0, 1.0, [{'r': 0}, {'r': 1}]]"
    assert res.results[1]["output"] == "[[0.0, 1.0], 10.0, None, 5.0, 0.0, [{'r': 0}, {'r': 1}]]"


def test_dist_recover_rebuilds_process_group(nb):
    sh, core, cap = nb
    sh.run_cell("%dist_recover")
    assert "Process group rebuilt on 2 ranks" in cap.take()
    r = sh.run_cell("x = torch.ones(3)\ndist.all_reduce(x)\nint(x.sum())")
    assert r.success and cap.take().count("  6\n") == 2


def test_reference_order_programmatic_bringup():
    """The reference's exact sequence (magic.py:493-504): spawn first, get a port back, bind the
    CommunicationManager on it afterwards, then send — the first request must not be lost."""
    from nbdistributed_amd.communication import CommunicationManager
    from nbdistributed_amd.process_manager import ProcessManager

    streamed = []
    pm = ProcessManager()
    port = pm.start_workers(2, "localhost", None, backend="gloo")
    assert isinstance(port, int) and pm.comm_port == port
    comm = CommunicationManager(2, port, output_callback=lambda r, t, s: streamed.append((r, t)),
                                default_timeout=120)
    try:
        res = comm.send_to_all("execute", "x = rank * 10\nprint('hello from', rank)\nx")
        assert res[0]["echo"] == "0" and res[1]["echo"] == "10"
        assert any("hello from 1" in t for r, t in streamed if r == 1)
        assert comm.send_to_rank(1, "get_var", "x") == 10
        assert comm.send_to_ranks([0], "execute", "dist.get_world_size()")[0]["echo"] == "2"
        st = pm.get_detailed_status(comm)
        assert all(st[r]["running"] and st[r]["world_size"] == 2 for r in (0, 1))
    finally:
        comm.send_to_all("shutdown", timeout=5)
        comm.shutdown()
        pm.shutdown()
    assert not pm.is_running()
