"""Fault injection: spec grammar, and each fault kind driving the failure paths
it exists for — fail-fast on a crashed rank, interrupt of a hung rank, stderr floods, injected
exceptions — on real gloo worker processes."""
import threading
import time

import pytest

from nbdistributed_amd import faults
from nbdistributed_amd.session import DistributedExecutionError, Session
from nbdistributed_amd.utils.fakeshell import HeadlessShell


def test_parse_grammar():
    fs = faults.parse("crash:7@1#3; hang@0-2 ;raise;flood:64@0,3")
    assert [(f.kind, f.arg, f.ranks, f.cell) for f in fs] == [
        ("crash", 7.0, {1}, 3), ("hang", None, {0, 1, 2}, 1), ("raise", None, None, 1), ("flood", 64.0, {0, 3}, 1)]
    assert [f.spec() for f in fs] == ["crash:7@1#3", "hang@0,1,2", "raise", "flood:64@0,3"]
    assert faults.parse("") == [] and faults.parse(None) == []
    with pytest.raises(ValueError, match="unknown fault kind"):
        faults.parse("explode@1")
    with pytest.raises(ValueError):
        faults.parse("crash#0")


def test_plan_counts_cells_and_fires_once():
    plan = faults.FaultPlan(rank=1, faults=faults.parse("raise@1#2; raise@0"))
    assert len(plan.pending) == 1  # the rank-0 fault is not armed on rank 1
    plan.before_cell()  # cell 1: nothing
    with pytest.raises(faults.InjectedFault):
        plan.before_cell()  # cell 2
    plan.before_cell()  # fired once only
    assert plan.fired == ["raise@1#2"] and plan.pending == []


def test_delay_fault_runs_the_cell_afterwards():
    plan = faults.FaultPlan(rank=0, faults=faults.parse("delay:0.2"))
    t = time.perf_counter()
    plan.before_cell()
    assert time.perf_counter() - t >= 0.19


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
    sh = HeadlessShell()
    core = sh.load_extension()
    cap = Capture()
    core.write = core.session.write = cap
    sh.run_cell("%dist_init -n 2 --backend gloo", raise_errors=True)
    cap.take()
    yield sh, core, cap
    sh.run_cell("%dist_shutdown")


def test_magic_arm_list_clear(nb):
    sh, core, cap = nb
    sh.run_cell("%dist_fault raise@1#5 delay:1@0#9")
    out = cap.take()
    assert "Rank 1: raise@1#5 (in 5 cells)" in out and "Rank 0: delay:1@0#9 (in 9 cells)" in out
    sh.run_cell("%dist_fault --clear")
    assert "Rank 0: cleared 1" in cap.take()
    sh.run_cell("%dist_fault --list")
    assert cap.take().count("none armed") == 2
    sh.run_cell("%dist_fault bogus")
    assert "unknown fault kind" in cap.take()


def test_injected_exception_fails_only_that_rank(nb):
    sh, core, cap = nb
    s = core.session
    s.fault("arm", "raise@1")
    with pytest.raises(DistributedExecutionError) as ei:
        s.execute("'ran'", render=False)
    res = ei.value.result
    assert res.results[0]["output"] == "'ran'"
    assert res.results[1]["ename"] == "InjectedFault"
    assert s.execute("'again'", render=False).results[1]["output"] == "'again'"  # fired once


def test_stderr_flood_is_drained(nb):
    sh, core, cap = nb
    s = core.session
    s.fault("arm", "flood:512@1")  # 512 KiB: the reference's undrained pipe wedged at 200 KB
    t = time.time()
    res = s.execute("'after flood'", render=False)
    assert time.time() - t < 30
    out = res.results[1]["output"]
    assert out.endswith("'after flood'") and out.count("x" * 1023) == 512


def test_hang_is_interruptible(nb):
    sh, core, cap = nb
    s = core.session
    s.fault("arm", "hang@1")
    threading.Timer(0.5, lambda: s.interrupt([1])).start()
    t = time.time()
    res = s.execute("'ok'", render=False, raise_on_error=False)
    assert time.time() - t < 20
    assert res.results[0]["output"] == "'ok'"
    assert res.results[1]["status"] == "interrupted"
    assert s.execute("rank", render=False).results[1]["output"] == "1"


def test_crash_from_env_fails_fast_on_the_named_cell():
    s = Session(writer=lambda t: None)
    s.start(2, backend="gloo", extra_env={"NBD_FAULTS": "crash:9@1#2"})
    try:
        assert s.execute("rank", render=False).results[1]["output"] == "1"  # cell 1: fine
        t = time.time()
        r = s.execute("'second'", render=False, raise_on_error=False)  # cell 2: rank 1 dies
        assert time.time() - t < 5
        assert 1 in r.dead and r.results[0]["output"] == "'second'"
        deadline = time.time() + 5  # the socket EOF can beat the process waiter
        while s.status()[1]["returncode"] is None and time.time() < deadline:
            time.sleep(0.05)
        assert s.status()[1]["returncode"] == 9
    finally:
        s.shutdown()
