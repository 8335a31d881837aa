"""Unit tests: protocol codec, rank specs, the REPL engine, namespace deltas and proxies, auto-mode
transformers, timeline, device placement helpers, CPU reference ops."""
import inspect
import json
import pickle

import pytest

from nbdistributed_amd import protocol as P
from nbdistributed_amd.executor import CellExecutor, make_namespace_module
from nbdistributed_amd.magic import auto_mode_transform, rank_nospace_transform
from nbdistributed_amd.namespace import NamespaceTracker, describe, namespace_info
from nbdistributed_amd.proxies import ProxyTable, RemoteOnlyError, _parse_signature, make_proxy
from nbdistributed_amd.timeline import Timeline
from nbdistributed_amd.utils import devices
from nbdistributed_amd.utils.ranks import RankSpecError, format_ranks, parse_ranks


# ------------------------------------------------------------------ protocol
def test_header_roundtrip():
    h = P.pack_header(P.T_EXECUTE, 3, 12345678901, P.S_STDERR, P.E_UTF8, P.F_NS_DELTA, ts=1.5)
    assert len(h) == P.HEADER_SIZE == 28
    d = P.unpack_header(h)
    assert (d.mtype, d.rank, d.seq, d.stream, d.enc, d.flags, d.ts) == (P.T_EXECUTE, 3, 12345678901, P.S_STDERR,
                                                                      P.E_UTF8, P.F_NS_DELTA, 1.5)
    assert d.type_name == "execute"


@pytest.mark.parametrize("data", [None, "print('é')", b"\x00\x01", {"a": [1, 2.5]}, [1, (2, 3)]])
def test_body_encodings(data):
    enc, body = P.encode_body(data)
    assert P.decode_body(enc, body) == data
    if isinstance(data, str):
        assert enc == P.E_UTF8  # code travels as raw text, never pickled
    if data is None:
        assert enc == P.E_NONE and body == b""


def test_message_compat():
    m = P.Message("42", "execute", -1, "x = 1")
    m2 = P.Message.from_frames(m.to_frames())
    assert (m2.msg_id, m2.msg_type, m2.rank, m2.data) == ("42", "execute", -1, "x = 1")
    with pytest.raises(ValueError):
        P.unpack_header(b"XX" + bytes(26))


def test_interrupt_prefix_matches_interrupt_header():
    h = P.pack_header(P.T_INTERRUPT, -1, 0)
    assert h.startswith(P.INTERRUPT_PREFIX)
    assert not P.pack_header(P.T_EXECUTE, -1, 0).startswith(P.INTERRUPT_PREFIX)


def test_identity_helpers():
    assert P.worker_identity(7) == b"worker_7"
    assert P.rank_of_identity(b"worker_12") == 12
    assert P.rank_of_identity(b"\x00abcd") is None


# ------------------------------------------------------------------ rank specs
@pytest.mark.parametrize("spec,ws,want", [
    ("[0,1,2]", 4, [0, 1, 2]), ("[0-2]", 4, [0, 1, 2]), ("[0-2,5]", 8, [0, 1, 2, 5]), ("0,1", 4, [0, 1]),
    ("[3]", 4, [3]), ("[1, 1, 0]", 4, [0, 1]), ("[0-7]", 4, [0, 1, 2, 3]), ("all", 3, [0, 1, 2]), ("[*]", 2, [0, 1]),
])
def test_parse_ranks(spec, ws, want):
    assert parse_ranks(spec, ws) == want


@pytest.mark.parametrize("spec", ["[", "[a]", "[3-1]", "[]", "[0-x]"])
def test_parse_ranks_errors(spec):
    with pytest.raises(RankSpecError):
        parse_ranks(spec, 4)


def test_parse_ranks_strict_and_format():
    with pytest.raises(RankSpecError):
        parse_ranks("[0,9]", 4, strict=True)
    assert format_ranks([0, 1, 2, 5, 7, 8]) == "0-2,5,7-8"


# ------------------------------------------------------------------ executor
@pytest.fixture
def ex():
    return CellExecutor(make_namespace_module("__cell_test__"), install_as_main=False)


def test_rerun_cell_reuses_compiled_code(ex):
    ex.run("n_runs = 0")
    a = ex.run("n_runs += 1\nn_runs * 10")
    b = ex.run("n_runs += 1\nn_runs * 10")
    assert (a.value, b.value) == (10, 20) and a.filename == b.filename  # executed again, not cached
    c = ex.run("n_runs += 1\nn_runs * 10", echo=False)  # other echo mode: compiled separately
    assert not c.has_value and ex.ns["n_runs"] == 3
    for _ in range(2):  # a re-run failing cell still points at its own source line
        e = ex.run("ok = 1\nraise ValueError('boom')")
        assert e.status == "error" and "raise ValueError('boom')" in e.traceback
    s = ex.run("def (:")
    assert s.status == "error" and s.ename == "SyntaxError"


def test_expression_and_trailing_expression(ex):
    r = ex.run("1 + 2")
    assert r.status == "ok" and r.value == 3 and r.has_value
    r = ex.run("x = 5\nx * 2")
    assert r.value == 10 and ex.ns["x"] == 5 and ex.ns["_"] == 10
    r = ex.run("y = 1")
    assert not r.has_value
    r = ex.run("None")
    assert not r.has_value
    r = ex.run("x + 1", echo=False)
    assert not r.has_value


def test_syntax_error_is_clean(ex):
    r = ex.run("def f(:\n  pass")
    assert r.status == "error" and r.ename == "SyntaxError"
    assert "During handling" not in r.traceback and "executor.py" not in r.traceback


def test_runtime_error_traceback_shows_cell_source(ex):
    r = ex.run("def f(a):\n    return 1 / a\nf(0)")
    assert r.status == "error" and r.ename == "ZeroDivisionError"
    assert "return 1 / a" in r.traceback and "<cell-" in r.traceback
    assert "executor.py" not in r.traceback and "During handling" not in r.traceback


def test_top_level_await(ex):
    r = ex.run("import asyncio\nawait asyncio.sleep(0)\n41 + 1")
    assert r.status == "ok" and r.value == 42


def test_sys_exit_does_not_kill(ex):
    r = ex.run("import sys\nsys.exit(3)")
    assert r.status == "error" and r.ename == "SystemExit"


def test_namespace_module_makes_cell_functions_picklable():
    ex = CellExecutor(make_namespace_module("__main__"), install_as_main=True)
    r = ex.run("def add(a, b):\n    return a + b\nclass K:\n    v = 3\n__name__")
    assert r.value == "__main__"
    f = pickle.loads(pickle.dumps(ex.ns["add"]))
    assert f(2, 3) == 5
    assert pickle.loads(pickle.dumps(ex.ns["K"]())).v == 3


# ------------------------------------------------------------------ namespace + proxies
def test_namespace_delta_tracks_changes():
    tr = NamespaceTracker()
    ns = {"a": 1, "_hidden": 2, "f": len}
    d = tr.delta(ns)
    assert {c["name"] for c in d["changed"]} == {"a", "f"}
    assert tr.delta(ns)["changed"] == []
    ns["a"] = 2
    del ns["f"]
    d = tr.delta(ns)
    assert [c["name"] for c in d["changed"]] == ["a"] and d["removed"] == ["f"]


def test_describe_kinds():
    import torch

    assert describe("t", torch.zeros(2, 3))["kind"] == "tensor"
    assert describe("t", torch.zeros(2, 3))["shape"] == (2, 3)
    assert describe("d", torch.device("cpu"))["kind"] == "device"
    assert describe("m", torch.nn.Linear(2, 2))["kind"] == "nn_module"
    assert describe("n", 5)["value"] == 5
    assert describe("s", "x" * 5000).get("value") is None
    info = namespace_info({"x": 1, "_y": 2})
    assert list(info) == ["x"]
    json.dumps(info)  # plain data


def test_proxies_meta_tensor_and_signature():
    import torch

    t = make_proxy({"name": "w", "kind": "tensor", "shape": (1024, 1024), "dtype": "torch.bfloat16"})
    assert t.device.type == "meta" and t.shape == (1024, 1024) and t.dtype == torch.bfloat16
    f = make_proxy({"name": "f", "kind": "callable", "signature": "(a, b=3, *args, c: int = 4, **kw)", "doc": "hi"})
    assert str(inspect.signature(f)) == "(a, b=3, *args, c=4, **kw)"
    with pytest.raises(RemoteOnlyError):
        f(1)
    assert _parse_signature("(<bad>)") is None


def test_proxy_table_never_clobbers_local_names():
    ns = {"mine": "local value"}
    pt = ProxyTable()
    pt.apply(ns, {"changed": [{"name": "mine", "kind": "builtin", "value": 1},
                              {"name": "remote", "kind": "builtin", "value": 2}], "removed": []})
    assert ns["mine"] == "local value" and ns["remote"] == 2
    pt.apply(ns, {"changed": [{"name": "remote", "kind": "builtin", "value": 3}], "removed": []})
    assert ns["remote"] == 3  # our own proxy is refreshed
    pt.apply(ns, {"changed": [], "removed": ["remote", "mine"]})
    assert "remote" not in ns and ns["mine"] == "local value"


# ------------------------------------------------------------------ transformers
@pytest.mark.parametrize("cell,shipped", [
    ("x = 1\n", True), ("%time x = 1\n", False), ("%%rank [0]\nx\n", False), ("!ls\n", False), ("x?\n", False),
    ("?x\n", False), ("# just a comment\n", False), ("\n\n", False), ("# c\nprint(1)\n", True),
    ("__jupyter_exec_background__()\n", False), ("print('what?')", True),
])
def test_auto_mode_transform(cell, shipped):
    lines = cell.splitlines(keepends=True)
    out = auto_mode_transform(lines)
    assert (out[0] == "%%distributed\n") == shipped
    if shipped:
        assert "".join(out[1:]).rstrip("\n") == cell.rstrip("\n")


def test_rank_nospace_transform():
    assert rank_nospace_transform(["%%rank[0]\n", "x\n"]) == ["%%rank [0]\n", "x\n"]
    assert rank_nospace_transform(["%%rank [0-1]\n"]) == ["%%rank [0-1]\n"]
    assert rank_nospace_transform(["x = '%%rank[0]'\n"]) == ["x = '%%rank[0]'\n"]


# ------------------------------------------------------------------ timeline
def test_timeline_bounded_and_exports(tmp_path):
    tl = Timeline(capacity=5)
    for i in range(12):
        rec = tl.start(i, "distributed", [0, 1], f"cell {i}")
        tl.end(rec, {0: {"exec_s": 0.001, "t_start": rec.t_start, "status": "success", "gpu_ms": {i: 0.5}},
                     1: {"dead": True}}, 0.002, "ok")
    assert len(tl.records) == 5
    assert tl.by_seq.keys() == {7, 8, 9, 10, 11}
    out = tl.save(str(tmp_path / "tl.json"))
    data = json.load(open(out["json"]))
    assert len(data["records"]) == 5
    tr = json.load(open(out["trace"]))
    assert any(e.get("args", {}).get("name") == "rank 0" for e in tr["traceEvents"])
    assert "p50" in tl.summary()
    assert tl.clear() == 5 and not tl.records


# ------------------------------------------------------------------ device placement
def test_worker_visible_devices(monkeypatch):
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    assert devices.worker_visible_devices([3, 4]) == "3,4"
    assert devices.local_device_index([3, 4], 1) == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "4,5,6,7")
    assert devices.worker_visible_devices([1, 2]) == "5,6"  # ids are relative to the kernel's view
    assert devices.worker_visible_devices([0, 0, 1]) == "4,5"
    assert devices.local_device_index([0, 0, 1], 2) == 1


def test_kfd_parsing_is_safe_without_gpu():
    g = devices.kfd_gpus()
    assert isinstance(g, list)
    m = devices.xgmi_matrix(g)
    assert m["n_gpus"] == len(g)


# ------------------------------------------------------------------ CPU reference ops
def test_reference_ops_cpu():
    import torch

    from nbdistributed_amd import ops

    ts = [torch.randn(5), torch.randn(3, 4), torch.randn(129)]
    offs, total = ops.plan_offsets([t.numel() for t in ts])
    assert all(o % 64 == 0 for o in offs) and total >= sum(t.numel() for t in ts)
    b, offs = ops.bucket_flatten(ts, dtype=torch.float32, scale=2.0)
    outs = [torch.zeros_like(t) for t in ts]
    ops.bucket_unflatten(b, outs, offs, scale=0.5)
    for a, t in zip(outs, ts):
        torch.testing.assert_close(a, t)
    ops.bucket_unflatten(b, outs, offs, scale=0.5, accumulate=True)
    for a, t in zip(outs, ts):
        torch.testing.assert_close(a, 2 * t)
    r = ops.local_prereduce([torch.ones(7), torch.full((7,), 3.0)], scale=0.5)
    assert torch.equal(r, torch.full((7,), 2.0))
    s = ops.tensor_summary(torch.tensor([1.0, 2.0, float("nan"), float("inf")]))
    assert s["count"] == 4 and s["nan"] == 1 and s["inf"] == 1 and s["min"] == 1.0 and s["max"] == float("inf")
    assert "mean=" in ops.tensor_summary_text(torch.arange(10.0))


def test_gpt2_return_logits_flag_cpu():
    import torch

    from nbdistributed_amd.models import GPT2, GPT2Config

    torch.manual_seed(0)
    m = GPT2(GPT2Config.tiny())
    idx = torch.randint(0, 512, (2, 16))
    logits, loss = m(idx, idx)
    none, loss2 = m(idx, idx, return_logits=False)
    assert logits.shape == (2, 16, 512) and none is None and torch.equal(loss, loss2)
    assert m(idx)[1] is None
