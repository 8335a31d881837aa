"""Execute examples/00_accelerate_mi355x.ipynb headlessly (CPU/gloo, tiny config): the reference
notebook's workflow end to end through the magics."""
import json
import os

import pytest

from nbdistributed_amd.utils.fakeshell import HeadlessShell

NB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "00_accelerate_mi355x.ipynb")


@pytest.mark.parametrize("hf_only", [False, True], ids=["native-swap", "hf-as-written"])
def test_example_notebook_runs_end_to_end(monkeypatch, hf_only):
    pytest.importorskip("transformers")
    pytest.importorskip("accelerate")
    monkeypatch.setenv("NBD_NOTEBOOK_TINY", "1")
    monkeypatch.setenv("NBD_NOTEBOOK_HF", "1" if hf_only else "0")
    cells = [c for c in json.load(open(NB))["cells"] if c["cell_type"] == "code"]
    sh = HeadlessShell()
    core = sh.load_extension()
    out = []
    core.write = core.session.write = out.append
    try:
        for c in cells:
            src = "".join(c["source"])
            if src.startswith("%load_ext"):
                continue
            if src.startswith("%dist_init"):
                src += " --backend gloo"
            r = sh.run_cell(src)
            assert r.success, (src, r.error_in_exec, "".join(out)[-3000:])
        text = "".join(out)
        assert "accuracy" in text and "epoch time" in text and "Distributed cluster status" in text
    finally:
        if core.session.active:
            core.session.shutdown()


NB1 = os.path.join(os.path.dirname(NB), "01_native_llama_graphs.ipynb")


def test_native_llama_notebook_runs_end_to_end(monkeypatch):
    monkeypatch.setenv("NBD_NOTEBOOK_TINY", "1")
    cells = [c for c in json.load(open(NB1))["cells"] if c["cell_type"] == "code"]
    sh = HeadlessShell()
    core = sh.load_extension()
    out = []
    core.write = core.session.write = out.append
    try:
        for c in cells:
            src = "".join(c["source"])
            if src.startswith("%load_ext"):
                continue
            if src.startswith("%dist_init"):
                src += " --backend gloo"
            r = sh.run_cell(src)
            assert r.success, (src, r.error_in_exec, "".join(out)[-3000:])
        text = "".join(out)
        assert "parameters identical to rank 0: True" in text and "CPU run, loss" in text
    finally:
        if core.session.active:
            core.session.shutdown()


NB3 = os.path.join(os.path.dirname(NB), "03_zero_sharded.ipynb")


def test_zero_notebook_runs_end_to_end(monkeypatch):
    monkeypatch.setenv("NBD_NOTEBOOK_TINY", "1")
    cells = [c for c in json.load(open(NB3))["cells"] if c["cell_type"] == "code"]
    sh = HeadlessShell()
    core = sh.load_extension()
    out = []
    core.write = core.session.write = out.append
    try:
        for c in cells:
            src = "".join(c["source"])
            if src.startswith("%load_ext"):
                continue
            if src.startswith("%dist_init"):
                src += " --backend gloo"
            r = sh.run_cell(src)
            assert r.success, (src, r.error_in_exec, "".join(out)[-3000:])
        text = "".join(out)
        assert "parameters identical to rank 0: True" in text and "step 4: loss" in text
    finally:
        if core.session.active:
            core.session.shutdown()


NB4 = os.path.join(os.path.dirname(NB), "04_train_and_generate.ipynb")


def test_generate_notebook_runs_end_to_end(monkeypatch):
    monkeypatch.setenv("NBD_NOTEBOOK_TINY", "1")
    cells = [c for c in json.load(open(NB4))["cells"] if c["cell_type"] == "code"]
    sh = HeadlessShell()
    core = sh.load_extension()
    out = []
    core.write = core.session.write = out.append
    try:
        for c in cells:
            src = "".join(c["source"])
            if src.startswith("%load_ext"):
                continue
            if src.startswith("%dist_init"):
                src += " --backend gloo"
            r = sh.run_cell(src)
            assert r.success, (src, r.error_in_exec, "".join(out)[-3000:])
        text = "".join(out)
        assert "step 300: loss" in text and "counting continuation correct: True" in text, text[-3000:]
    finally:
        if core.session.active:
            core.session.shutdown()
