"""Real IPython as the notebook kernel.

The PyTorch interpreter here has no IPython, but /opt/conda/bin/python3.9 has IPython 7.29 (and
no torch).  That is exactly the split the framework is designed for: the coordinator (kernel)
needs neither torch nor pyzmq; the workers run the PyTorch interpreter.  Skipped when the oracle
interpreter is absent."""
import os
import subprocess
import sys
import textwrap

import pytest

PY39 = "/opt/conda/bin/python3.9"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _has_ipython():
    if not os.path.exists(PY39):
        return False
    return subprocess.run([PY39, "-c", "import IPython"], capture_output=True).returncode == 0


@pytest.mark.skipif(not _has_ipython(), reason="no IPython interpreter available")
def test_magics_under_real_ipython_with_torchless_kernel():
    code = f"""
        import sys
        sys.path.insert(0, {ROOT!r})
        from IPython.core.interactiveshell import InteractiveShell
        sh = InteractiveShell.instance()
        sh.run_cell("%load_ext nbdistributed_amd")
        sh.run_cell("%dist_init -n 2 --backend gloo --python {sys.executable}")
        r = sh.run_cell("x = torch.ones(4) * (rank + 1)\\ndist.all_reduce(x)\\nint(x[0])")
        assert r.error_in_exec is None, r.error_in_exec
        r = sh.run_cell("%%rank[0]\\nprint('hi from', rank)")
        assert r.error_in_exec is None
        r = sh.run_cell("1/0")
        assert type(r.error_in_exec).__name__ == "DistributedExecutionError"
        r = sh.run_cell("!echo local-shell-ok")
        assert "torch" not in sys.modules, "the kernel must not import torch"
        print("PROXY", repr(sh.user_ns.get("x")))
        sh.run_cell("%dist_shutdown")
        print("REAL IPYTHON OK")
    """
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "PYTHONHOME")}
    res = subprocess.run([PY39, "-c", textwrap.dedent(code)], capture_output=True, text=True, timeout=180, env=env)
    out = res.stdout + res.stderr
    assert "REAL IPYTHON OK" in res.stdout, out[-3000:]
    assert res.stdout.count("  3\n") == 2  # (1 + 2) all-reduced, echoed by both ranks
    assert "hi from 0" in res.stdout and "hi from 1" not in res.stdout
    assert "ZeroDivisionError" in out
    assert "local-shell-ok" in out
    assert "PROXY <remote tensor shape=[4]" in res.stdout
