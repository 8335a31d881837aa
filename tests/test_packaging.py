"""The package installs and runs from a read-only location (reference: a ``pip install``-able
package, ``/root/reference/pyproject.toml:1-82``).

``pip install --target`` into a temporary directory, ``chmod -R a-w`` it, then a fresh torch-less
IPython 7.29 kernel (python3.9), started from ``/`` with only that directory on its path and as an
unprivileged user, runs ``%load_ext nbdistributed_amd``, ``%dist_init -n 2 --backend gloo`` and a
``dist.all_reduce`` cell.  Nothing in the installed tree may change (no build outputs, no lock
files)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IPY = "/opt/conda/bin/python3.9"

KERNEL = r'''
import sys
from IPython.core.interactiveshell import InteractiveShell
sh = InteractiveShell.instance()
for cell in ["%load_ext nbdistributed_amd", "%dist_init -n 2 --backend gloo",
             "x = torch.ones(4) * (rank + 1)\ndist.all_reduce(x)\nprint('allreduce', x.tolist())",
             "import nbdistributed_amd._native as N\nprint('csrc', N.CSRC)",
             "%dist_shutdown"]:
    r = sh.run_cell(cell)
    if r.error_in_exec is not None or r.error_before_exec is not None:
        print("CELL FAILED", repr(cell), r.error_in_exec, r.error_before_exec)
        sys.exit(1)
import nbdistributed_amd
print("PKG", nbdistributed_amd.__file__)
'''


def _snapshot(d):
    out = {}
    for base, _dirs, files in os.walk(d):
        if "__pycache__" in base:
            continue
        for f in files:
            p = os.path.join(base, f)
            st = os.stat(p)
            out[p] = (st.st_size, st.st_mtime_ns)
    return out


@pytest.mark.skipif(not os.path.exists(IPY), reason="no IPython interpreter")
def test_pip_install_read_only_ipython():
    import tempfile
    from pathlib import Path

    tmp_path = Path(tempfile.mkdtemp(prefix="nbd-pkg-", dir="/tmp"))  # traversable by an unprivileged user
    sys.path.insert(0, ROOT)
    from nbdistributed_amd import _native as N

    target = tmp_path / "site"
    env = dict(os.environ)
    if not N._fresh(N.OPS_LIB, N._ops_deps(), N._ops_salt()):
        env["NBD_SKIP_OPS_BUILD"] = "1"  # (no multi-minute hipcc build inside a unit test)
    # pip builds from a copy of the tree: setuptools writes its build/ and *.egg-info next to
    # setup.py, and the source tree must never be written by a test (a stale build/lib beside the
    # package is a trap).  copy2 keeps mtimes, so the in-tree native libraries stay "fresh".
    src = tmp_path / "src"
    shutil.copytree(ROOT, src, ignore=shutil.ignore_patterns(
        ".git", "build", "gpurun_out", "gpurun_ab", "profiles", "benchmarks", "docs", "tests", "examples",
        "*.egg-info", "__pycache__", ".pytest_cache", ".hypothesis", "*.json", "*.log"))
    p = subprocess.run([sys.executable, "-m", "pip", "install", "--no-build-isolation", "--no-deps", "--target",
                        str(target), str(src)], capture_output=True, text=True, timeout=600, env=env, cwd=str(tmp_path))
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    pkg = target / "nbdistributed_amd"
    assert (pkg / "_native" / "libnbd_transport.so").exists()
    assert (pkg / "_csrc" / "kernels" / "bucket.hip").exists()
    if "NBD_SKIP_OPS_BUILD" not in env:
        assert (pkg / "_native" / "libnbd_ops.so").exists()
    os.chmod(tmp_path, 0o755)
    subprocess.run(["chmod", "-R", "a-w,a+rX", str(target)], check=True)
    before = _snapshot(target)
    kenv = {"PATH": "/usr/bin:/bin", "HOME": "/nonexistent", "PYTHONPATH": str(target),
            "NBD_WORKER_PYTHON": sys.executable, "HSA_ENABLE_IPC_MODE_LEGACY": "0", "NBD_CACHE_DIR": "/nonexistent"}
    cmd = [IPY, "-c", KERNEL]
    if os.geteuid() == 0 and shutil.which("setpriv"):  # root ignores file modes: drop to nobody
        cmd = ["setpriv", "--reuid=65534", "--regid=65534", "--clear-groups"] + cmd
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd="/", env=kenv)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        assert r.stdout.count("allreduce [3.0, 3.0, 3.0, 3.0]") == 2, r.stdout[-3000:]
        assert f"PKG {pkg}/__init__.py" in r.stdout and f"csrc {pkg}/_csrc" in r.stdout
        assert _snapshot(target) == before  # nothing built, locked or written in the install
        if "NBD_SKIP_OPS_BUILD" not in env:
            # the installed ops library is the one a worker would load (source hash, no rebuild)
            r2 = subprocess.run([sys.executable, "-c", "import nbdistributed_amd._native as N; print(N.ops_lib_path())"],
                                capture_output=True, text=True, timeout=120, cwd="/", env=kenv)
            assert r2.stdout.strip() == str(pkg / "_native" / "libnbd_ops.so"), r2.stdout + r2.stderr
    finally:
        subprocess.run(["chmod", "-R", "u+w", str(target)])
        shutil.rmtree(tmp_path, ignore_errors=True)


def test_fresh_detects_added_and_removed_sources(tmp_path):
    """A library is fresh only for the exact source set it was built from: deleting (or adding)
    a source changes the stored hash although no remaining file is newer than the library."""
    import os
    import time

    from nbdistributed_amd import _native as N

    srcs = [tmp_path / f"k{i}.hip" for i in range(3)]
    for i, p in enumerate(srcs):
        p.write_text(f"// kernel {i}\n")
    lib = tmp_path / "libx.so"
    time.sleep(0.01)
    lib.write_bytes(b"\0")
    N._hash_file(lib).write_text(N.source_hash(srcs, "salt") + "\n")
    assert N._fresh(lib, srcs, "salt")
    assert not N._fresh(lib, srcs[:2], "salt")  # a source removed since the build
    extra = tmp_path / "k9.hip"
    extra.write_text("// new\n")
    os.utime(extra, (lib.stat().st_mtime - 10, lib.stat().st_mtime - 10))  # older than the library
    assert not N._fresh(lib, srcs + [extra], "salt")  # a source added since the build
    N._hash_file(lib).unlink()
    assert N._fresh(lib, srcs, "salt")  # no stored hash: the mtimes decide
