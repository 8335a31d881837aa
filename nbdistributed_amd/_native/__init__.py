"""Builders and loaders for the framework's native code.

Two native artefacts:

* ``libnbd_transport.so`` — the C++17 ZMTP/3.1 DEALER/ROUTER control-plane transport
  (``csrc/transport``).  Plain ``g++``; no GPU, no Python headers (C ABI, loaded with ctypes),
  so the same library serves the PyTorch workers and a torch-less IPython coordinator.
* ``libnbd_ops.so`` — the CDNA4 (gfx950) HIP kernels (``csrc/kernels``) registered as
  ``torch.ops.nbd.*`` through ``TORCH_LIBRARY``; built with ``hipcc --offload-arch=gfx950`` and
  loaded with ``torch.ops.load_library``.

Where they live:

* in a source checkout (``csrc/`` next to the package, package directory writable) they are
  built in-tree, in this directory, so they travel with a repository snapshot;
* an installed package (``pip install .``) ships them prebuilt here, with the sources under
  ``nbdistributed_amd/_csrc``.  The package directory may be read-only: nothing is written
  there at run time.  A library whose sources changed is rebuilt into the writable cache
  ``$NBD_CACHE_DIR`` (default ``~/.cache/nbdistributed_amd``), one sub-directory per source
  hash.

A library is up to date when it is newer than its sources, or when the source hash recorded next
to it at build time (``<lib>.srchash``) matches the sources (installers do not keep mtimes).
"""
from __future__ import annotations

import fcntl
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path
from typing import List, Optional

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
# a checkout keeps csrc/ at the repository root; an installed package carries a copy
CSRC = REPO / "csrc" if (REPO / "csrc" / "kernels").exists() else HERE.parent / "_csrc"

TRANSPORT_NAME = "libnbd_transport.so"
OPS_NAME = "libnbd_ops.so"
TRANSPORT_LIB = HERE / TRANSPORT_NAME
OPS_LIB = HERE / OPS_NAME

TRANSPORT_SOURCES = [CSRC / "transport" / "nbd_transport.cpp"]
TRANSPORT_HEADERS = [CSRC / "transport" / "nbd_transport.h"]

OPS_HIP_SOURCES = sorted((CSRC / "kernels").glob("*.hip")) if (CSRC / "kernels").exists() else []
OPS_CPP_SOURCES = sorted((CSRC / "kernels").glob("*.cpp")) if (CSRC / "kernels").exists() else []
OPS_HEADERS = sorted((CSRC / "kernels").glob("*.h")) if (CSRC / "kernels").exists() else []

GPU_ARCH = os.environ.get("NBD_GPU_ARCH", "gfx950")

# per-source flags.  attn.hip: no SLP vectorisation — beside MFMAs a packed v_pk_{add,mul}_f32
# costs more issue cycles than the two scalar ops it replaces (MI355X_MICROARCH.md, per-instruction
# cycle constants), and the softmax VALU work is what bounds the attention loops.
EXTRA_HIP_FLAGS = {"attn.hip": ["-fno-slp-vectorize"]}


def cache_root() -> Path:
    return Path(os.environ.get("NBD_CACHE_DIR") or Path.home() / ".cache" / "nbdistributed_amd")


def _stale(target: Path, deps: List[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.exists() and d.stat().st_mtime > t for d in deps)


def source_hash(deps: List[Path], salt: str = "") -> str:
    h = hashlib.sha256(salt.encode())
    for d in sorted(deps, key=lambda p: p.name):
        if d.exists():
            h.update(d.name.encode())
            h.update(d.read_bytes())
    return h.hexdigest()[:16]


def _hash_file(lib: Path) -> Path:
    return lib.with_name(lib.name + ".srchash")


def _fresh(lib: Path, deps: List[Path], salt: str) -> bool:
    """Built from exactly these sources: no source newer than the library, and — when the build
    left its source hash — the same set of files (a deleted or added source changes the hash
    without changing any mtime)."""
    if not lib.exists():
        return False
    try:
        stored = _hash_file(lib).read_text().strip()
    except OSError:
        stored = None
    if not _stale(lib, deps):
        return stored is None or stored == source_hash(deps, salt)
    return stored is not None and stored == source_hash(deps, salt)


def _writable(d: Path) -> bool:
    return d.is_dir() and os.access(d, os.W_OK)


def _target(name: str, deps: List[Path], salt: str) -> Path:
    """Where ``name`` is (or is to be built): here if up to date or writable, else the cache."""
    here = HERE / name
    if _fresh(here, deps, salt) or _writable(HERE):
        return here
    d = cache_root() / source_hash(deps, salt)
    d.mkdir(parents=True, exist_ok=True)
    return d / name


class _BuildLock:
    """Cross-process lock so parallel test workers don't race on the same output file."""

    def __init__(self, name: str, where: Path = HERE):
        self.path = where / f".{name}.lock"

    def __enter__(self):
        self.fh = open(self.path, "w")
        fcntl.flock(self.fh, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        fcntl.flock(self.fh, fcntl.LOCK_UN)
        self.fh.close()


def _run(cmd: List[str], env: Optional[dict] = None) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
    if proc.returncode != 0:
        raise RuntimeError(f"native build failed ({proc.returncode}):\n$ {' '.join(cmd)}\n{proc.stdout}")


def _transport_salt(sanitize=None) -> str:
    return f"transport:{sanitize}"


def build_transport(force: bool = False, sanitize: Optional[str] = None, out: Optional[Path] = None) -> Path:
    """Compile libnbd_transport.so (g++, -O2, C++17).  ``sanitize`` = 'thread'|'address' builds
    an instrumented copy at ``out`` (used by the host-side sanitizer tests)."""
    deps = TRANSPORT_SOURCES + TRANSPORT_HEADERS
    salt = _transport_salt()
    target = Path(out) if out else _target(TRANSPORT_NAME, deps, salt)
    if not force and sanitize is None and _fresh(target, deps, salt):
        return target  # no lock, nothing written (read-only installs)
    with _BuildLock("transport", target.parent):
        if not force and sanitize is None and _fresh(target, deps, salt):
            return target
        cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
        cmd = [cxx, "-O2", "-g", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall",
               "-static-libstdc++", "-static-libgcc",
               f"-I{CSRC / 'transport'}"]
        if sanitize:
            cmd += [f"-fsanitize={sanitize}", "-fno-omit-frame-pointer"]
        tmp = target.with_suffix(f".tmp{os.getpid()}.so")
        cmd += ["-o", str(tmp)] + [str(s) for s in TRANSPORT_SOURCES]
        _run(cmd)
        os.replace(tmp, target)
        if sanitize is None:
            _hash_file(target).write_text(source_hash(deps, salt) + "\n")
    return target


def _torch_build_flags() -> tuple:
    import torch
    from torch.utils import cpp_extension

    inc = cpp_extension.include_paths()
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    import sysconfig

    # Python.h: ddp_hooks.cpp calls back into the interpreter (symbols resolve in the host process)
    inc = list(inc) + [sysconfig.get_paths()["include"]]
    cflags = [f"-I{p}" for p in inc] + [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    ldflags = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-ltorch", "-ltorch_cpu", "-lc10_hip", "-ltorch_hip"]
    return cflags, ldflags


def hipcc_path() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    p = Path(rocm) / "bin" / "hipcc"
    return str(p) if p.exists() else (shutil.which("hipcc") or "hipcc")


def _ops_deps() -> List[Path]:
    return OPS_HIP_SOURCES + OPS_CPP_SOURCES + OPS_HEADERS


def _ops_salt() -> str:
    return f"ops:{GPU_ARCH}:{sorted(EXTRA_HIP_FLAGS.items())}"


def ops_lib_path() -> Path:
    """The libnbd_ops.so this process would load (without building anything)."""
    return _target(OPS_NAME, _ops_deps(), _ops_salt())


def build_ops(force: bool = False, jobs: int = 4) -> Path:
    """Compile the gfx950 HIP kernels + TORCH_LIBRARY registrations into libnbd_ops.so.

    Each source is compiled separately (parallel) to an object, then linked.  hipcc
    cross-compiles for gfx950 without a GPU present."""
    deps = _ops_deps()
    salt = _ops_salt()
    target = _target(OPS_NAME, deps, salt)
    if not force and _fresh(target, deps, salt):
        return target  # no lock, nothing written (read-only installs)
    with _BuildLock("ops", target.parent):
        if not force and _fresh(target, deps, salt):
            return target
        cflags, ldflags = _torch_build_flags()
        hipcc = hipcc_path()
        objdir = target.parent / "build"
        objdir.mkdir(exist_ok=True)
        common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC / 'kernels'}", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                  "-Wno-unused-result", "-Wno-deprecated-declarations"] + cflags
        procs = []
        objs = []
        for src in OPS_HIP_SOURCES + OPS_CPP_SOURCES:
            obj = objdir / (src.name + ".o")
            objs.append(obj)
            if not force and not _stale(obj, [src] + OPS_HEADERS):
                continue
            if src.suffix == ".hip":
                cmd = [hipcc, f"--offload-arch={GPU_ARCH}", "-x", "hip", "-c", str(src), "-o", str(obj)] + common
                cmd += EXTRA_HIP_FLAGS.get(src.name, [])
            else:
                cmd = [hipcc, "-c", str(src), "-o", str(obj)] + common
            procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
            if len(procs) >= jobs:
                _wait(procs.pop(0))
        while procs:
            _wait(procs.pop(0))
        tmp = target.with_suffix(f".tmp{os.getpid()}.so")
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={GPU_ARCH}", "-o", str(tmp)] + [str(o) for o in objs] + ldflags)
        os.replace(tmp, target)
        _hash_file(target).write_text(source_hash(deps, salt) + "\n")
    return target


def _wait(item) -> None:
    cmd, proc = item
    out, _ = proc.communicate()
    if proc.returncode != 0:
        raise RuntimeError(f"native build failed ({proc.returncode}):\n$ {' '.join(cmd)}\n{out}")


def build_all(force: bool = False) -> None:
    build_transport(force=force)
    build_ops(force=force)


if __name__ == "__main__":  # python -m nbdistributed_amd._native [--force]
    build_all(force="--force" in sys.argv)
    print(build_transport(), build_ops())
