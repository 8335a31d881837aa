"""setuptools build for nbdistributed_amd (metadata + native libraries).

``build_py`` additionally
* builds ``libnbd_transport.so`` (g++) and ``libnbd_ops.so`` (hipcc, gfx950; skipped with
  ``NBD_SKIP_OPS_BUILD=1`` or when torch/hipcc are missing — the ops then build on first use into
  ``$NBD_CACHE_DIR``) through ``nbdistributed_amd._native`` (incremental: an up-to-date in-tree
  build is reused);
* copies them into the package with a ``.srchash`` sidecar (installers do not keep mtimes, the
  loader checks the source hash instead);
* copies ``csrc/`` (kernel and transport sources) to ``nbdistributed_amd/_csrc``.

Dependencies follow the reference (``/root/reference/pyproject.toml:28-33``) minus pyzmq: the
control plane is the framework's own C++ ZMTP transport.
"""
import os
import shutil
import sys
from pathlib import Path

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py

ROOT = Path(__file__).resolve().parent


def _version() -> str:
    for line in (ROOT / "nbdistributed_amd" / "__init__.py").read_text().splitlines():
        if line.startswith("__version__"):
            return line.split("=")[1].strip().strip("\"'")
    return "0.0.0"


class BuildPyWithNative(build_py):
    def run(self):
        super().run()
        sys.path.insert(0, str(ROOT))
        from nbdistributed_amd import _native as N

        pkg = Path(self.build_lib) / "nbdistributed_amd"
        dst = pkg / "_native"
        dst.mkdir(parents=True, exist_ok=True)
        libs = [(N.build_transport(), N.TRANSPORT_SOURCES + N.TRANSPORT_HEADERS, N._transport_salt())]
        if os.environ.get("NBD_SKIP_OPS_BUILD") != "1":
            try:
                libs.append((N.build_ops(), N._ops_deps(), N._ops_salt()))
            except Exception as e:  # noqa: BLE001 - the ops build again on first use
                print(f"warning: libnbd_ops.so not prebuilt ({type(e).__name__}: {str(e)[:300]})")
        for lib, deps, salt in libs:
            shutil.copyfile(lib, dst / lib.name)
            os.chmod(dst / lib.name, 0o755)
            (dst / (lib.name + ".srchash")).write_text(N.source_hash(deps, salt) + "\n")
        csrc = pkg / "_csrc"
        for sub in ("kernels", "transport"):
            (csrc / sub).mkdir(parents=True, exist_ok=True)
            for f in (ROOT / "csrc" / sub).iterdir():
                if f.is_file() and f.suffix in (".hip", ".cpp", ".h"):
                    shutil.copyfile(f, csrc / sub / f.name)


setup(
    name="nbdistributed_amd",
    version=_version(),
    description="Interactive distributed PyTorch notebooks, native to AMD MI355X (RCCL over xGMI, gfx950 HIP kernels)",
    long_description=(ROOT / "README.md").read_text(encoding="utf-8"),
    long_description_content_type="text/markdown",
    license="Apache-2.0",
    python_requires=">=3.8",
    packages=find_packages(include=["nbdistributed_amd", "nbdistributed_amd.*"]),
    install_requires=["ipython>=7.16", "torch>=2.1"],
    extras_require={
        "notebook": ["jupyter>=1.0.0"],
        "test": ["pytest>=7.0.0", "pytest-timeout", "pytest-xdist"],
        "models": ["transformers", "accelerate"],
    },
    cmdclass={"build_py": BuildPyWithNative},
    zip_safe=False,
    classifiers=[
        "Development Status :: 3 - Alpha",
        "Intended Audience :: Science/Research",
        "Programming Language :: Python :: 3",
        "Framework :: Jupyter",
        "Topic :: Scientific/Engineering :: Artificial Intelligence",
    ],
)
