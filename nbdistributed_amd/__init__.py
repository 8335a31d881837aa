"""nbdistributed_amd — interactive distributed PyTorch notebooks, native to AMD MI355X.

Same notebook-facing API as the reference ``nbdistributed`` (``%load_ext``, ``%dist_init``,
``%%distributed``, ``%%rank [n]``, ``%sync``, ``%dist_status``, ``%dist_mode``,
``%dist_shutdown``, ``%dist_reset``, ``%dist_debug``, ``%dist_sync_ide``, ``%timeline_*``) on a
new runtime: a native C++ ZMTP/3.1 control plane, one PyTorch-ROCm worker per GPU bound
through HIP_VISIBLE_DEVICES ordering, RCCL over xGMI as the data plane (``backend="rccl"``), and
hand-written gfx950 HIP kernels for the hot path (``nbdistributed_amd.ops``).

Reference entry points: ``src/nbdistributed/__init__.py:7-25``.

Importing this package is cheap and imports neither torch nor IPython, so the same package can
be loaded by a torch-less coordinator kernel and by the workers.
"""
from __future__ import annotations

__version__ = "0.1.0"

_magics = None


def load_ipython_extension(ipython) -> None:
    """``%load_ext nbdistributed_amd``."""
    global _magics
    from .magic import register

    _magics = register(ipython)


def unload_ipython_extension(ipython) -> None:
    """``%unload_ext nbdistributed_amd`` — actually stops the workers (reference D-1)."""
    global _magics
    if _magics is not None:
        _magics.core.teardown()
        _magics = None


def __getattr__(name):
    # lazy public API: nbd.Session, nbd.ops, nbd.parallel, nbd.models ...
    import importlib

    if name in ("Session", "CellResult", "DistributedExecutionError"):
        mod = importlib.import_module(".session", __name__)
        return getattr(mod, name)
    if name in ("ProcessManager",):
        return importlib.import_module(".process_manager", __name__).ProcessManager
    if name in ("CommunicationManager", "Message"):
        return getattr(importlib.import_module(".communication", __name__), name)
    if name in ("ops", "parallel", "models", "utils", "transport", "timeline", "checkpoint", "benchmarking", "guard"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
