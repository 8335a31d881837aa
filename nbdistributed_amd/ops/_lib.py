"""Loading ``libnbd_ops.so`` (the gfx950 kernels registered as ``torch.ops.nbd.*``)."""
from __future__ import annotations

import os
import threading
from typing import Optional

_lock = threading.Lock()
_loaded: Optional[bool] = None
_load_error: Optional[str] = None


def load_library(build: bool = True) -> bool:
    """Load libnbd_ops.so into this process (building it first if stale and ``build``)."""
    global _loaded, _load_error
    if _loaded is not None:
        return _loaded
    with _lock:
        if _loaded is not None:
            return _loaded
        import torch

        from .._native import OPS_HIP_SOURCES, build_ops, ops_lib_path

        try:
            path = os.environ.get("NBD_OPS_LIB")
            if not path:
                path = str(build_ops()) if build and OPS_HIP_SOURCES else str(ops_lib_path())
            torch.ops.load_library(path)
            _loaded = True
        except Exception as e:  # pragma: no cover - reported by native_available()/_require
            _loaded = False
            _load_error = f"{type(e).__name__}: {e}"
    return _loaded

def native_available() -> bool:
    return load_library()

def _require() -> None:
    if not load_library():
        raise RuntimeError(f"nbdistributed_amd HIP ops unavailable ({_load_error}); "
                           "run `python -m nbdistributed_amd._native` to build libnbd_ops.so")
