"""One place for every tunable, with ``NBD_*`` environment overrides.

The reference has no configuration beyond magic flags and hard-codes its timings
(100 ms display poll ``magic.py:1094``, 10 ms completion poll
``communication.py:358``, 2 s startup sleep ``process_manager.py:137``, 5 s status timeout
``process_manager.py:365``...).  Here none of those sleeps exist (everything is event-driven);
what remains configurable is listed below.
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass, field, fields


def _env(name: str, default, cast=str):
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    if cast is bool:
        return v.lower() in ("1", "true", "yes", "on")
    return cast(v)


@dataclass
class Config:
    # worker launch
    worker_python: str = field(default_factory=lambda: _env("NBD_WORKER_PYTHON", sys.executable))
    zygote: bool = field(default_factory=lambda: _env("NBD_ZYGOTE", True, bool))
    startup_timeout_s: float = field(default_factory=lambda: _env("NBD_STARTUP_TIMEOUT", 600.0, float))
    # transport
    transport: str = field(default_factory=lambda: _env("NBD_TRANSPORT", "ipc"))  # ipc | tcp
    bind_host: str = field(default_factory=lambda: _env("NBD_BIND_HOST", "127.0.0.1"))
    heartbeat_ivl_ms: int = field(default_factory=lambda: _env("NBD_HEARTBEAT_IVL_MS", 1000, int))
    heartbeat_timeout_ms: int = field(default_factory=lambda: _env("NBD_HEARTBEAT_TIMEOUT_MS", 15000, int))
    stream_flush_us: int = field(default_factory=lambda: _env("NBD_STREAM_FLUSH_US", 2000, int))
    # receivers (coordinator and worker main threads, native I/O threads) poll this long before
    # sleeping: a reply within the window costs no futex / epoll wake-up (0 = always sleep)
    spin_us: int = field(default_factory=lambda: _env("NBD_SPIN_US", 200, int))
    # the workers' poll window (-1 = spin_us when the machine has a spare CPU per polling thread)
    worker_spin_us: int = field(default_factory=lambda: _env("NBD_WORKER_SPIN_US", -1, int))
    use_token: bool = field(default_factory=lambda: _env("NBD_TOKEN_AUTH", True, bool))
    # data plane
    backend: str = field(default_factory=lambda: _env("NBD_BACKEND", "auto"))  # auto | rccl | nccl | gloo
    eager_comm_init: bool = field(default_factory=lambda: _env("NBD_EAGER_COMM_INIT", True, bool))
    # interrupt handling: seconds after SIGINT before the worker aborts its communicator
    interrupt_abort_s: float = field(default_factory=lambda: _env("NBD_INTERRUPT_ABORT_S", 10.0, float))
    # REPL echo of tensors: auto | repr | summary
    echo_mode: str = field(default_factory=lambda: _env("NBD_ECHO", "auto"))
    echo_summary_min_numel: int = field(default_factory=lambda: _env("NBD_ECHO_SUMMARY_MIN_NUMEL", 1001, int))
    # namespace -> local proxy sync after %%distributed cells (IDE support)
    ide_sync: bool = field(default_factory=lambda: _env("NBD_IDE_SYNC", True, bool))
    # timeline ring buffer
    timeline_capacity: int = field(default_factory=lambda: _env("NBD_TIMELINE_CAPACITY", 2000, int))
    log_level: str = field(default_factory=lambda: _env("NBD_LOG_LEVEL", "WARNING"))
    # fault injection armed at worker start (faults.py grammar, e.g. "crash:7@1#3")
    faults: str = field(default_factory=lambda: _env("NBD_FAULTS", ""))

    def as_dict(self):
        return {f.name: getattr(self, f.name) for f in fields(self)}


_logging_configured = False


def get_config() -> Config:
    global _logging_configured
    cfg = Config()
    if not _logging_configured:
        import logging

        logger = logging.getLogger("nbdistributed_amd")
        logger.setLevel(getattr(logging, cfg.log_level.upper(), logging.WARNING))
        if not logger.handlers:
            h = logging.StreamHandler()
            h.setFormatter(logging.Formatter("[nbd %(levelname)s %(name)s] %(message)s"))
            logger.addHandler(h)
            logger.propagate = False
        _logging_configured = True
    return cfg
