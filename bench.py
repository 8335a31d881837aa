#!/usr/bin/env python3
"""bench.py — headline benchmark of nbdistributed_amd (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-sweep]

Two launch forms, one measurement:

* **Self-launch** (``python bench.py --gpus N``, no torchrun variables in the environment): this
  process is the notebook kernel.  It never touches the GPU; it starts the N workers with the
  framework's own launcher exactly as ``%dist_init -n N`` does (``Session.start`` →
  ``ProcessManager.start_workers``: one process per GPU, HIP_VISIBLE_DEVICES ordering,
  ``backend="rccl"``), waits a bounded time for every rank's READY and drives the phases as
  ``%%distributed`` cells.  Reference: ``src/nbdistributed/process_manager.py:57-152`` (the
  coordinator spawns its own ranks), ``worker.py:151``.
* **Attach** (the driver's ``python -m torch.distributed.run --nproc-per-node N ... bench.py
  --gpus N``): every torchrun process becomes a framework worker (RANK/WORLD_SIZE/LOCAL_RANK/
  MASTER_* from the environment) and rank 0 also starts the coordinator as a child process that
  never touches the GPU.

Either way rank 0 (or the self-launching kernel) prints exactly ONE JSON line (value = trivial
``%%distributed`` cell p50 round trip in ms, reference 111.6 ms; plus 1 GiB bf16 all_reduce
algbw/busbw and the 1 KiB..1 GiB sweep).  Nothing here may hang silently:

* ranks that do not all reach READY within ``NBD_BENCH_RENDEZVOUS_S`` (default 300 s) produce the
  line with ``"value": null`` and ``"error": "rendezvous: k/N ranks joined"``;
* past ``NBD_BENCH_HARD_S`` (default 540 s) the line is printed from the last checkpointed phase
  with ``"partial": true``;
* the exit status is non-zero whenever the line is partial or carries an error, and 5 when a
  data-plane correctness check (``nbdistributed_amd.checks``: collectives against closed-form
  values, nbd DDP against torch DDP, ZeRO-2, the graphed step, accelerate, ``%%rank`` +
  broadcast) failed — ``"checks_passed"`` / ``"checks"`` in the line say which.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

# bench.py must print its line well inside the driver's 600 s limit: past this many seconds from
# start the measured phases are printed as they stand
HARD_DEADLINE_S = float(os.environ.get("NBD_BENCH_HARD_S", "540"))
# every rank must have reached READY (process up, device bound, RCCL communicator built) by then;
# a fresh box's first `import torch` alone can take 1-2 minutes
RENDEZVOUS_S = float(os.environ.get("NBD_BENCH_RENDEZVOUS_S", "300"))
EXIT_PARTIAL = 3
EXIT_CHECKS = 5  # the line is complete but a data-plane correctness check failed
_T0 = time.monotonic()


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--sweep", action="store_true", default=True, help=argparse.SUPPRESS)  # the default now
    ap.add_argument("--no-sweep", dest="sweep", action="store_false",
                    help="skip the 1 KiB..1 GiB all_reduce bus-bandwidth sweep")
    ap.add_argument("--no-allreduce", action="store_true")
    ap.add_argument("--ar-bytes", type=int, default=1 << 30)
    ap.add_argument("--no-ddp", action="store_true", help="skip the DDP phases (configs 4 and 5)")
    ap.add_argument("--ddp-steps", type=int, default=20)
    ap.add_argument("--no-bcast", action="store_true", help="skip the %%%%rank[0] build + broadcast phase (config 3)")
    ap.add_argument("--no-notebook", action="store_true", help="skip the reference notebook workload (SmolLM2)")
    ap.add_argument("--no-checks", action="store_true", help="skip the data-plane correctness checks")
    ap.add_argument("--backend", default="auto", help="worker backend (auto = rccl on GPUs, gloo on CPU)")
    ap.add_argument("--coordinator", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--endpoint", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--world", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--out", default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def _log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _phases_kw(a) -> dict:
    return dict(allreduce=not a.no_allreduce, sweep=a.sweep, ar_bytes=a.ar_bytes, ddp=not a.no_ddp,
                ddp_steps=a.ddp_steps, bcast=not a.no_bcast, notebook=not a.no_notebook, checks=not a.no_checks)


def _snapshot(out: dict) -> dict:
    """A frozen copy of the phases measured so far (the live dict keeps changing)."""
    return json.loads(json.dumps(out, default=str))


def _session_meta(sess, res: dict) -> dict:
    res = dict(res)
    res["init_ready"] = {r: sess.ready[r].get("init_s") for r in sess.ready}
    res["device"] = sess.ready.get(0, {}).get("gpu_name")
    res["rccl_version"] = sess.ready.get(0, {}).get("rccl_version")
    res["launch"] = "attach (torchrun)" if sess.attached else "self (Session.start, as %dist_init -n N)"
    return res


def _rendezvous_error(sess, world: int, e: BaseException) -> dict:
    f = getattr(sess, "start_failure", None) or {}
    joined, ready = f.get("connected", 0), f.get("ready", 0)
    return {"error": f"rendezvous: {joined}/{world} ranks joined",
            "rendezvous": {"connected": joined, "ready": ready, "world": world, "timeout_s": RENDEZVOUS_S,
                           "detail": f"{type(e).__name__}: {e}"[-800:]}}


class _Printer:
    """Prints the one JSON result line exactly once, from whichever thread gets there first."""

    def __init__(self, world: int, a):
        self.world, self.a = world, a
        # the real stdout, kept aside (an attach-mode worker redirects fd 1 into the control plane)
        self.fd = os.dup(1)
        self.lock = threading.Lock()
        self.done = False

    def emit(self, res, why=None) -> int:
        """Print the line for ``res`` (a run_all result, or {"error": ...}); return the exit code."""
        from nbdistributed_amd.benchmarking import error_line, result_line

        with self.lock:
            if self.done:
                return 0
            res = res or {"error": why or "nothing was measured"}
            if "cell" in res and "p50_ms" in res["cell"]:
                line = result_line(res, self.world, self.a.steps, self.a.warmup)
            else:
                line = error_line(res.get("error") or why or "nothing was measured", self.world, self.a.steps,
                                  self.a.warmup)
                if "rendezvous" in res:
                    line["rendezvous"] = res["rendezvous"]
            for k in ("device", "rccl_version", "launch", "init_ready"):
                if res.get(k) is not None:
                    line[k] = res[k]
            # a failed correctness check makes the run fail (exit status), whatever was timed
            bad = bool(res.get("partial") or why or line.get("error") or line.get("checks_passed") is False)
            if res.get("partial") or why:
                line["partial"] = True
                line["partial_reason"] = why or "coordinator ended before the last phase"
            line["wall_s"] = round(time.monotonic() - _T0, 2)
            sys.stdout.flush()
            os.write(self.fd, (json.dumps(line) + "\n").encode())
            self.done = True
            if bad and line.get("checks_passed") is False and not line.get("partial") and not line.get("error"):
                return EXIT_CHECKS
            return EXIT_PARTIAL if bad else 0


# --------------------------------------------------------------------------- self-launch
def selflaunch_main(a) -> int:
    """``python bench.py --gpus N`` without torchrun: this process is the notebook kernel and
    starts its N workers itself (``%dist_init -n N``).  No GPU call happens in this process."""
    from nbdistributed_amd.benchmarking import run_all
    from nbdistributed_amd.session import Session

    n = a.gpus or 1
    printer = _Printer(n, a)
    sess = Session(writer=lambda s: sys.stderr.write(s))
    state = {"res": None}

    def _watch():
        while time.monotonic() - _T0 < HARD_DEADLINE_S:
            time.sleep(0.5)
            if printer.done:
                return
        _log(f"hard deadline {HARD_DEADLINE_S:.0f}s: printing the phases measured so far")
        code = printer.emit(state["res"] and _session_meta(sess, state["res"]), "hard deadline")
        pm = sess.pm
        if pm is not None:  # the workers live in their own sessions: never leave them behind
            pm.signal_all(signal.SIGKILL)
        sys.stderr.flush()
        os._exit(code or EXIT_PARTIAL)

    threading.Thread(target=_watch, name="nbd-bench-deadline", daemon=True).start()
    try:
        _log(f"self-launch: starting {n} worker(s) (rendezvous limit {RENDEZVOUS_S:.0f}s)")
        try:
            sess.start(n, master_addr="127.0.0.1", backend=a.backend, startup_timeout=RENDEZVOUS_S)
        except Exception as e:  # noqa: BLE001 - reported in the line
            res = _rendezvous_error(sess, n, e)
            _log(res["error"] + f" ({res['rendezvous']['detail'][:300]})")
            return printer.emit(res)
        _log(f"{n} rank(s) ready in {sess.init_s:.1f}s")
        res = run_all(sess, a.steps, a.warmup, checkpoint=lambda out: state.__setitem__("res", _snapshot(out)),
                      **_phases_kw(a))
        return printer.emit(_session_meta(sess, res))
    finally:
        sess.shutdown(graceful=True)


# --------------------------------------------------------------------------- attach (torchrun)
def coordinator_main(a) -> int:
    """Child process of torchrun's rank 0: the notebook-kernel role.  No torch import, no GPU."""
    from nbdistributed_amd.benchmarking import run_all
    from nbdistributed_amd.session import Session

    sess = Session(writer=lambda s: sys.stderr.write(s))

    def write(res, partial):
        res = _session_meta(sess, res)
        res["partial"] = partial
        tmp = a.out + ".tmp"
        with open(tmp, "w") as f:
            json.dump(res, f, default=str)
        os.replace(tmp, a.out)  # rank 0 reads whole files only

    try:
        try:
            sess.attach(a.world, bind=a.endpoint, token=None, startup_timeout=RENDEZVOUS_S)
        except Exception as e:  # noqa: BLE001
            res = _rendezvous_error(sess, a.world, e)
            _log(res["error"])
            with open(a.out + ".tmp", "w") as f:
                json.dump(res, f)
            os.replace(a.out + ".tmp", a.out)
            return EXIT_PARTIAL
        res = run_all(sess, a.steps, a.warmup, checkpoint=lambda out: write(out, True), **_phases_kw(a))
        write(res, False)
        return 0
    finally:
        sess.shutdown(graceful=True)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _read(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def attach_main(a) -> int:
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(_free_port())
    if a.gpus is not None and a.gpus != world:
        print(f"--gpus {a.gpus} disagrees with WORLD_SIZE {world}", file=sys.stderr)
        return 2
    tag = f"{os.environ['MASTER_PORT']}-{os.getuid()}"
    endpoint = f"ipc://{tempfile.gettempdir() if len(tempfile.gettempdir()) < 60 else '/tmp'}/nbd-bench-{tag}.sock"
    out_path = os.path.join(tempfile.gettempdir(), f"nbd-bench-{tag}.json")
    child = None
    if rank == 0:
        try:
            os.unlink(out_path)
        except OSError:
            pass
        # started before this process touches the GPU; a child, never an exec
        cmd = [sys.executable, os.path.abspath(__file__), "--coordinator", "--endpoint", endpoint, "--world", str(world),
               "--steps", str(a.steps), "--warmup", str(a.warmup), "--out", out_path, "--ar-bytes", str(a.ar_bytes),
               "--ddp-steps", str(a.ddp_steps)]
        for flag, on in (("--no-sweep", not a.sweep), ("--no-allreduce", a.no_allreduce), ("--no-ddp", a.no_ddp),
                         ("--no-bcast", a.no_bcast), ("--no-notebook", a.no_notebook), ("--no-checks", a.no_checks)):
            if on:
                cmd.append(flag)
        child = subprocess.Popen(cmd, stdin=subprocess.DEVNULL)
    from nbdistributed_amd import protocol as P
    from nbdistributed_amd.worker import worker_from_env

    w = worker_from_env(endpoint, backend=a.backend, token=None, capture=True)
    w.exit_on_disconnect = True  # the coordinator is bench.py's own child: when it ends, so do we
    printer = _Printer(world, a) if rank == 0 else None
    main_done = threading.Event()

    def _emit_file(why=None) -> int:
        code = printer.emit(_read(out_path), why)
        try:
            os.unlink(out_path)
        except OSError:
            pass
        return code

    if child is not None:
        def _watch():
            # the coordinator ends normally, fails (rendezvous) or outlives the hard deadline; in
            # every case this rank may itself be stuck (in the RCCL rendezvous or a collective):
            # after a grace period print what the coordinator recorded and leave
            while child.poll() is None and time.monotonic() - _T0 < HARD_DEADLINE_S:
                time.sleep(0.5)
            why = None
            if child.poll() is None:
                _log(f"hard deadline {HARD_DEADLINE_S:.0f}s: stopping the coordinator")
                child.kill()
                why = "hard deadline"
            if main_done.wait(float(os.environ.get("NBD_BENCH_GRACE_S", "30"))):
                return
            rc = child.poll()
            code = _emit_file(why or (f"coordinator exit {rc}" if rc else None))
            sys.stdout.flush()
            os._exit(code or (EXIT_PARTIAL if why or rc else 0))

        threading.Thread(target=_watch, name="nbd-bench-deadline", daemon=True).start()
    rc = 0
    stall = os.environ.get("NBD_FAULT_STALL_RANK")
    if stall is not None and int(stall) == rank:  # fault injection (tests): this rank never joins
        time.sleep(float(os.environ.get("NBD_FAULT_STALL_S", "3600")))
        return 4
    try:
        w.connect()
        status = w.bootstrap()
        w.sock.send(P.encode(P.T_READY, w.rank, 0, status))
        w.run()
    finally:
        w.shutdown()  # restores fd 1/2
    if child is None:
        return rc
    try:
        rc = child.wait(timeout=max(5.0, HARD_DEADLINE_S + 40.0 - (time.monotonic() - _T0)))
    except subprocess.TimeoutExpired:
        child.kill()
        rc = -9
    main_done.set()
    code = _emit_file(None if rc == 0 else f"coordinator exit {rc}")
    return code or (EXIT_PARTIAL if rc else 0)


def _under_launcher() -> bool:
    """True when torchrun (or a compatible launcher) started this process as one rank."""
    env = os.environ
    return "RANK" in env and "WORLD_SIZE" in env and ("LOCAL_RANK" in env or "TORCHELASTIC_RUN_ID" in env)


def main(argv=None) -> int:
    a = _args(argv)
    if a.coordinator:
        return coordinator_main(a)
    if not _under_launcher():
        return selflaunch_main(a)
    return attach_main(a)


if __name__ == "__main__":
    code = main()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)
