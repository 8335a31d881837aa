#!/usr/bin/env python3
"""bench.py — headline benchmark of nbdistributed_amd (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-sweep]

Single GPU (default): this process plays rank 0.  Multi-GPU: launched by the driver as
``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` — every torchrun
process becomes a framework worker in *attach* mode (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* from
the environment, ``backend="rccl"``), and rank 0 additionally starts the coordinator as a child
process that never touches the GPU (exactly what a notebook kernel is).  The coordinator drives
the benchmark as ``%%distributed`` cells through the native control plane; each worker runs them
in its REPL engine with RCCL over xGMI as the data plane.

Printed by rank 0: one JSON line (value = trivial ``%%distributed`` cell p50 round trip in ms,
reference 111.6 ms; plus 1 GiB bf16 all_reduce algbw/busbw).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


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
    ap.add_argument("--coordinator", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--endpoint", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--world", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--out", default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def coordinator_main(a) -> int:
    """Child process: the notebook-kernel role.  No torch import, no GPU."""
    from nbdistributed_amd.benchmarking import run_all
    from nbdistributed_amd.session import Session

    sess = Session(writer=lambda s: sys.stderr.write(s))

    def write(res, partial):
        res = dict(res)
        res["init_ready"] = {r: sess.ready[r].get("init_s") for r in sess.ready}
        res["device"] = sess.ready.get(0, {}).get("gpu_name")
        res["rccl_version"] = sess.ready.get(0, {}).get("rccl_version")
        res["partial"] = partial
        tmp = a.out + ".tmp"
        with open(tmp, "w") as f:
            json.dump(res, f)
        os.replace(tmp, a.out)  # rank 0 reads whole files only

    try:
        sess.attach(a.world, bind=a.endpoint, token=None, startup_timeout=900)
        res = run_all(sess, a.steps, a.warmup, allreduce=not a.no_allreduce, sweep=a.sweep, ar_bytes=a.ar_bytes,
                      ddp=not a.no_ddp, ddp_steps=a.ddp_steps, bcast=not a.no_bcast,
                      notebook=not a.no_notebook, checkpoint=lambda out: write(out, True))
        write(res, False)
        return 0
    finally:
        sess.shutdown(graceful=True)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# bench.py must print its line well inside the driver's 600 s limit: past this many seconds from
# start, rank 0 stops the coordinator and prints what has been measured so far
HARD_DEADLINE_S = float(os.environ.get("NBD_BENCH_HARD_S", "540"))
_T0 = time.monotonic()


class _Emitter:
    """Prints the one JSON result line exactly once, from whichever thread gets there first."""

    def __init__(self, out_path, world, a):
        self.out_path, self.world, self.a = out_path, world, a
        # the real stdout, kept aside before the worker redirects fd 1 into the control plane
        self.fd = os.dup(1)
        self.lock = threading.Lock()
        self.done = False

    def emit(self, why=None) -> bool:
        with self.lock:
            if self.done:
                return True
            try:
                with open(self.out_path) as f:
                    res = json.load(f)
            except (OSError, ValueError):
                return False
            from nbdistributed_amd.benchmarking import result_line

            line = result_line(res, self.world, self.a.steps, self.a.warmup)
            line["device"] = res.get("device")
            line["rccl_version"] = res.get("rccl_version")
            if res.get("partial") or why:
                line["partial"] = True
                line["partial_reason"] = why or "coordinator ended before the last phase"
            sys.stdout.flush()
            os.write(self.fd, (json.dumps(line) + "\n").encode())
            self.done = True
            try:
                os.unlink(self.out_path)
            except OSError:
                pass
            return True


def main(argv=None) -> int:
    a = _args(argv)
    if a.coordinator:
        return coordinator_main(a)
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", str(a.gpus or 1))
    os.environ.setdefault("LOCAL_RANK", os.environ["RANK"])
    os.environ.setdefault("LOCAL_WORLD_SIZE", os.environ["WORLD_SIZE"])
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(_free_port())
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    if a.gpus is not None and a.gpus != world:
        print(f"--gpus {a.gpus} disagrees with WORLD_SIZE {world}", file=sys.stderr)
        return 2
    tag = f"{os.environ['MASTER_PORT']}-{os.getuid()}"
    endpoint = f"ipc://{tempfile.gettempdir() if len(tempfile.gettempdir()) < 60 else '/tmp'}/nbd-bench-{tag}.sock"
    out_path = os.path.join(tempfile.gettempdir(), f"nbd-bench-{tag}.json")
    child = None
    if rank == 0:
        # started before this process touches the GPU; a child, never an exec
        cmd = [sys.executable, os.path.abspath(__file__), "--coordinator", "--endpoint", endpoint, "--world", str(world),
               "--steps", str(a.steps), "--warmup", str(a.warmup), "--out", out_path, "--ar-bytes", str(a.ar_bytes)]
        if not a.sweep:
            cmd.append("--no-sweep")
        if a.no_allreduce:
            cmd.append("--no-allreduce")
        if a.no_ddp:
            cmd.append("--no-ddp")
        if a.no_bcast:
            cmd.append("--no-bcast")
        if a.no_notebook:
            cmd.append("--no-notebook")
        cmd += ["--ddp-steps", str(a.ddp_steps)]
        child = subprocess.Popen(cmd, stdin=subprocess.DEVNULL)
    from nbdistributed_amd import protocol as P
    from nbdistributed_amd.worker import worker_from_env

    w = worker_from_env(endpoint, backend="auto", token=None, capture=True)
    w.exit_on_disconnect = True  # the coordinator is bench.py's own child: when it ends, so do we
    emitter = _Emitter(out_path, world, a) if rank == 0 else None
    if child is not None:
        def _watch():
            # hard deadline: stop the coordinator (the workers see it disconnect and return from
            # run()); if this process is still stuck after a grace period (e.g. inside a
            # collective), print what was measured and leave
            while child.poll() is None and time.monotonic() - _T0 < HARD_DEADLINE_S:
                time.sleep(0.5)
            if child.poll() is None:
                print(f"[bench] hard deadline {HARD_DEADLINE_S:.0f}s: stopping the coordinator", file=sys.stderr,
                      flush=True)
                child.kill()
                time.sleep(float(os.environ.get("NBD_BENCH_GRACE_S", "30")))
                if emitter.emit("hard deadline"):
                    sys.stdout.flush()
                    os._exit(0)

        threading.Thread(target=_watch, name="nbd-bench-deadline", daemon=True).start()
    rc = 0
    try:
        w.connect()
        status = w.bootstrap()
        w.sock.send(P.encode(P.T_READY, w.rank, 0, status))
        w.run()
    finally:
        w.shutdown()  # restores fd 1/2
    if child is not None:
        try:
            rc = child.wait(timeout=max(5.0, HARD_DEADLINE_S + 40.0 - (time.monotonic() - _T0)))
        except subprocess.TimeoutExpired:
            child.kill()
            rc = -9
        if not emitter.emit(None if rc == 0 else f"coordinator exit {rc}"):
            print(f"coordinator failed (exit {rc}) before measuring anything", file=sys.stderr)
            return rc or 1
        return 0
    return rc


if __name__ == "__main__":
    code = main()
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)
