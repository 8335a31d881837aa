"""Worker fork server: spawn through the zygote, exit codes, pipes, speed."""
import os
import sys
import time

from nbdistributed_amd.session import Session
from nbdistributed_amd.zygote import get_zygote


def test_zygote_spawn_exit_code_and_pipes():
    z = get_zygote(sys.executable)
    assert z.wait_ready(120)
    # a worker whose bootstrap fails (no rendezvous port) exits with code 3: the code must travel
    # back through the zygote
    p = z.spawn(["--rank", "0", "--world-size", "1", "--coord", "ipc:///nonexistent/x.sock", "--backend", "gloo"],
                dict(os.environ), "/tmp")
    assert p.pid > 0
    assert p.wait(30) == 3
    # a live worker killed from outside reports the signal
    p = z.spawn(["--rank", "0", "--world-size", "2", "--master-addr", "127.0.0.1", "--master-port", "1",
                 "--coord", "ipc:///nonexistent/y.sock", "--backend", "gloo"], dict(os.environ), "/tmp")
    time.sleep(0.3)
    os.killpg(p.pid, 9)
    assert p.wait(10) == -9


def test_session_uses_zygote_and_starts_fast():
    s = Session(writer=lambda t: None)
    s.start(2, backend="gloo")
    s.shutdown()
    s = Session(writer=lambda t: None)
    t = time.perf_counter()
    s.start(2, backend="gloo")
    dt = time.perf_counter() - t
    try:
        assert s.pm.zygote_used
        assert dt < 1.0, dt  # torch is already imported in the forked workers
        r = s.execute("import os\n(os.getpid() != os.getppid(), rank)", render=False)
        assert r.results[1]["output"] == "(True, 1)"
    finally:
        s.shutdown()
