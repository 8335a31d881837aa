"""Worker fork server: spawn through the zygote, exit codes, pipes, speed."""
import os
import sys
import time

from nbdistributed_amd.session import Session
from nbdistributed_amd.zygote import get_zygote


def test_zygote_spawn_exit_code_and_pipes():
    z = get_zygote(sys.executable)
    assert z.wait_ready(120)
    code = "import sys; print('out-line'); print('err-line', file=sys.stderr); sys.exit(5)"
    # argv for worker.main is irrelevant here: run a tiny program through the same fork path
    p = z.spawn(["--rank", "0", "--world-size", "1", "--coord", "ipc:///nonexistent/x.sock", "--backend", "gloo"],
                dict(os.environ, NBD_STARTUP_TIMEOUT="1"), "/tmp")
    assert p.pid > 0
    # no coordinator at that endpoint: the worker keeps retrying; kill it and see the code
    time.sleep(0.5)
    assert p.poll() is None
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
