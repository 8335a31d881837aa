"""GPU: the data plane at every world size this box has — RCCL over xGMI, one rank per GPU.

Parameterised on ``min(torch.cuda.device_count(), 8)`` (skipped below 2 GPUs: RCCL refuses two
ranks on one device): a ``%dist_init``-style session over RCCL runs every check of
``nbdistributed_amd.checks`` — each collective a user types into a cell (all_reduce, broadcast,
all_gather_into_tensor, reduce_scatter_tensor, all_to_all_single, send/recv,
batch_isend_irecv; fp32 and bf16; 1 KiB and 64 MiB) against closed-form values, nbd DDP against
torch DDP (losses and parameter update after 5 steps), the bench recipe's cross-rank sync,
ZeRO-2 against unsharded, the whole step as a HIP graph with RCCL collectives captured against
eager, accelerate's ``Accelerator()`` on the ``"rccl"`` group, and ``%%rank [0]`` build +
broadcast.  Reference: ``/root/reference/README.md:106-124`` (collectives typed into cells),
``src/nbdistributed/worker.py:151`` (the process group every rank gets).

On a one-GPU box the same checks run at world size 1 over RCCL (each collective then has its
world-1 semantics), and two ranks sharing GPU 0 over gloo run the DDP / recipe / %%rank checks.
"""
import pytest

from nbdistributed_amd.checks import run_checks
from nbdistributed_amd.session import Session

pytestmark = pytest.mark.gpu


def _ngpus() -> int:
    try:
        import torch

        return min(torch.cuda.device_count(), 8)
    except Exception:
        return 0


def _run(n, backend, gpu_ids=None, only=None, big=None):
    s = Session(writer=lambda t: None)
    s.start(n, backend=backend, gpu_ids=gpu_ids, startup_timeout=600, timeout=300)
    try:
        out = run_checks(s, gpu=True, big_bytes=big, only=only, log=lambda m: None)
        # the group every rank got: the requested backend, bound to the rank's own device
        r = s.execute("(dist.get_world_size(), dist.get_backend(), str(getattr(dist.group.WORLD, 'bound_device_id', None)),"
                      " str(device))", render=False)
        worlds = {k: r.results[k]["echo"] for k in r.ranks}
    finally:
        s.shutdown()
    return out, worlds


@pytest.mark.parametrize("n", [pytest.param(_ngpus(), id="all_gpus")])
def test_rccl_checks_every_gpu(require_gpu, n):
    if n < 2:
        pytest.skip("needs >= 2 GPUs (RCCL refuses two ranks on one device)")
    out, worlds = _run(n, "rccl", gpu_ids=list(range(n)))
    assert out["passed"], out
    assert out["world_size"] == n
    for rank, echo in worlds.items():
        ws, be, bound, dev = eval(echo)  # noqa: S307 - our own worker's repr of a tuple of str/int
        assert ws == n and be == "rccl" and bound == dev, (rank, echo)


def test_rccl_checks_world1(require_gpu):
    """Every check at world size 1 over RCCL (the driver's one-GPU box): the collectives' world-1
    semantics, the graphed step with its RCCL collectives captured, accelerate on the rccl group."""
    out, worlds = _run(1, "rccl", gpu_ids=[0])
    assert out["passed"], out
    ws, be, bound, dev = eval(worlds[0])  # noqa: S307
    assert ws == 1 and be == "rccl" and bound == dev == "cuda:0"


def test_gloo_two_ranks_on_gpu0_checks(require_gpu):
    """Two ranks sharing GPU 0 over gloo (a one-GPU box's multi-rank rehearsal): the DDP parity,
    recipe / ZeRO-2 and %%rank + broadcast checks with real HIP kernels on both ranks."""
    out, _ = _run(2, "gloo", gpu_ids=[0, 0], only=["ddp", "recipe", "rank_broadcast"])
    assert out["passed"], out
