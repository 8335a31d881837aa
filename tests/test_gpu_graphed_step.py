"""GPU: a GraphedStep whose capture fails leaves the process usable (graphs.py ``_capture``).

``torch.cuda.graph`` leaves its capture stream current when ``capture_end`` raises, so every later
call on the thread ran on a stream that still reported a capture — ``torch.manual_seed`` then
failed.  Seen on the N = 2 bench rehearsal (gloo collectives inside the graph arm: their side
stream's work was never joined, hipErrorStreamCaptureUnjoined), which cost every later arm."""
import pytest
import torch

from nbdistributed_amd.graphs import GraphedStep

pytestmark = pytest.mark.gpu


@pytest.fixture
def dev(require_gpu):
    return torch.device("cuda", 0)


def _after_failure_ok(dev):
    assert not torch.cuda.is_current_stream_capturing()
    torch.manual_seed(1234)  # raised "set_current_seed ... during stream capture" before the fix
    x = torch.randn(1024, device=dev)
    torch.cuda.synchronize()
    assert torch.isfinite(x).all()
    ok = GraphedStep(lambda a: a * 2 + 1, (torch.ones(4, device=dev),), warmup=1)  # a later capture works
    assert torch.equal(ok(torch.full((4,), 3.0, device=dev)), torch.full((4,), 7.0, device=dev))


def test_capture_body_error_restores_stream(dev):
    calls = [0]

    def fn(a):
        calls[0] += 1
        if calls[0] > 1:  # the warm-up call passes, the captured one fails
            raise ValueError("boom inside capture")
        return a + 1

    with pytest.raises(ValueError, match="boom"):
        GraphedStep(fn, (torch.ones(4, device=dev),), warmup=1)
    _after_failure_ok(dev)


def test_capture_unjoined_side_stream_restores_stream(dev):
    side = torch.cuda.Stream()

    def fn(a):
        b = a + 1
        side.wait_stream(torch.cuda.current_stream())  # forked into the capture ...
        with torch.cuda.stream(side):
            c = b * 3                                 # ... and never joined back
        return b, c

    with pytest.raises(Exception):
        GraphedStep(fn, (torch.ones(4, device=dev),), warmup=1)
    _after_failure_ok(dev)
