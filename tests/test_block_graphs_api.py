"""CPU: the per-block graph switch (ops.block_graphs) — modes, the GraphedStep suspension helper,
and that a CPU model is unaffected by it (graphs are a GPU path; tests/test_gpu_block_graphs.py
covers the numerics)."""
import pytest
import torch

from nbdistributed_amd import ops


@pytest.fixture
def native():
    if not ops.native_available():
        pytest.skip("native ops library not built")
    prev = ops.block_graphs()
    yield
    ops.block_graphs(prev)


def test_modes_and_stats(native):
    ops.block_graphs(0)
    assert ops.block_graphs(1) == 0
    assert ops.block_graphs(2) == 1
    assert ops.block_graphs(True) == 2  # True is mode 1
    assert ops.block_graphs(None) == 1
    assert ops.block_graphs(7) == 1     # clamped to 2
    assert ops.block_graphs() == 2
    st = ops.block_graphs_stats()
    assert set(st) == {"captures", "replays", "eager", "live", "bwd_captures", "bwd_replays", "bwd_eager",
                       "stack_captures", "stack_replays", "stack_served", "stacks_dropped"}
    ops.block_graphs_reset()
    assert ops.block_graphs_stats()["live"] == 0


def test_graphed_step_suspends_block_graphs(native):
    from nbdistributed_amd.graphs import _suspend_block_graphs

    ops.block_graphs(2)
    with _suspend_block_graphs():
        assert torch.ops.nbd.llama_block_graphs_suspend(True) is True  # (suspended; stays so)
        assert ops.block_graphs() == 2  # the process mode itself is untouched
    assert torch.ops.nbd.llama_block_graphs_suspend(False) is False
    with pytest.raises(RuntimeError):
        with _suspend_block_graphs():
            raise RuntimeError("step failed")
    assert torch.ops.nbd.llama_block_graphs_suspend(False) is False  # restored on error too


def test_cpu_model_unaffected(native):
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification

    cfg = LlamaConfig.smollm2_135m(num_hidden_layers=2, hidden_size=64, intermediate_size=128,
                                   num_attention_heads=4, num_key_value_heads=2, vocab_size=256)
    torch.manual_seed(0)
    m = LlamaForSequenceClassification(cfg)
    ids = torch.randint(1, 256, (2, 16))
    lab = torch.tensor([0, 1])
    ops.block_graphs(0)
    l0 = m(ids, torch.ones_like(ids), lab)[0]
    ops.block_graphs(2)
    l1 = m(ids, torch.ones_like(ids), lab)[0]
    assert torch.equal(l0, l1)
    assert ops.block_graphs_stats()["live"] == 0
