"""GPU: per-block HIP graphs for the eager Llama step (ops.block_graphs, csrc/kernels/autograd.hip
namespace ``bg``).  The graphed block runs the eager block's kernels in the same order, so every
loss, gradient and updated parameter must be bit-identical to graphs off — across optimizer steps
(weights change in place under the graph), with DDP bucket gradients and no_sync accumulation, a
second forward before backward (the block is still armed: eager), and inside a whole-step
GraphedStep capture (the outer graph takes the blocks)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

from nbdistributed_amd import ops  # noqa: E402


@pytest.fixture
def dev(require_gpu):
    assert ops.native_available(), ops._load_error
    prev = ops.block_graphs()
    ops.block_graphs_reset()
    yield torch.device("cuda")
    ops.block_graphs(prev)
    ops.block_graphs_reset()


def _model(dev, layers=3, seed=0):
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification

    torch.manual_seed(seed)
    return LlamaForSequenceClassification(LlamaConfig.smollm2_135m(num_hidden_layers=layers)).to(dev, torch.bfloat16)


def _batches(dev, n=4, bs=4, T=128):
    g = torch.Generator(device=dev).manual_seed(1)
    return [(torch.randint(1, 49152, (bs, T), device=dev, generator=g), torch.randint(0, 2, (bs,), device=dev, generator=g))
            for _ in range(n)]


def _train(m, batches, graphs: int, steps=6):
    ops.block_graphs(graphs)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3, foreach=False)
    losses = []
    for i in range(steps):
        ids, lab = batches[i % len(batches)]
        loss = m(ids, torch.ones_like(ids), lab)[0]
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(loss.detach())
    torch.cuda.synchronize()
    return torch.stack(losses), torch.cat([p.detach().float().flatten() for p in m.parameters()])


@pytest.mark.parametrize("mode", [1, 2])
def test_block_graphs_bit_identical_across_steps(dev, mode):
    """Plain training (no DDP slices): mode 2 keeps the backward eager (its weight gradients would
    be static graph memory)."""
    base = _model(dev)
    batches = _batches(dev)
    l0, p0 = _train(copy.deepcopy(base), batches, 0)
    s0 = ops.block_graphs_stats()
    l1, p1 = _train(copy.deepcopy(base), batches, mode)
    s1 = ops.block_graphs_stats()
    assert s1["bwd_replays"] == s0["bwd_replays"]
    assert torch.equal(l0, l1), (l0, l1)
    assert torch.equal(p0, p1)
    # 3 blocks: two eager calls each, one capture each, then replays (the capturing call replays too)
    assert s1["captures"] - s0["captures"] == 3, s1
    assert s1["replays"] - s0["replays"] == 3 * 4, s1
    assert s1["live"] == 3, s1


def test_block_graphs_second_forward_before_backward(dev):
    """Two forwards before one backward: the second finds every block armed (its static memory
    still holds the first pass) and runs eagerly; the summed gradients match graphs off."""
    base = _model(dev, layers=2, seed=3)
    (a, la), (b, lb) = _batches(dev, n=2)

    def grads(graphs):
        ops.block_graphs(graphs)
        m = copy.deepcopy(base)
        for _ in range(3):  # warm + capture
            m(a, torch.ones_like(a), la)[0].backward()
        for p in m.parameters():
            p.grad = None
        e0 = ops.block_graphs_stats()["eager"]
        out_a = m(a, torch.ones_like(a), la)
        out_b = m(b, torch.ones_like(b), lb)
        (out_a[0] + out_b[0]).backward()
        torch.cuda.synchronize()
        return (torch.cat([p.grad.float().flatten() for p in m.parameters()]), out_a[1].float(), out_b[1].float(),
                ops.block_graphs_stats()["eager"] - e0)

    g0, a0, b0, _ = grads(False)
    g1, a1, b1, eager = grads(True)
    assert torch.equal(a0, a1) and torch.equal(b0, b1)
    assert torch.equal(g0, g1)
    assert eager == 2  # the second forward's two blocks


@pytest.mark.parametrize("mode,force", [(1, False), (2, False), (2, True)])
def test_block_graphs_ddp_buckets_and_no_sync(dev, mode, force):
    """DDP bucket gradients (graddst slices), alternating plain and no_sync-accumulated steps: in
    mode 2 the backward graphs replay with both accumulate patterns; force: the N-GPU code path
    (a real RCCL all-reduce per bucket at world size 1) with the recorded deferred reductions."""
    from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
    from nbdistributed_amd.parallel.backend import init_data_plane
    import torch.distributed as dist

    if not dist.is_initialized():
        import os

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        init_data_plane("rccl", 0, 1, dev)
    base = _model(dev, layers=2, seed=5)
    batches = _batches(dev, n=2, bs=8)

    def run(graphs):
        ops.block_graphs(graphs)
        m = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", force_collectives=force)
        outs = []
        for k in (1, 2, 1, 2):
            for p in m.parameters():
                p.grad = None
            for i in range(k):
                ids, lab = batches[i]
                with (m.no_sync() if i < k - 1 else torch.enable_grad()):
                    m(ids, torch.ones_like(ids), lab)[0].backward()
            torch.cuda.synchronize()
            outs.append(torch.cat([b.buffer.float() for b in m.buckets]))
        m.unpatch()
        return outs

    o0 = run(0)
    s0 = ops.block_graphs_stats()
    o1 = run(mode)
    s1 = ops.block_graphs_stats()
    assert all(torch.equal(x, y) for x, y in zip(o0, o1))
    assert s1["replays"] > s0["replays"]
    if mode == 2:  # (k=2 passes: the no_sync pass accumulates, a second backward variant)
        assert s1["bwd_replays"] - s0["bwd_replays"] >= 4, s1
        assert s1["bwd_captures"] - s0["bwd_captures"] >= 2, s1


def test_block_graphs_inside_whole_step_capture(dev):
    """Under graphs.GraphedStep the blocks run inside the outer capture (no nested capture)."""
    from nbdistributed_amd.graphs import GraphedStep

    base = _model(dev, layers=2, seed=7)
    batches = _batches(dev, n=1)

    def run(graphs):
        ops.block_graphs(graphs)
        m = copy.deepcopy(base)
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3, capturable=True, foreach=False)

        def step(x, y):
            loss = m(x, torch.ones_like(x), y)[0]
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=False)
            return loss.detach()

        call = GraphedStep(step, batches[0], warmup=3, optimizers=[opt])
        ls = torch.stack([call(*batches[0]).clone() for _ in range(5)])  # (static output)
        torch.cuda.synchronize()
        return ls, torch.cat([p.detach().float().flatten() for p in m.parameters()])

    l0, p0 = run(False)
    l1, p1 = run(True)
    assert len(set(l0.tolist())) > 1  # the parameters move between replays
    assert torch.equal(l0, l1) and torch.equal(p0, p1)


def test_block_graphs_shape_cap(dev):
    """Each (block, shape) keeps its activations: past 4 sequence lengths a block runs eagerly."""
    base = _model(dev, layers=1, seed=9)
    g = torch.Generator(device=dev).manual_seed(2)
    batches = [torch.randint(1, 49152, (2, T), device=dev, generator=g) for T in (128, 256, 384, 512, 640)]
    lab = torch.tensor([0, 1], device=dev)

    def run(mode):
        ops.block_graphs(mode)
        ops.block_graphs_reset()
        m = copy.deepcopy(base)
        out = []
        for ids in batches:
            for _ in range(3):
                for p in m.parameters():
                    p.grad = None
                loss = m(ids, torch.ones_like(ids), lab)[0]
                loss.backward()
            out.append(torch.cat([loss.detach().view(1)] + [p.grad.float().flatten() for p in m.parameters()]))
        torch.cuda.synchronize()
        return out, ops.block_graphs_stats()["live"]

    o0, _ = run(0)
    o1, live = run(1)
    assert live == 4, live
    assert all(torch.equal(a, b) for a, b in zip(o0, o1))


def test_block_graphs_on_the_hf_swap_path(dev):
    """models.native() (fp32 master weights cast per layer): the cast buffers are kept and
    rewritten in place, so the blocks' bf16 weights keep their addresses and the forward graphs
    replay; losses and updated fp32 weights equal graphs off."""
    transformers = pytest.importorskip("transformers")
    from nbdistributed_amd.models import SMOLLM2_135M, native

    cfg = dict(SMOLLM2_135M)
    cfg.update(num_hidden_layers=2, vocab_size=4096)
    torch.manual_seed(0)
    hf = transformers.LlamaForSequenceClassification(transformers.LlamaConfig(num_labels=2, pad_token_id=0, **cfg))
    state = copy.deepcopy(hf.state_dict())
    g = torch.Generator(device=dev).manual_seed(3)
    ids = torch.randint(1, 4096, (4, 128), device=dev, generator=g)
    lab = torch.tensor([0, 1, 1, 0], device=dev)

    def run(mode):
        ops.block_graphs(mode)
        ops.block_graphs_reset()
        hf.load_state_dict(state)
        m = native(copy.deepcopy(hf).to(dev))  # (native() turns block graphs on for its model)
        assert m.model.block_graphs == 1
        m.model.block_graphs = mode
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
        s0 = ops.block_graphs_stats()
        ls = []
        for _ in range(6):
            out = m(input_ids=ids, attention_mask=torch.ones_like(ids), labels=lab)
            out.loss.backward()
            opt.step()
            opt.zero_grad()
            ls.append(out.loss.detach())
        torch.cuda.synchronize()
        s1 = ops.block_graphs_stats()
        return torch.stack(ls), torch.cat([p.detach().flatten() for p in m.parameters()]), s1["replays"] - s0["replays"]

    l0, p0, _ = run(0)
    l1, p1, replays = run(1)
    assert replays >= 2 * 4, replays
    assert torch.equal(l0, l1) and torch.equal(p0, p1)


def test_block_stack_graph_bit_identical_and_deviation(dev):
    """After the per-block graphs replay steadily, a run of consecutive blocks becomes ONE stack
    graph (one launch per forward); its results equal eager.  A pass that calls the blocks in
    another order drops the stack and still computes the right thing."""
    base = _model(dev, layers=4, seed=11)
    batches = _batches(dev, n=2)

    def run(mode, reorder_at=None):
        ops.block_graphs(mode)
        ops.block_graphs_reset()
        m = copy.deepcopy(base)
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3, foreach=False)
        ls = []
        for i in range(12):
            layers = m.model.layers
            if reorder_at is not None and i == reorder_at:
                # (block 0 unchanged: the stack's head replays; block 1 arrives with another
                # next-norm weight and is not the recorded member -> the stack is dropped)
                m.model.layers = torch.nn.ModuleList([layers[0], layers[1], layers[3], layers[2]])
            ids, lab = batches[i % 2]
            loss = m(ids, torch.ones_like(ids), lab)[0]
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=True)
            m.model.layers = layers
            ls.append(loss.detach())
        torch.cuda.synchronize()
        return torch.stack(ls), torch.cat([p.detach().float().flatten() for p in m.parameters()])

    l0, p0 = run(0)
    s0 = ops.block_graphs_stats()
    l1, p1 = run(1)
    s1 = ops.block_graphs_stats()
    assert torch.equal(l0, l1) and torch.equal(p0, p1)
    assert s1["stack_captures"] - s0["stack_captures"] == 1, s1
    assert s1["stack_replays"] - s0["stack_replays"] >= 4, s1
    assert s1["stack_served"] - s0["stack_served"] >= 3 * 4, s1
    # a pass in another block order (at step 9, after the stack formed): dropped, still exact
    l2, p2 = run(0, reorder_at=9)
    s2 = ops.block_graphs_stats()
    l3, p3 = run(1, reorder_at=9)
    s3 = ops.block_graphs_stats()
    assert torch.equal(l2, l3) and torch.equal(p2, p3)
    assert s3["stacks_dropped"] - s2["stacks_dropped"] >= 1, s3


def test_stack_then_whole_step_graph(dev):
    """Eager steps long enough for a stack graph, then the same model captured whole by
    GraphedStep (block graphs suspended inside): losses and parameters equal the run without
    block graphs — the graph registries hold no autograd history that could leak into the
    capture (the stream hazard of FINDINGS §30)."""
    from nbdistributed_amd.graphs import GraphedStep

    base = _model(dev, layers=2, seed=13)
    batches = _batches(dev, n=1)

    def run(mode):
        ops.block_graphs(mode)
        ops.block_graphs_reset()
        m = copy.deepcopy(base)
        opt = torch.optim.AdamW(m.parameters(), lr=1e-3, capturable=True, foreach=False)

        def step(x, y):
            loss = m(x, torch.ones_like(x), y)[0]
            loss.backward()
            opt.step()
            opt.zero_grad(set_to_none=False)
            return loss.detach()

        ls = [step(*batches[0]).clone() for _ in range(9)]  # eager: per-block graphs, then a stack
        call = GraphedStep(step, batches[0], warmup=2, optimizers=[opt])
        ls += [call(*batches[0]).clone() for _ in range(4)]
        torch.cuda.synchronize()
        return torch.stack(ls), torch.cat([p.detach().float().flatten() for p in m.parameters()])

    l0, p0 = run(0)
    l1, p1 = run(1)
    assert ops.block_graphs_stats()["stack_replays"] >= 1
    assert torch.equal(l0, l1) and torch.equal(p0, p1)
