"""GPU: the one-line swap keeps HF semantics and the block graphs stay a pure
performance feature.

* ``ops.seqcls_prep`` (csrc/kernels/mask.hip) against its PyTorch reference;
* a left-padded batch through ``native()`` (bf16 fused path) matches the fp32 HF model's logits
  and loss, as the right-padded batch does;
* a forward hook on ``layers[3]`` fires on the GPU model and sees HF's activations;
* a backward block-graph capture that fails falls back to the eager backward with eager-equal
  gradients (the claims made while capturing are rolled back);
* dropping one model's block graphs leaves another model's graphs alone;
* the memory the block graphs hold is reported (``ops.block_graphs_memory``)."""
import copy
import gc
import os

import pytest
import torch

from nbdistributed_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture
def dev(require_gpu):
    assert ops.native_available(), ops._load_error
    prev = ops.block_graphs()
    ops.block_graphs_reset()
    yield torch.device("cuda", 0)
    ops.block_graphs(prev)
    ops.block_graphs_reset()


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("dtype", [torch.int64, torch.int32, torch.bool])
def test_seqcls_prep_matches_reference(dev, dtype):
    from nbdistributed_amd.ops.mask import _ref_seqcls_prep

    g = torch.Generator().manual_seed(0)
    B, T = 37, 300
    ids = torch.randint(1, 1000, (B, T), generator=g)
    lens = torch.randint(0, T + 1, (B,), generator=g)
    left = torch.rand(B, generator=g) < 0.5
    ar = torch.arange(T)
    mask = torch.where(left[:, None], ar[None] >= T - lens[:, None], ar[None] < lens[:, None])
    ids = ids * mask
    mask_d = mask.to(dtype)
    for pad in (0, None):
        bad_r = torch.zeros(1, dtype=torch.int32)
        r_ids, r_pool = _ref_seqcls_prep(ids, mask_d, pad, bad_r)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        k_ids, k_pool = ops.seqcls_prep(ids.to(dev), mask_d.to(dev), pad, bad)
        assert torch.equal(k_ids.cpu(), r_ids) and torch.equal(k_pool.cpu(), r_pool)
        assert int(bad.cpu()) == int(bad_r) == 2  # left-padded rows present, no holes
    holes = mask.clone()
    holes[3, :] = True
    holes[3, 7] = False
    bad = torch.zeros(1, dtype=torch.int32, device=dev)
    ops.seqcls_prep(ids.to(dev), holes.to(dev), 0, bad)
    assert int(bad.cpu()) & 1


def _hf_and_native(dev, layers=2):
    transformers = pytest.importorskip("transformers")
    import nbdistributed_amd as nbd
    from nbdistributed_amd.models import SMOLLM2_135M

    cfg = dict(SMOLLM2_135M)
    cfg.update(num_hidden_layers=layers, vocab_size=4096)
    torch.manual_seed(0)
    hf = transformers.LlamaForSequenceClassification(
        transformers.LlamaConfig(num_labels=2, pad_token_id=0, **cfg)).to(dev)
    return hf, nbd.models.native(hf)


def _batch(dev, left: bool, B=4, T=128):
    """The same token rows right-padded, or shifted to the right end (left-padded)."""
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(1, 4096, (B, T), generator=g)
    lens = torch.tensor([T, 100, 57, 9])[:B]
    ar = torch.arange(T)
    mask = ar[None] < lens[:, None]
    ids = ids * mask
    if left:
        ids = torch.stack([torch.roll(ids[b], int(T - lens[b])) for b in range(B)])
        mask = torch.stack([torch.roll(mask[b], int(T - lens[b])) for b in range(B)])
    return ids.to(dev), mask.long().to(dev), torch.tensor([0, 1, 1, 0])[:B].to(dev)


@pytest.mark.parametrize("left", [False, True])
def test_native_padded_batch_matches_hf(dev, left):
    hf, m = _hf_and_native(dev)
    ids, mask, labels = _batch(dev, left)
    assert not m.model.hooked()
    for _ in range(3):  # (block graphs capture after two eager calls: replays too)
        out = m(input_ids=ids, attention_mask=mask, labels=labels)
    ref = hf(input_ids=ids, attention_mask=mask, labels=labels)
    assert _rel(out.logits.float(), ref.logits) < 5e-2, (out.logits, ref.logits)
    assert abs(float(out.loss) - float(ref.loss)) < 3e-2
    if left:  # ... and equal to the same rows right-padded through the fused path
        rids, rmask, _ = _batch(dev, False)
        r = m(input_ids=rids, attention_mask=rmask, labels=labels)
        assert _rel(out.logits.float(), r.logits.float()) < 2e-2


def test_native_mask_with_holes_raises_next_call(dev):
    hf, m = _hf_and_native(dev)
    ids, mask, labels = _batch(dev, False)
    mask[1, 5] = 0
    m(input_ids=ids, attention_mask=mask, labels=labels)
    torch.cuda.synchronize()
    with pytest.raises(ValueError, match="holes"):
        m(input_ids=ids, attention_mask=torch.ones_like(mask), labels=labels)


def test_native_mask_check_sync_raises_on_the_offending_call(dev, monkeypatch):
    """NBD_MASK_CHECK_SYNC=1: the call that gets the bad mask raises (nothing of it applied)."""
    from nbdistributed_amd.models import llama

    monkeypatch.setattr(llama, "_MASK_CHECK_SYNC", True)
    hf, m = _hf_and_native(dev)
    ids, mask, labels = _batch(dev, False)
    m(input_ids=ids, attention_mask=mask, labels=labels)  # a good mask: fine
    mask[1, 5] = 0
    with pytest.raises(ValueError, match="nothing of this batch was applied"):
        m(input_ids=ids, attention_mask=mask, labels=labels)


def test_native_mask_check_follows_graph_replays(dev):
    """A mask check captured into a GraphedStep: a replay on a mask with holes is reported at the
    next replay (the capture-time check alone would never see replayed batches)."""
    from nbdistributed_amd.graphs import GraphedStep

    hf, m = _hf_and_native(dev)
    ids, mask, labels = _batch(dev, False)
    with torch.no_grad():
        g = GraphedStep(lambda i, k: m(input_ids=i, attention_mask=k).logits, (ids, mask), warmup=2)
        g(ids, mask)
        g(ids, mask)
        holes = mask.clone()
        holes[1, 5] = 0
        g(ids, holes)
        torch.cuda.synchronize()
        with pytest.raises(ValueError, match="EARLIER call"):
            g(ids, mask)


def test_native_layer_hook_fires_with_hf_activations(dev):
    hf, m = _hf_and_native(dev, layers=4)
    ids, mask, labels = _batch(dev, True)
    seen = {}

    def grab(tag):
        def hook(mod, args, out):
            seen[tag] = (args[0].detach().float(), out.detach().float())
        return hook

    hs = [hf.model.layers[3].register_forward_hook(grab("hf")), m.model.layers[3].register_forward_hook(grab("nbd"))]
    try:
        ref = hf(input_ids=ids, attention_mask=mask, labels=labels)
        out = m(input_ids=ids, attention_mask=mask, labels=labels)
    finally:
        for h in hs:
            h.remove()
    valid = mask.bool()
    for i in (0, 1):
        assert _rel(seen["nbd"][i][valid], seen["hf"][i][valid]) < 1e-3  # (module path: fp32 compute)
    assert _rel(out.logits.float(), ref.logits) < 1e-3
    assert not m.model.hooked()


def _ddp_step_grads(base, batches, graphs, fail=0):
    from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP

    ops.block_graphs(graphs)
    m = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket")
    outs = []
    for step in range(4):
        if step == 2 and fail:
            torch.ops.nbd.llama_block_graphs_fault(fail)
        for p in m.parameters():
            p.grad = None
        ids, lab = batches[step % len(batches)]
        m(ids, torch.ones_like(ids), lab)[0].backward()
        torch.cuda.synchronize()
        outs.append(torch.cat([b.buffer.float() for b in m.buckets]))
    m.unpatch()
    return outs


def test_backward_capture_failure_falls_back_to_eager(dev):
    """Mode 2 (backward graphs into DDP bucket slices): the first backward capture is forced to
    fail; that step's gradients still equal the eager step's (claims rolled back, eager backward)."""
    import torch.distributed as dist

    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification
    from nbdistributed_amd.parallel.backend import init_data_plane

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        init_data_plane("rccl", 0, 1, dev)
    torch.manual_seed(5)
    base = LlamaForSequenceClassification(LlamaConfig.smollm2_135m(num_hidden_layers=2)).to(dev, torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(1)
    batches = [(torch.randint(1, 49152, (8, 128), device=dev, generator=g), torch.randint(0, 2, (8,), device=dev, generator=g))
               for _ in range(2)]
    ref = _ddp_step_grads(base, batches, 0)
    ops.block_graphs_reset()
    with pytest.warns(UserWarning, match="backward graph capture failed"):
        got = _ddp_step_grads(base, batches, 2, fail=100)
    torch.ops.nbd.llama_block_graphs_fault(0)
    assert all(torch.equal(a, b) for a, b in zip(ref, got))


def test_per_model_graph_reset_and_memory(dev):
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification

    def model(seed):
        torch.manual_seed(seed)
        return LlamaForSequenceClassification(LlamaConfig.smollm2_135m(num_hidden_layers=2)).to(dev, torch.bfloat16)

    ids = torch.randint(1, 49152, (4, 128), device=dev)
    lab = torch.randint(0, 2, (4,), device=dev)
    ops.block_graphs(1)
    keep, throw = model(1), model(2)
    for m in (keep, throw):
        for _ in range(4):
            m(ids, torch.ones_like(ids), lab)[0].backward()
    del m  # (the loop variable would keep `throw` alive)
    torch.cuda.synchronize()
    live = ops.block_graphs_stats()["live"] + ops.block_graphs_stats()["stack_captures"]
    mem = ops.block_graphs_memory()
    assert mem["graphs"] >= 2 and mem["reserved_bytes"] > 0 and mem["reserved_bytes"] >= mem["allocated_bytes"]
    pools_before = mem["graphs"]
    del throw
    gc.collect()
    mem2 = ops.block_graphs_memory()
    assert 0 < mem2["graphs"] < pools_before, (mem, mem2)  # the live model kept its graphs
    r0 = ops.block_graphs_stats()["replays"] + ops.block_graphs_stats()["stack_replays"]
    keep(ids, torch.ones_like(ids), lab)[0].backward()
    r1 = ops.block_graphs_stats()["replays"] + ops.block_graphs_stats()["stack_replays"]
    assert r1 > r0 and live > 0  # replayed, not recaptured from scratch
    del keep
    gc.collect()
    assert ops.block_graphs_memory()["graphs"] == 0


@pytest.mark.parametrize("cast_layers", [None, "1", "3"])
def test_native_graphs_follow_optimizer_updates(dev, cast_layers, monkeypatch):
    """native() with torch AdamW over enough steps for the stack graph (one graph replaying every
    block at the first block's call) to form: block_graphs 0 (eager), 1 and 2 give the same losses
    and gradients at every step.  (The fp32-master path casts each layer's weights; a cast issued
    between two block calls used to land after the stack had read them — one step stale.)  Cast
    nodes of all layers (world size 1), one per layer, and groups of 3 of the 4 layers."""
    transformers = pytest.importorskip("transformers")
    import nbdistributed_amd as nbd
    from nbdistributed_amd.models import SMOLLM2_135M

    if cast_layers:
        monkeypatch.setenv("NBD_NATIVE_CAST_LAYERS", cast_layers)
    cfg = dict(SMOLLM2_135M)
    cfg.update(num_hidden_layers=4, vocab_size=4096)
    torch.manual_seed(0)
    hf = transformers.LlamaForSequenceClassification(
        transformers.LlamaConfig(num_labels=2, pad_token_id=0, **cfg)).to(dev)
    ms = [nbd.models.native(copy.deepcopy(hf), block_graphs=g) for g in (0, 1, 2)]
    opts = [torch.optim.AdamW(m.parameters(), lr=1e-3) for m in ms]
    ids, mask, labels = _batch(dev, False)
    s0 = ops.block_graphs_stats()
    for step in range(12):
        losses, grads = [], []
        for m, o in zip(ms, opts):
            out = m(input_ids=ids, attention_mask=mask, labels=labels)
            out.loss.backward()
            losses.append(float(out.loss.detach()))
            grads.append([p.grad.clone() for p in m.parameters()])
            o.step()
            o.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        assert losses[0] == losses[1] == losses[2], (step, losses)
        for k in (1, 2):
            assert all(torch.equal(a, b) for a, b in zip(grads[0], grads[k])), (step, k)
    s1 = ops.block_graphs_stats()
    assert s1["stack_replays"] > s0["stack_replays"], (s0, s1)  # the stack graph did serve forwards


def test_native_backward_graphs_match_eager_backward(dev):
    """native(..., block_graphs=2): the cast weights' gradients go to kept buffers (graddst), so
    each decoder block's backward is captured and replayed as a HIP graph on the fp32-master path;
    the fp32 gradients equal the eager backward's (block_graphs=1), step after step, and a second
    backward without zero_grad accumulates."""
    transformers = pytest.importorskip("transformers")
    import nbdistributed_amd as nbd
    from nbdistributed_amd.models import SMOLLM2_135M

    cfg = dict(SMOLLM2_135M)
    cfg.update(num_hidden_layers=3, vocab_size=4096)
    torch.manual_seed(0)
    hf = transformers.LlamaForSequenceClassification(
        transformers.LlamaConfig(num_labels=2, pad_token_id=0, **cfg)).to(dev)
    m1 = nbd.models.native(copy.deepcopy(hf), block_graphs=1)
    m2 = nbd.models.native(copy.deepcopy(hf), block_graphs=2)
    ids, mask, labels = _batch(dev, False)
    s0 = ops.block_graphs_stats()
    for step in range(5):
        grads = []
        for m in (m1, m2):
            m.zero_grad(set_to_none=True)
            m(input_ids=ids, attention_mask=mask, labels=labels).loss.backward()
            if step == 4:  # accumulate a second micro-batch
                m(input_ids=ids, attention_mask=mask, labels=labels).loss.backward()
            torch.cuda.synchronize()
            grads.append([p.grad.clone() for p in m.parameters()])
        for a, b in zip(*grads):
            assert torch.equal(a, b), (step, float((a - b).abs().max()))
    s1 = ops.block_graphs_stats()
    assert s1["bwd_captures"] > s0["bwd_captures"] and s1["bwd_replays"] - s0["bwd_replays"] >= 3 * 3, (s0, s1)


def test_native_cast_buffers_reported_and_released(dev):
    """native()'s kept weight casts and their gradient buffers are reported
    (ops.cast_buffers_memory, shown by %dist_status) and released with the model: a re-run
    `model = native(...)` cell does not keep the previous model's buffers."""
    hf, m = _hf_and_native(dev, layers=2)
    ids, mask, labels = _batch(dev, False)
    m(input_ids=ids, attention_mask=mask, labels=labels).loss.backward()
    torch.cuda.synchronize()
    mem = ops.cast_buffers_memory()
    n_bf16 = sum(p.numel() for n, p in m.named_parameters() if ".layers." in n)
    assert mem["groups"] >= 1 and mem["cast_bytes"] >= 2 * n_bf16 and mem["grad_bytes"] >= 2 * n_bf16, mem
    del m, hf
    gc.collect()
    hf2, m2 = _hf_and_native(dev, layers=2)  # the next cast purges the dead model's groups
    m2(input_ids=ids, attention_mask=mask, labels=labels).loss.backward()
    torch.cuda.synchronize()
    mem2 = ops.cast_buffers_memory()  # (bytes of every held group: one model's, not two)
    assert mem2["groups"] == mem["groups"] and mem2["cast_bytes"] == mem["cast_bytes"], (mem, mem2)
    assert mem2["grad_bytes"] == mem["grad_bytes"], (mem, mem2)


def test_fast_adamw_matches_torch_fused_adamw(dev):
    """nbd::adamw_tensors (optim.install_fast_adamw, what native() gives the notebook's AdamW)
    against torch's fused AdamW: 300 parameters (three table launches), odd sizes, two parameter
    groups with their own lr / weight decay, a parameter without a gradient, an LR scheduler;
    parameters and the per-parameter state after 6 steps."""
    from nbdistributed_amd.optim import install_fast_adamw

    torch.manual_seed(5)
    shapes = [(7,), (1000, 3), (33, 65), (4096,), (5, 5, 5)] * 60
    ref = [torch.randn(s, device=dev).requires_grad_() for s in shapes]
    mine = [p.detach().clone().requires_grad_() for p in ref]

    def groups(ps):
        return [{"params": ps[:150], "lr": 3e-3, "weight_decay": 0.1},
                {"params": ps[150:], "lr": 1e-3, "weight_decay": 0.0}]

    oa = torch.optim.AdamW(groups(ref), betas=(0.9, 0.95), eps=1e-6, fused=True)
    ob = torch.optim.AdamW(groups(mine), betas=(0.9, 0.95), eps=1e-6, fused=True)
    assert install_fast_adamw(ob)
    sa = torch.optim.lr_scheduler.LinearLR(oa, 1.0, 0.5, total_iters=6)
    sb = torch.optim.lr_scheduler.LinearLR(ob, 1.0, 0.5, total_iters=6)
    for step in range(6):
        for ps, o, s in ((ref, oa, sa), (mine, ob, sb)):
            for i, p in enumerate(ps):
                p.grad = None if i == 3 else torch.randn(p.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(100 * step + i))
            o.step()
            s.step()
    torch.cuda.synchronize()
    for p, q in zip(ref, mine):
        assert _rel(q, p) < 1e-6
    for p, q in zip(ref, mine):
        if p.grad is None:
            assert len(ob.state[q]) == 0
            continue
        sa_, sb_ = oa.state[p], ob.state[q]
        assert float(sb_["step"]) == float(sa_["step"]) == 6.0
        assert _rel(sb_["exp_avg"], sa_["exp_avg"]) < 1e-6
        assert _rel(sb_["exp_avg_sq"], sa_["exp_avg_sq"]) < 1e-6


def test_native_gives_the_notebook_adamw_the_hip_step(dev, monkeypatch):
    """models.native(): an AdamW built afterwards on the swapped model steps through
    nbd::adamw_tensors (the op runs), and NBD_NATIVE_NBD_ADAMW=0 keeps torch's fused step."""
    from transformers import LlamaConfig as HFConfig, LlamaForSequenceClassification as HFSeqCls

    from nbdistributed_amd.models import native

    cfg = HFConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                   num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=128, num_labels=2,
                   pad_token_id=0)
    torch.manual_seed(0)
    m = native(HFSeqCls(cfg).to(dev))
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    assert getattr(opt, "_nbd_fast_step", False)
    ids = torch.randint(1, 512, (2, 64), device=dev)
    out = m(input_ids=ids, labels=torch.tensor([0, 1], device=dev))
    out.loss.backward()
    opt.step()
    assert all(float(opt.state[p]["step"]) == 1.0 for p in m.parameters() if p.grad is not None)
    monkeypatch.setenv("NBD_NATIVE_NBD_ADAMW", "0")
    opt2 = torch.optim.AdamW(m.parameters(), lr=1e-3)
    assert not getattr(opt2, "_nbd_fast_step", False)
    del m, opt, opt2
    gc.collect()
