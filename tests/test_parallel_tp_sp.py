"""Tensor, sequence, expert and pipeline parallelism (parallel/tensor.py, sequence.py, expert.py,
pipeline.py) vs the unsharded single-process computation — CPU/gloo, 2 and 4 ranks (world 1 for
the degenerate path)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, n):
    port = _port()
    mp.spawn(_entry, args=(fn, n, port), nprocs=n, join=True)


def _entry(rank, fn, n, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    try:
        fn(rank, n)
        # every rank done before any tears its gloo pairs down: a peer closing its sockets while
        # another still exchanges made gloo's I/O thread call std::terminate (SIGABRT, ~1 run in 6)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _close(a, b, tol=2e-5):
    assert a.shape == b.shape, (a.shape, b.shape)
    err = (a - b).abs().max().item()
    assert err <= tol * max(1.0, b.abs().max().item()), err


def _tp_linear_case(rank, n):
    from nbdistributed_amd.parallel.tensor import ColumnParallelLinear, RowParallelLinear

    torch.manual_seed(0)
    l1, l2 = torch.nn.Linear(16, 32), torch.nn.Linear(32, 8)
    x = torch.randn(4, 5, 16, requires_grad=True)
    ref = l2(torch.relu(l1(x)))
    ref.square().sum().backward()
    c = ColumnParallelLinear.from_linear(l1)
    r = RowParallelLinear.from_linear(l2)
    xs = x.detach().clone().requires_grad_()
    y = r(torch.relu(c(xs)))
    _close(y, ref)
    y.square().sum().backward()
    _close(xs.grad, x.grad)
    sl = slice(rank * 32 // n, (rank + 1) * 32 // n)
    _close(c.weight.grad, l1.weight.grad[sl])
    _close(c.bias.grad, l1.bias.grad[sl])
    _close(r.weight.grad, l2.weight.grad[:, sl])
    _close(r.bias.grad, l2.bias.grad)
    # gather_output / input_is_parallel=False round trip
    c2 = ColumnParallelLinear.from_linear(l1, gather_output=True)
    r2 = RowParallelLinear.from_linear(l2, input_is_parallel=False)
    xs2 = x.detach().clone().requires_grad_()
    y2 = r2(torch.relu(c2(xs2)))
    _close(y2, ref)
    y2.square().sum().backward()
    _close(xs2.grad, x.grad)


def _tp_gpt2_case(rank, n):
    from nbdistributed_amd.models import GPT2, GPT2Config
    from nbdistributed_amd.parallel.tensor import parallelize_gpt2

    torch.manual_seed(0)
    cfg = GPT2Config(vocab_size=96, n_positions=32, n_embd=32, n_layer=2, n_head=4)
    ref = GPT2(cfg)
    tp = GPT2(cfg)
    tp.load_state_dict(ref.state_dict())
    parallelize_gpt2(tp)
    idx = torch.randint(0, 96, (2, 16), generator=torch.Generator().manual_seed(1))
    _, l_ref = ref(idx, idx)
    _, l_tp = tp(idx, idx)
    _close(l_tp, l_ref, 1e-5)
    l_ref.backward()
    l_tp.backward()
    C, H = 32, 4
    D, Hl = C // H, H // n
    heads = torch.arange(rank * Hl * D, (rank + 1) * Hl * D)
    rows = torch.cat([heads + i * C for i in range(3)])
    hid = slice(rank * 4 * C // n, (rank + 1) * 4 * C // n)
    for b_ref, b_tp in zip(ref.h, tp.h):
        _close(b_tp.attn.c_attn.weight.grad, b_ref.attn.c_attn.weight.grad[rows], 1e-4)
        _close(b_tp.attn.c_attn.bias.grad, b_ref.attn.c_attn.bias.grad[rows], 1e-4)
        _close(b_tp.attn.c_proj.weight.grad, b_ref.attn.c_proj.weight.grad[:, heads], 1e-4)
        _close(b_tp.attn.c_proj.bias.grad, b_ref.attn.c_proj.bias.grad, 1e-4)
        _close(b_tp.mlp.c_fc.weight.grad, b_ref.mlp.c_fc.weight.grad[hid], 1e-4)
        _close(b_tp.mlp.c_proj.weight.grad, b_ref.mlp.c_proj.weight.grad[:, hid], 1e-4)
        _close(b_tp.ln_1.weight.grad, b_ref.ln_1.weight.grad, 1e-4)
    _close(tp.wte.weight.grad, ref.wte.weight.grad, 1e-4)


def _ulysses_case(rank, n):
    import torch.nn.functional as F

    from nbdistributed_amd.parallel.sequence import (gather_sequence, head_to_seq, seq_to_head, shard_sequence,
                                                     ulysses_attention)

    torch.manual_seed(0)
    B, H, Hkv, T, D = 2, 4, 2, 16, 8
    q = torch.randn(B, H, T, D, requires_grad=True)
    k = torch.randn(B, Hkv, T, D, requires_grad=True)
    v = torch.randn(B, Hkv, T, D, requires_grad=True)
    w = torch.randn(B, H, T, D)
    for causal in (True, False):
        for t in (q, k, v):
            t.grad = None
        ref = F.scaled_dot_product_attention(q, k, v, is_causal=causal, enable_gqa=True)
        (ref * w).sum().backward()
        ql, kl, vl = (shard_sequence(t.detach(), dim=2).clone().requires_grad_() for t in (q, k, v))
        out = ulysses_attention(ql, kl, vl, causal=causal)
        _close(out, shard_sequence(ref.detach(), dim=2), 1e-5)
        (out * shard_sequence(w, dim=2)).sum().backward()
        _close(ql.grad, shard_sequence(q.grad, dim=2), 1e-5)
        _close(kl.grad, shard_sequence(k.grad, dim=2), 1e-5)
        _close(vl.grad, shard_sequence(v.grad, dim=2), 1e-5)
        _close(gather_sequence(out, dim=2), ref.detach(), 1e-5)
    # the two all-to-alls are inverses
    x = torch.randn(B, H, T // n, D)
    _close(head_to_seq(seq_to_head(x)), x, 0)


def _tp_generate_case(rank, n):
    # tensor-parallel generation: heads / MLP features and the KV cache split over the ranks, one
    # all-reduce per half block — the same tokens as one process, decode logits to fp32 rounding
    from nbdistributed_amd.generation import KVCache
    from nbdistributed_amd.models import GPT2, GPT2Config
    from nbdistributed_amd.parallel.tensor import parallelize_gpt2

    torch.manual_seed(0)
    ref = GPT2(GPT2Config(vocab_size=256, n_positions=128, n_embd=64, n_layer=2, n_head=4)).eval()
    with torch.no_grad():
        ref.wte.weight.mul_(8.0)  # peaked logits: greedy tokens far from ties
    import copy

    tp = parallelize_gpt2(copy.deepcopy(ref))
    ids = torch.randint(1, 256, (2, 9), generator=torch.Generator().manual_seed(1))
    lens = torch.tensor([9, 5])
    want = ref.generate(ids, 7, lengths=lens)
    got = tp.generate(ids, 7, lengths=lens)
    assert torch.equal(got, want), (got, want)
    assert tp.kv_layout()[1] == 4 // n
    c_ref, c_tp = KVCache.for_model(ref, 2, 16), KVCache.for_model(tp, 2, 16)
    ref.prefill(ids[:, :5], c_ref, torch.tensor([5, 5]))
    tp.prefill(ids[:, :5], c_tp, torch.tensor([5, 5]))
    for t in range(5, 9):
        p = torch.full((2,), t)
        _close(tp.decode_step(ids[:, t], p, c_tp), ref.decode_step(ids[:, t], p, c_ref), tol=1e-4)


def _tp_llama_case(rank, n):
    # Llama-family TP (GQA heads split by kv group, SwiGLU features split, biased q|k|v like Qwen2):
    # loss and gradients = the unsharded model; generation = the unsharded model's tokens
    import copy

    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForCausalLM
    from nbdistributed_amd.parallel.tensor import parallelize_llama

    torch.manual_seed(0)
    ref = LlamaForCausalLM(LlamaConfig.tiny(hidden_size=128, num_attention_heads=4, num_key_value_heads=2,
                                            qkv_bias=True))
    with torch.no_grad():
        for layer in ref.model.layers:
            layer.self_attn.qkv_proj.bias.normal_(0, 0.3)
    tp = parallelize_llama(copy.deepcopy(ref))
    ids = torch.randint(1, 512, (2, 12), generator=torch.Generator().manual_seed(2))
    l_ref, _ = ref(ids, labels=ids)
    l_tp, _ = tp(ids, labels=ids)
    _close(l_tp.detach(), l_ref.detach())
    l_ref.backward()
    l_tp.backward()
    inter = ref.config.intermediate_size
    sl = slice(rank * inter // n, (rank + 1) * inter // n)
    _close(tp.model.layers[0].mlp.gate_up_proj.weight.grad[: inter // n], ref.model.layers[0].mlp.gate_up_proj.weight.grad[sl])
    _close(tp.model.embed_tokens.weight.grad, ref.model.embed_tokens.weight.grad)
    ref.eval(), tp.eval()
    with torch.no_grad():
        ref.model.embed_tokens.weight.mul_(8.0)
        tp.model.embed_tokens.weight.mul_(8.0)
    lens = torch.tensor([12, 6])
    assert torch.equal(tp.generate(ids, 6, lengths=lens), ref.generate(ids, 6, lengths=lens))
    assert tp.kv_layout()[1:3] == (4 // n, 2 // n)


@pytest.mark.parametrize("case", [_tp_linear_case, _tp_gpt2_case, _ulysses_case, _tp_generate_case, _tp_llama_case],
                         ids=["tp_linear", "tp_gpt2", "ulysses", "tp_generate", "tp_llama"])
def test_two_ranks(case):
    _spawn(case, 2)


def test_single_process_is_identity():
    """Without an initialised process group every wrapper degenerates to the plain op."""
    assert not dist.is_initialized()
    _tp_linear_case(0, 1)
    _ulysses_case(0, 1)


def _moe_case(rank, n):
    import torch.nn.functional as F

    from nbdistributed_amd.parallel.expert import MoE

    C, Hd, E, k, N = 16, 32, 4, 2, 24
    torch.manual_seed(0)
    moe = MoE(C, Hd, E, top_k=k)
    g = torch.Generator().manual_seed(7)
    X = torch.randn(n, N, C, generator=g)       # every rank's tokens, identical everywhere
    W = torch.randn(n, N, C, generator=g)
    x = X[rank].clone().requires_grad_()
    out = moe(x)
    (out * W[rank]).sum().backward()
    assert moe.aux_loss is not None and torch.isfinite(moe.aux_loss)

    # dense single-process reference over all ranks' tokens with the full expert set
    def full(p):
        if n == 1:
            return p.detach().clone()
        parts = [torch.empty_like(p) for _ in range(n)]
        dist.all_gather(parts, p.detach().contiguous())
        return torch.cat(parts)
    w1 = full(moe.w1).requires_grad_()
    w2 = full(moe.w2).requires_grad_()
    router = moe.router.weight.detach().clone().requires_grad_()
    Xr = X.reshape(-1, C).clone().requires_grad_()
    probs = F.softmax(Xr @ router.t(), -1)
    gates, idx = probs.topk(k, -1)
    gates = gates / gates.sum(-1, keepdim=True)
    ref = torch.zeros_like(Xr)
    for j in range(k):
        for e in range(E):
            m = idx[:, j] == e
            h = F.gelu(Xr[m] @ w1[e].t(), approximate="tanh") @ w2[e].t()
            ref = ref.index_add(0, m.nonzero().squeeze(1), h * gates[m, j:j + 1])
    (ref * W.reshape(-1, C)).sum().backward()
    _close(out, ref.detach().view(n, N, C)[rank], 1e-5)
    _close(x.grad, Xr.grad.view(n, N, C)[rank], 1e-5)
    sl = slice(rank * E // n, (rank + 1) * E // n)
    _close(moe.w1.grad, w1.grad[sl], 1e-5)
    _close(moe.w2.grad, w2.grad[sl], 1e-5)
    rg = moe.router.weight.grad.clone()
    if n > 1:
        dist.all_reduce(rg)
    _close(rg, router.grad, 1e-5)


def test_moe_two_ranks():
    _spawn(_moe_case, 2)


def test_moe_single_process():
    _moe_case(0, 1)


def _pipe_model():
    torch.manual_seed(0)
    layers = []
    for _ in range(4):
        layers += [torch.nn.Linear(12, 12), torch.nn.Tanh()]
    return torch.nn.Sequential(*layers)


def _pipeline_case(rank, n, schedule="1f1b"):
    from nbdistributed_amd.parallel.pipeline import pipeline_step, split_sequential

    M, mb = 6, 3
    full = _pipe_model()
    g = torch.Generator().manual_seed(3)
    X, Y = torch.randn(M * mb, 12, generator=g), torch.randn(M * mb, 12, generator=g)
    torch.nn.functional.mse_loss(full(X), Y).backward()
    stage = split_sequential(_pipe_model(), n, rank)
    xs, ys = list(X.chunk(M)), list(Y.chunk(M))
    loss = pipeline_step(stage, xs if rank == 0 else None, ys if rank == n - 1 else None,
                         torch.nn.functional.mse_loss, M, (mb, 12), schedule=schedule)
    if rank == n - 1:
        _close(loss, torch.nn.functional.mse_loss(full(X), Y).detach(), 1e-5)
    else:
        assert loss is None
    # the stage holds copies of a contiguous run of layers: match them by position
    full_layers = list(full)
    stage_layers = list(stage)
    for k0 in range(len(full_layers) - len(stage_layers) + 1):
        if all(type(a) is type(b) and all(torch.equal(pa, pb) for pa, pb in zip(a.parameters(), b.parameters()))
               for a, b in zip(full_layers[k0:], stage_layers)):
            break
    else:
        raise AssertionError("stage layers not found in the full model")
    for a, b in zip(full_layers[k0:], stage_layers):
        for pa, pb in zip(a.parameters(), b.parameters()):
            _close(pb.grad, pa.grad, 1e-5)


def _pipeline_gpipe_case(rank, n):
    _pipeline_case(rank, n, "gpipe")


@pytest.mark.parametrize("n", [2, 4])
@pytest.mark.parametrize("case", [_pipeline_case, _pipeline_gpipe_case], ids=["1f1b", "gpipe"])
def test_pipeline_schedules(case, n):
    _spawn(case, n)


def test_split_sequential_balanced():
    from nbdistributed_amd.parallel.pipeline import split_sequential

    m = _pipe_model()
    parts = [split_sequential(m, 4, s) for s in range(4)]
    assert sum(len(p) for p in parts) == len(m)
    assert all(len(p) == 2 for p in parts)
    assert len(split_sequential(m, 1, 0)) == len(m)


def _ring_case(rank, n):
    import torch.nn.functional as F

    from nbdistributed_amd.parallel.context import gather_context, ring_attention, shard_context

    torch.manual_seed(0)
    B, H, Hkv, T, D = 2, 4, 2, 16, 8
    q = torch.randn(B, H, T, D, requires_grad=True)
    k = torch.randn(B, Hkv, T, D, requires_grad=True)
    v = torch.randn(B, Hkv, T, D, requires_grad=True)
    w = torch.randn(B, H, T, D)
    for layout in ("contiguous", "zigzag"):
        for causal in (True, False):
            for t in (q, k, v):
                t.grad = None
            ref = F.scaled_dot_product_attention(q, k, v, is_causal=causal, enable_gqa=True)
            (ref * w).sum().backward()
            sh = lambda t: shard_context(t, dim=2, layout=layout)  # noqa: E731
            ql, kl, vl = (sh(t.detach()).clone().requires_grad_() for t in (q, k, v))
            out = ring_attention(ql, kl, vl, causal=causal, layout=layout)
            _close(out, sh(ref.detach()), 1e-5)
            (out * sh(w)).sum().backward()
            _close(ql.grad, sh(q.grad), 1e-5)
            _close(kl.grad, sh(k.grad), 1e-5)
            _close(vl.grad, sh(v.grad), 1e-5)
            _close(gather_context(out, dim=2, layout=layout), ref.detach(), 1e-5)


@pytest.mark.parametrize("n", [2, 4])
def test_ring_attention(n):
    """parallel.context: ring attention (contiguous and zigzag layouts, causal and full, GQA) —
    outputs and q/k/v gradients = attention on the gathered sequence."""
    _spawn(_ring_case, n)


def test_ring_attention_single_process():
    _ring_case(0, 1)


def _cp_gpt2_case(rank, n):
    from nbdistributed_amd.models import GPT2, GPT2Config
    from nbdistributed_amd.parallel.context import parallelize_gpt2_context, shard_context

    for layout in ("contiguous", "zigzag"):
        torch.manual_seed(0)
        c = GPT2Config(vocab_size=128, n_positions=32, n_embd=32, n_layer=2, n_head=4)
        ref = GPT2(c)
        cp = GPT2(c)
        cp.load_state_dict(ref.state_dict())
        parallelize_gpt2_context(cp, layout=layout)
        idx = torch.randint(0, 128, (2, 32), generator=torch.Generator().manual_seed(1))
        tgt = torch.randint(0, 128, (2, 32), generator=torch.Generator().manual_seed(2))
        tgt[0, :11] = -100  # ignored targets spread unevenly over the shards
        tgt[1, 27:] = -100
        _, loss_ref = ref(idx, tgt)
        loss_ref.backward()
        _, loss = cp(shard_context(idx, dim=1, layout=layout), shard_context(tgt, dim=1, layout=layout))
        loss.backward()
        tot = loss.detach().clone()
        dist.all_reduce(tot)
        _close(tot / n, loss_ref.detach(), 1e-5)
        for (name, p), (_, pr) in zip(cp.named_parameters(), ref.named_parameters()):
            g = p.grad.clone()
            dist.all_reduce(g)
            _close(g / n, pr.grad, 1e-4)


@pytest.mark.parametrize("n", [2, 4])
def test_context_parallel_gpt2(n):
    """parallel.context.parallelize_gpt2_context: every rank trains on its shard of each sequence
    (global positions, ring attention); averaged losses and gradients = the unsplit model's."""
    _spawn(_cp_gpt2_case, n)


def _cp_llama_case(rank, n):
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaModel
    from nbdistributed_amd.parallel.context import parallelize_llama_context, shard_context

    for layout in ("contiguous", "zigzag"):
        torch.manual_seed(0)
        c = LlamaConfig.tiny(vocab_size=64, hidden_size=64, intermediate_size=128, num_attention_heads=4,
                             num_key_value_heads=2)
        ref = LlamaModel(c)
        cp = LlamaModel(c)
        cp.load_state_dict(ref.state_dict())
        parallelize_llama_context(cp, layout=layout)
        ids = torch.randint(0, 64, (2, 32), generator=torch.Generator().manual_seed(1))
        w = torch.randn(2, 32, 64, generator=torch.Generator().manual_seed(2))
        h_ref = ref(ids)
        (h_ref * w).sum().backward()
        h = cp(shard_context(ids, dim=1, layout=layout))
        _close(h, shard_context(h_ref.detach(), dim=1, layout=layout), 1e-4)
        (h * shard_context(w, dim=1, layout=layout)).sum().backward()
        for (name, p), (_, pr) in zip(cp.named_parameters(), ref.named_parameters()):
            g = p.grad.clone()
            dist.all_reduce(g)
            _close(g, pr.grad, 1e-4)


def _cp_llama_causal_case(rank, n):
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForCausalLM
    from nbdistributed_amd.parallel.context import parallelize_llama_context, shard_context, shift_labels

    for layout in ("contiguous", "zigzag"):
        torch.manual_seed(0)
        c = LlamaConfig.tiny(vocab_size=64, hidden_size=64, intermediate_size=128, num_attention_heads=4,
                             num_key_value_heads=2)
        ref = LlamaForCausalLM(c)
        cp = LlamaForCausalLM(c)
        cp.load_state_dict(ref.state_dict())
        parallelize_llama_context(cp, layout=layout)
        ids = torch.randint(0, 64, (2, 32), generator=torch.Generator().manual_seed(1))
        labels = ids.clone()
        labels[0, :13] = -100  # prompt tokens not trained on: uneven counts per shard
        loss_ref, _ = ref(ids, labels)
        loss_ref.backward()
        sh = lambda t: shard_context(t, dim=1, layout=layout)  # noqa: E731
        loss, _ = cp(sh(ids), sh(shift_labels(labels)))
        loss.backward()
        tot = loss.detach().clone()
        dist.all_reduce(tot)
        _close(tot / n, loss_ref.detach(), 1e-5)
        for (name, p), (_, pr) in zip(cp.named_parameters(), ref.named_parameters()):
            g = p.grad.clone()
            dist.all_reduce(g)
            _close(g / n, pr.grad, 1e-4)


@pytest.mark.parametrize("n", [2, 4])
def test_context_parallel_llama_causal_lm(n):
    """parallel.context + LlamaForCausalLM: labels shifted on the full sequence before sharding
    (the zigzag chunk boundaries keep their real next-token targets), loss normalised by the
    group-wide token count — averaged loss and gradients = the unsplit model's, with unevenly
    ignored targets."""
    _spawn(_cp_llama_causal_case, n)


def test_context_parallel_refuses_unsupported_models():
    from nbdistributed_amd.models import GPT2, GPT2Config
    from nbdistributed_amd.models.llama import LlamaConfig, LlamaForSequenceClassification
    from nbdistributed_amd.parallel.context import parallelize_gpt2_context, parallelize_llama_context, shift_labels

    with pytest.raises(TypeError):
        parallelize_llama_context(LlamaForSequenceClassification(LlamaConfig.tiny(num_hidden_layers=1)))
    with pytest.raises(ValueError):
        parallelize_gpt2_context(GPT2(GPT2Config(vocab_size=64, n_positions=32, n_embd=32, n_layer=1, n_head=2,
                                                 dropout=0.1)))
    assert shift_labels(torch.tensor([[1, 2, 3]])).tolist() == [[2, 3, -100]]


@pytest.mark.parametrize("n", [2, 4])
def test_context_parallel_llama(n):
    """parallel.context.parallelize_llama_context: RoPE at global positions + GQA ring attention;
    hidden states = the shard of the unsplit model's, summed gradients = its gradients."""
    _spawn(_cp_llama_case, n)


def _mesh_dp_cp_case(rank, n):
    from nbdistributed_amd.models import GPT2, GPT2Config
    from nbdistributed_amd.parallel import ParallelMesh
    from nbdistributed_amd.parallel.context import parallelize_gpt2_context, shard_context

    mesh = ParallelMesh(dp=2, cp=2)
    assert mesh.members("cp") == [2 * (rank // 2), 2 * (rank // 2) + 1]
    assert mesh.members("dp") == [rank % 2, rank % 2 + 2]
    assert mesh.coord("cp") == rank % 2 and mesh.coord("dp") == rank // 2
    torch.manual_seed(0)
    c = GPT2Config(vocab_size=128, n_positions=32, n_embd=32, n_layer=2, n_head=4)
    ref = GPT2(c)
    cp = GPT2(c)
    cp.load_state_dict(ref.state_dict())
    parallelize_gpt2_context(cp, group=mesh.group("cp"), layout="zigzag")
    idx = torch.randint(0, 128, (4, 32), generator=torch.Generator().manual_seed(1))
    tgt = torch.randint(0, 128, (4, 32), generator=torch.Generator().manual_seed(2))
    _, loss_ref = ref(idx, tgt)  # the global batch, full sequences
    loss_ref.backward()
    d = mesh.coord("dp")
    mine = lambda t: shard_context(t[2 * d:2 * d + 2], group=mesh.group("cp"), dim=1, layout="zigzag")  # noqa: E731
    _, loss = cp(mine(idx), mine(tgt))
    loss.backward()
    for (_, p), (_, pr) in zip(cp.named_parameters(), ref.named_parameters()):
        g = p.grad.clone()
        dist.all_reduce(g)  # DP x CP: average over all four ranks
        _close(g / 4, pr.grad, 1e-4)


def test_mesh_dp_x_cp_gpt2():
    """parallel.mesh.ParallelMesh(dp=2, cp=2) on 4 ranks: group membership, and GPT-2 with the batch
    split over dp and each sequence ring-attended over cp = the single-process model's gradients."""
    _spawn(_mesh_dp_cp_case, 4)


def test_mesh_single_process_and_shape_check():
    from nbdistributed_amd.parallel import ParallelMesh

    m = ParallelMesh(dp=1, tp=1)
    assert m.coord("dp") == 0 and m.size("tp") == 1 and m.members("tp") == [0]
    with pytest.raises(ValueError):
        ParallelMesh(dp=3)
    with pytest.raises(ValueError):
        ParallelMesh()


def test_four_ranks_tp_generation():
    # one GPT-2 head per rank: the per-rank caches hold a single head each
    _spawn(_tp_generate_case, 4)
