"""GPU: Llama-family kernels (RMSNorm, RoPE, SwiGLU, GQA flash attention) against fp32
PyTorch references, the bf16 HIP model path against the fp32 math path, and a HIP-graph
captured training step against eager."""
import pytest
import torch
import torch.nn.functional as F

from nbdistributed_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(require_gpu):
    assert ops.native_available(), ops._load_error
    return torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("res", [False, True])
@pytest.mark.parametrize("C", [576, 64, 2048])
def test_rms_norm(dev, res, C):
    x = torch.randn(257, C, device=dev, dtype=torch.bfloat16)
    d = torch.randn(257, C, device=dev, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(C, device=dev)).to(torch.bfloat16)
    dy = torch.randn(257, C, device=dev, dtype=torch.bfloat16)
    xs, ds, ws = (t.clone().requires_grad_(True) for t in (x, d, w))
    xr, dr, wr = (t.float().cpu().requires_grad_(True) for t in (x, d, w))
    if res:
        s, y = ops.add_rms_norm(xs, ds, ws, 1e-5)
        sr = xr + dr
    else:
        y = ops.rms_norm(xs, ws, 1e-5)
        sr = xr
    yr = sr * torch.rsqrt(sr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    y.backward(dy)
    yr.backward(dy.float().cpu())
    assert _rel(y, yr) < 2e-2
    assert _rel(xs.grad, xr.grad) < 3e-2 and _rel(ws.grad, wr.grad) < 3e-2
    if res:
        assert _rel(ds.grad, dr.grad) < 3e-2


@pytest.mark.parametrize("C", [576, 64])
def test_embed_rms_norm_matches_separate_ops(dev, C):
    """ops.embed_rms_norm (one forward launch; in backward the residual stream's gradient added in
    the norm's pass) against F.embedding + ops.rms_norm: x0 and h bit-identical, the table and
    weight gradients equal to the two-op path's, both gradients arriving (ds from the residual
    stream, dh from the norm's output), a repeated id included."""
    g = torch.Generator(device="cpu").manual_seed(C)
    V = 300
    table = torch.randn(V, C, generator=g).to(dev, torch.bfloat16)
    w = (1 + 0.1 * torch.randn(C, generator=g)).to(dev, torch.bfloat16)
    ids = torch.randint(0, V, (3, 128), generator=g).to(dev)
    ids[0, 5] = ids[1, 7]
    ds = torch.randn(3, 128, C, generator=g).to(dev, torch.bfloat16)
    dh = torch.randn(3, 128, C, generator=g).to(dev, torch.bfloat16)
    t1, w1 = table.clone().requires_grad_(True), w.clone().requires_grad_(True)
    x1, h1 = ops.embed_rms_norm(ids, t1, w1, 1e-5)
    torch.autograd.backward([x1, h1], [ds, dh])
    t2, w2 = table.clone().requires_grad_(True), w.clone().requires_grad_(True)
    x2 = F.embedding(ids, t2)
    h2 = ops.rms_norm(x2, w2, 1e-5)
    torch.autograd.backward([x2, h2], [ds, dh])
    torch.cuda.synchronize()
    assert torch.equal(x1, x2) and torch.equal(h1, h2)
    assert _rel(t1.grad, t2.grad) < 1e-2 and _rel(w1.grad, w2.grad) < 1e-2
    # only the norm's output used: the residual-gradient path absent
    t3 = table.clone().requires_grad_(True)
    ops.embed_rms_norm(ids, t3, w, 1e-5)[1].backward(dh)
    t4 = table.clone().requires_grad_(True)
    ops.rms_norm(F.embedding(ids, t4), w, 1e-5).backward(dh)
    assert _rel(t3.grad, t4.grad) < 1e-2


def test_tokpos_layer_norm_matches_separate_ops(dev):
    """ops.tokpos_layer_norm (GPT-2's input + first LayerNorm as one node) against
    embedding_tok_pos + layer_norm: x0 bit-identical, h equal to rounding; token table (padded past the
    vocabulary: zero gradient there), position table, weight and bias gradients equal to the
    two-op path's with both the residual and the norm gradient arriving."""
    g = torch.Generator(device="cpu").manual_seed(3)
    V, Vp, P, C, T = 500, 512, 256, 256, 128
    wte = torch.randn(Vp, C, generator=g).to(dev, torch.bfloat16)
    wte[V:] = 0
    wpe = torch.randn(P, C, generator=g).to(dev, torch.bfloat16)
    w = (1 + 0.1 * torch.randn(C, generator=g)).to(dev, torch.bfloat16)
    b = (0.1 * torch.randn(C, generator=g)).to(dev, torch.bfloat16)
    idx = torch.randint(0, V, (2, T), generator=g).to(dev)
    pos = torch.arange(T, device=dev)
    ds = torch.randn(2, T, C, generator=g).to(dev, torch.bfloat16)
    dh = torch.randn(2, T, C, generator=g).to(dev, torch.bfloat16)
    outs = []
    for fused in (True, False):
        ps = [t.clone().requires_grad_(True) for t in (wte, wpe, w, b)]
        if fused:
            x, h = ops.tokpos_layer_norm(idx, ps[0], pos, ps[1], V, ps[2], ps[3], 1e-5)
        else:
            x = ops.embedding_tok_pos(idx, ps[0], pos, ps[1], V)
            h = ops.layer_norm(x, ps[2], ps[3], 1e-5)
        torch.autograd.backward([x, h], [ds, dh])
        torch.cuda.synchronize()
        outs.append((x, h, [p.grad for p in ps]))
    (x1, h1, g1), (x2, h2, g2) = outs
    # (h: the separate LayerNorm may take the 16-B kernel, whose partial sums group differently)
    assert torch.equal(x1, x2) and _rel(h1, h2) < 1e-2
    for a, r in zip(g1, g2):
        assert _rel(a, r) < 1e-2
    assert (g1[0][V:] == 0).all()


def test_rope_forward_backward(dev):
    B, T, H, Hkv, D = 2, 128, 9, 3, 64
    x = torch.randn(B, T, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    cos, sin = ops.rope_tables(T, D, 100000.0, dev)
    xr = x.float().cpu().requires_grad_(True)
    ref = ops.rope_(xr, cos.cpu(), sin.cpu(), H + Hkv, D)  # CPU math path
    xs = x.clone().requires_grad_(True)
    y = ops.rope_(xs * 1, cos, sin, H + Hkv, D)
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g.float().cpu())
    assert _rel(y, ref) < 1e-2
    assert _rel(xs.grad, xr.grad) < 1e-2


def test_swiglu(dev):
    gu = torch.randn(300, 2 * 1536, device=dev, dtype=torch.bfloat16)
    d = torch.randn(300, 1536, device=dev, dtype=torch.bfloat16)
    a = gu.clone().requires_grad_(True)
    r = gu.float().cpu().requires_grad_(True)
    y = ops.swiglu(a)
    yr = F.silu(r[:, :1536]) * r[:, 1536:]
    y.backward(d)
    yr.backward(d.float().cpu())
    assert _rel(y, yr) < 1e-2 and _rel(a.grad, r.grad) < 2e-2


@pytest.mark.parametrize("causal", [True, False])
def test_gqa_flash_attention(dev, causal):
    B, H, Hkv, T = 2, 9, 3, 256
    q = torch.randn(B, H, T, 64, device=dev, dtype=torch.bfloat16)
    k, v = (torch.randn(B, Hkv, T, 64, device=dev, dtype=torch.bfloat16) for _ in range(2))
    do = torch.randn_like(q)
    qs, ks, vs = (t.clone().requires_grad_(True) for t in (q, k, v))
    out = ops.flash_attention(qs, ks, vs, causal=causal)
    out.backward(do)
    qr, kr, vr = (t.float().requires_grad_(True) for t in (q, k, v))
    s = qr @ kr.repeat_interleave(H // Hkv, 1).transpose(-1, -2) * 0.125
    if causal:
        s = s.masked_fill(torch.ones(T, T, dtype=torch.bool, device=dev).triu(1), float("-inf"))
    ref = torch.softmax(s, -1) @ vr.repeat_interleave(H // Hkv, 1)
    ref.backward(do.float())
    assert _rel(out, ref) < 2e-2
    for a, b in ((qs.grad, qr.grad), (ks.grad, kr.grad), (vs.grad, vr.grad)):
        assert _rel(a, b) < 3e-2


def _smol_tiny():
    from nbdistributed_amd.models.llama import LlamaConfig

    # SmolLM2's head geometry (9 query heads, 3 kv heads, head_dim 64) with fewer layers
    return LlamaConfig(vocab_size=4096, hidden_size=576, intermediate_size=1536, num_hidden_layers=3)


def _batch(dev, B=4, T=128, V=4096):
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(1, V, (B, T), generator=g)
    lens = torch.randint(T // 3, T + 1, (B,), generator=g)
    mask = (torch.arange(T)[None] < lens[:, None]).long()
    return (ids * mask).to(dev), mask.to(dev), torch.randint(0, 2, (B,), generator=g).to(dev)


def test_llama_bf16_hip_path_matches_fp32_math(dev):
    from nbdistributed_amd.models.llama import LlamaForSequenceClassification

    torch.manual_seed(0)
    ref = LlamaForSequenceClassification(_smol_tiny())
    m = LlamaForSequenceClassification(_smol_tiny())
    m.load_state_dict(ref.state_dict())
    m = m.to(dev, torch.bfloat16)
    ids, mask, labels = _batch(dev)
    loss, logits = m(ids, mask, labels)
    loss.backward()
    lr_, logr = ref(ids.cpu(), mask.cpu(), labels.cpu())
    lr_.backward()
    assert _rel(logits, logr) < 5e-2, (logits, logr)
    assert abs(float(loss.detach()) - float(lr_.detach())) < 3e-2
    for name in ("model.layers.0.self_attn.qkv_proj.weight", "model.layers.2.mlp.gate_up_proj.weight",
                 "model.embed_tokens.weight", "score.weight"):
        a = dict(m.named_parameters())[name].grad
        b = dict(ref.named_parameters())[name].grad
        assert _rel(a, b) < 0.1, (name, _rel(a, b))


def test_llama_training_step_graph_capture(dev):
    from nbdistributed_amd.graphs import GraphedStep
    from nbdistributed_amd.models.llama import LlamaForSequenceClassification

    def build():
        torch.manual_seed(3)
        m = LlamaForSequenceClassification(_smol_tiny()).to(dev, torch.bfloat16)
        return m, torch.optim.AdamW(m.parameters(), lr=1e-3, capturable=True)

    batches = [_batch(dev, seed) if False else _batch(dev) for seed in range(1)]
    ids, mask, labels = batches[0]

    def make(m, o):
        def step(i, mk, y):
            loss, _ = m(i, mk, y)
            loss.backward()
            o.step()
            o.zero_grad(set_to_none=False)
            return loss.detach()
        return step

    m1, o1 = build()
    s1 = make(m1, o1)
    eager = [float(s1(ids, mask, labels)) for _ in range(6)]
    m2, o2 = build()
    gs = GraphedStep(make(m2, o2), (ids, mask, labels), warmup=3)
    graphed = [float(gs(ids, mask, labels)) for _ in range(3)]
    torch.cuda.synchronize()
    assert max(abs(a - b) for a, b in zip(eager[3:], graphed)) < 2e-2, (eager, graphed)


@pytest.mark.parametrize("Hkv", [3, 9])
def test_attention_with_fused_rope_matches_separate_rope(dev, Hkv):
    """RoPE inside the attention kernels == rope_ kernel + attention (fwd and packed dqkv)."""
    B, T, H, D = 2, 256, 9, 64
    qkv = torch.randn(B, T, (H + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(B, T, H * D, device=dev, dtype=torch.bfloat16)
    cos, sin = ops.rope_tables(T, D, 100000.0, dev)
    a = qkv.clone().requires_grad_(True)
    y1 = ops.attention_qkv(a, H, causal=True, n_kv_head=Hkv, rope=(cos, sin))
    y1.backward(dy)
    b = qkv.clone().requires_grad_(True)
    y2 = ops.attention_qkv(ops.rope_(b * 1, cos, sin, H + Hkv, D), H, causal=True, n_kv_head=Hkv)
    y2.backward(dy)
    torch.cuda.synchronize()
    assert _rel(y1, y2) < 1e-2, _rel(y1, y2)
    assert _rel(a.grad, b.grad) < 2e-2, _rel(a.grad, b.grad)


def test_native_swap_bf16_compute_fp32_master(dev):
    """``nbd.models.native(hf_fp32)`` on the GPU: fp32 parameters, bf16 fused compute (one cast
    per layer), loss/logits close to the fp32 HF model, fp32 gradients on every parameter,
    and one torch AdamW step moves the fp32 weights."""
    transformers = pytest.importorskip("transformers")
    import nbdistributed_amd as nbd
    from nbdistributed_amd.models import SMOLLM2_135M

    cfg = dict(SMOLLM2_135M)
    cfg.update(num_hidden_layers=2, vocab_size=4096)
    torch.manual_seed(0)
    hf = transformers.LlamaForSequenceClassification(
        transformers.LlamaConfig(num_labels=2, pad_token_id=0, **cfg)).to(dev)
    m = nbd.models.native(hf)
    assert m.model.compute_dtype == torch.bfloat16
    assert all(p.dtype == torch.float32 and p.is_cuda for p in m.parameters())
    ids, mask, labels = _batch(dev)
    assert m.model.cast_dtype(ids) == torch.bfloat16
    out = m(input_ids=ids, attention_mask=mask, labels=labels)
    ref = hf(input_ids=ids, attention_mask=mask, labels=labels)
    assert out.logits.dtype == torch.bfloat16
    assert _rel(out.logits.float(), ref.logits) < 5e-2, (out.logits, ref.logits)
    assert abs(float(out.loss) - float(ref.loss)) < 3e-2
    out.loss.backward()
    ref.loss.backward()
    grads = {n: p.grad for n, p in m.named_parameters()}
    assert all(g is not None and g.dtype == torch.float32 for g in grads.values()), \
        [n for n, g in grads.items() if g is None or g.dtype != torch.float32]
    hg = dict(hf.named_parameters())
    assert _rel(grads["model.norm.weight"], hg["model.norm.weight"].grad) < 0.1
    assert _rel(grads["model.embed_tokens.weight"], hg["model.embed_tokens.weight"].grad) < 0.1
    w0 = m.model.layers[0].mlp.down_proj.weight.detach().clone()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    opt.step()
    assert not torch.equal(w0, m.model.layers[0].mlp.down_proj.weight)
    # native(): torch AdamW on exactly these parameters defaults to the fused implementation, and
    # its update equals the multi-tensor one (same math; fp32)
    assert opt.defaults["fused"] is True
    state = {n: p.detach().clone() for n, p in m.named_parameters()}
    gr = {n: p.grad.clone() for n, p in m.named_parameters()}
    res = []
    for kw in ({}, {"foreach": True}):
        with torch.no_grad():
            for n, p in m.named_parameters():
                p.copy_(state[n])
                p.grad = gr[n].clone()
        o = torch.optim.AdamW(m.parameters(), lr=1e-3, **kw)
        assert o.defaults["fused"] is (True if not kw else None)
        o.step()
        res.append(torch.cat([p.detach().flatten() for p in m.parameters()]))
    assert _rel(res[0], res[1]) < 1e-5
    # other parameters keep torch's default
    assert torch.optim.AdamW([torch.nn.Parameter(torch.randn(4, device=dev))], lr=1e-3).defaults["fused"] is None


def test_cast_group_native_matches_python(dev):
    """The C++ cast node (models.native's per-layer bf16 casts) against the Python _CastGroup:
    identical values forward and identical fp32 gradients backward, odd sizes included."""
    from nbdistributed_amd.models.llama import _CastGroup, cast_group

    g = torch.Generator(device=dev).manual_seed(4)
    shapes = [(576, 960), (576,), (7, 13), (1,), (3, 5, 9)]
    ps = [torch.randn(s, device=dev, generator=g, requires_grad=True) for s in shapes]
    gs = [torch.randn(s, device=dev, generator=g).to(torch.bfloat16) for s in shapes]
    outs_c = cast_group(torch.bfloat16, ps)
    outs_p = _CastGroup.apply(torch.bfloat16, *ps)
    assert all(a.dtype == torch.bfloat16 and a.shape == b.shape and torch.equal(a, b) for a, b in zip(outs_c, outs_p))
    gc = torch.autograd.grad(outs_c, ps, gs)
    gp = torch.autograd.grad(outs_p, ps, gs)
    assert all(a.dtype == torch.float32 and torch.equal(a, b) for a, b in zip(gc, gp))
    # a gradient for only some outputs: the others get zeros (materialized, as the Python node)
    gc2 = torch.autograd.grad(outs_c[0].float().sum() + outs_c[3].float().sum(), ps)
    assert torch.equal(gc2[1], torch.zeros(576, device=dev)) and torch.equal(gc2[3], torch.ones(1, device=dev))
    with torch.inference_mode():
        inf = cast_group(torch.bfloat16, [p.detach() for p in ps])
    assert all(torch.equal(a, b) for a, b in zip(inf, outs_p))
