"""Native Llama family vs HF transformers (same random weights), CPU fp32 math path:
sequence classification (the reference notebook's model type) and causal LM — logits, loss
and gradients mapped back onto HF's separate q/k/v and gate/up projections."""
import pytest
import torch

from nbdistributed_amd.models.llama import LlamaConfig, from_hf

transformers = pytest.importorskip("transformers")


def _hf_config(c: LlamaConfig, **kw):
    hc = transformers.LlamaConfig(vocab_size=c.vocab_size, hidden_size=c.hidden_size,
                                  intermediate_size=c.intermediate_size, num_hidden_layers=c.num_hidden_layers,
                                  num_attention_heads=c.num_attention_heads,
                                  num_key_value_heads=c.num_key_value_heads,
                                  max_position_embeddings=c.max_position_embeddings, rms_norm_eps=c.rms_norm_eps,
                                  rope_theta=c.rope_theta, tie_word_embeddings=True, pad_token_id=0, **kw)
    hc._attn_implementation = "eager"
    return hc


def _batch(B=3, T=24, V=512, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1, V, (B, T), generator=g)
    lens = torch.tensor([T, T - 5, T // 2])[:B]
    mask = (torch.arange(T)[None] < lens[:, None]).long()
    return ids * mask, mask


def test_sequence_classification_matches_hf():
    torch.manual_seed(0)
    c = LlamaConfig.tiny(rope_theta=100000.0)
    hf = transformers.LlamaForSequenceClassification(_hf_config(c, num_labels=2)).eval()
    ours = from_hf(hf).eval()
    ids, mask = _batch()
    labels = torch.tensor([0, 1, 1])
    out = hf(input_ids=ids, attention_mask=mask, labels=labels)
    loss, logits = ours(ids, mask, labels)
    assert torch.allclose(logits, out.logits, atol=2e-5, rtol=1e-4), (logits, out.logits)
    assert abs(float(loss) - float(out.loss)) < 1e-5
    out.loss.backward()
    loss.backward()
    H, Hkv, D = c.num_attention_heads, c.num_key_value_heads, c.head_dim
    l0h, l0o = hf.model.layers[0], ours.model.layers[0]
    gq = l0o.self_attn.qkv_proj.weight.grad
    pairs = [(gq[: H * D], l0h.self_attn.q_proj.weight.grad),
             (gq[H * D:(H + Hkv) * D], l0h.self_attn.k_proj.weight.grad),
             (gq[(H + Hkv) * D:], l0h.self_attn.v_proj.weight.grad),
             (l0o.mlp.gate_up_proj.weight.grad[: c.intermediate_size], l0h.mlp.gate_proj.weight.grad),
             (ours.model.embed_tokens.weight.grad, hf.model.embed_tokens.weight.grad),
             (ours.model.norm.weight.grad, hf.model.norm.weight.grad),
             (ours.score.weight.grad, hf.score.weight.grad)]
    for a, b in pairs:
        assert torch.allclose(a, b, atol=1e-5, rtol=1e-3), float((a - b).abs().max())


def test_causal_lm_matches_hf():
    torch.manual_seed(1)
    c = LlamaConfig.tiny(num_key_value_heads=4)
    hf = transformers.LlamaForCausalLM(_hf_config(c)).eval()
    ours = from_hf(hf).eval()
    ids = torch.randint(1, 512, (2, 16))
    out = hf(input_ids=ids, labels=ids)
    loss, logits = ours(ids, labels=ids)
    assert torch.allclose(logits, out.logits, atol=5e-5, rtol=1e-4)
    assert abs(float(loss) - float(out.loss)) < 1e-5


def test_tied_lm_head_and_param_count():
    from nbdistributed_amd.models.llama import LlamaForCausalLM

    m = LlamaForCausalLM(LlamaConfig.smollm2_135m())
    assert m.lm_head.weight is m.model.embed_tokens.weight
    assert sum(p.numel() for p in m.parameters()) == 134_515_008  # SmolLM2-135M


def test_native_swap_has_hf_outputs_and_signature():
    """``nbd.models.native(hf)``: same keyword call, ``out.loss`` / ``out.logits``, fp32 master
    parameters kept (CPU: the plain-math path)."""
    import nbdistributed_amd as nbd

    torch.manual_seed(0)
    c = LlamaConfig.tiny(rope_theta=100000.0)
    hf = transformers.LlamaForSequenceClassification(_hf_config(c, num_labels=2)).eval()
    ours = nbd.models.native(hf).eval()
    assert all(p.dtype == torch.float32 for p in ours.parameters())
    ids, mask = _batch()
    labels = torch.tensor([0, 1, 1])
    ref = hf(input_ids=ids, attention_mask=mask, labels=labels)
    out = ours(input_ids=ids, attention_mask=mask, labels=labels, return_dict=True)
    assert torch.allclose(out.logits, ref.logits, atol=2e-5, rtol=1e-4)
    assert abs(float(out.loss) - float(ref.loss)) < 1e-5
    loss, logits = out  # still a (loss, logits) tuple
    assert loss is out.loss and logits is out.logits
    assert ours(input_ids=ids, attention_mask=mask).loss is None
    with pytest.raises(TypeError):
        ours(input_ids=ids, output_attentions=True)


def _left_pad(ids, mask):
    """The same rows left-padded (pad id 0)."""
    B, T = ids.shape
    out_ids, out_mask = torch.zeros_like(ids), torch.zeros_like(mask)
    for b in range(B):
        n = int(mask[b].sum())
        out_ids[b, T - n:] = ids[b, :n]
        out_mask[b, T - n:] = 1
    return out_ids, out_mask


def test_left_padded_batch_matches_hf():
    """HF masks padded keys; the fused path rotates left-padded rows into right-padded ones
    (RoPE scores depend on position differences only) and re-indexes the pooled token."""
    torch.manual_seed(0)
    c = LlamaConfig.tiny(rope_theta=100000.0)
    hf = transformers.LlamaForSequenceClassification(_hf_config(c, num_labels=2)).eval()
    ours = from_hf(hf).eval()
    ids, mask = _left_pad(*_batch())
    labels = torch.tensor([0, 1, 1])
    out = hf(input_ids=ids, attention_mask=mask, labels=labels)
    loss, logits = ours(input_ids=ids, attention_mask=mask, labels=labels)
    assert torch.allclose(logits, out.logits, atol=2e-5, rtol=1e-4), (logits, out.logits)
    assert abs(float(loss) - float(out.loss)) < 1e-5
    out.loss.backward()
    loss.backward()
    assert torch.allclose(ours.score.weight.grad, hf.score.weight.grad, atol=1e-5, rtol=1e-3)
    # the same batch through the module path (a hook registered): exact masking, same answer
    h = ours.model.layers[0].register_forward_hook(lambda m, a, o: None)
    try:
        loss2, logits2 = ours(input_ids=ids, attention_mask=mask, labels=labels)
    finally:
        h.remove()
    assert torch.allclose(logits2, out.logits, atol=2e-5, rtol=1e-4)


def test_prep_rotation_reference():
    from nbdistributed_amd.ops.mask import _ref_seqcls_prep

    ids = torch.tensor([[0, 0, 5, 6, 7], [3, 4, 0, 0, 0], [1, 2, 3, 4, 5]])
    mask = (ids != 0).long()
    bad = torch.zeros(1, dtype=torch.int32)
    r, pool = _ref_seqcls_prep(ids, mask, 0, bad)
    assert r.tolist() == [[5, 6, 7, 0, 0], [3, 4, 0, 0, 0], [1, 2, 3, 4, 5]] and pool.tolist() == [2, 1, 4]
    assert int(bad) == 2  # left padding: the causal LM's failing bit, not the classifier's
    bad.zero_()
    _ref_seqcls_prep(torch.tensor([[1, 0, 2]]), torch.tensor([[1, 0, 1]]), 0, bad)
    assert int(bad) & 1


def test_mask_with_holes_is_reported():
    torch.manual_seed(0)
    c = LlamaConfig.tiny()
    hf = transformers.LlamaForSequenceClassification(_hf_config(c, num_labels=2)).eval()
    ours = from_hf(hf).eval()
    ids, mask = _batch()
    mask[0, 3] = 0
    with pytest.raises(ValueError, match="holes"):
        ours(input_ids=ids, attention_mask=mask)


def test_decoder_layer_hook_fires_with_hf_activations():
    """A hook on ``layers[3]`` (and on its MLP) fires and sees HF's hidden states: the model runs
    module by module while any hook is registered."""
    torch.manual_seed(0)
    c = LlamaConfig.tiny(num_hidden_layers=4)
    hf = transformers.LlamaForSequenceClassification(_hf_config(c, num_labels=2)).eval()
    ours = from_hf(hf).eval()
    ids, mask = _batch()
    seen = {}

    def grab(tag):
        def hook(m, args, out):
            seen[tag] = (args[0].detach().clone(), (out[0] if isinstance(out, tuple) else out).detach().clone())
        return hook

    hs = [hf.model.layers[3].register_forward_hook(grab("hf")), hf.model.layers[3].mlp.register_forward_hook(grab("hf_mlp")),
          ours.model.layers[3].register_forward_hook(grab("ours")),
          ours.model.layers[3].mlp.register_forward_hook(grab("ours_mlp"))]
    try:
        out = hf(input_ids=ids, attention_mask=mask)
        res = ours(input_ids=ids, attention_mask=mask)
    finally:
        for h in hs:
            h.remove()
    valid = mask.bool()
    for a, b in (("hf", "ours"), ("hf_mlp", "ours_mlp")):
        for i in (0, 1):
            x, y = seen[a][i][valid], seen[b][i][valid]
            assert torch.allclose(x, y, atol=5e-5, rtol=1e-4), (a, i, float((x - y).abs().max()))
    assert torch.allclose(res.logits, out.logits, atol=2e-5, rtol=1e-4)
    assert not ours.model.hooked()  # removed: the fused path again


def test_native_fused_optimizer_default_is_reversible():
    """``native()`` wraps AdamW/Adam.__init__ while a native model lives (fused=True default) and
    restores the originals when the last one is collected."""
    import gc

    from nbdistributed_amd.models import llama as L

    orig_adamw, orig_adam = torch.optim.AdamW.__init__, torch.optim.Adam.__init__
    c = LlamaConfig.tiny()
    hf = transformers.LlamaForSequenceClassification(_hf_config(c, num_labels=2))
    m1 = L.native(hf, compute_dtype=None)
    m2 = L.native(hf, compute_dtype=None)
    assert torch.optim.AdamW.__init__ is not orig_adamw and torch.optim.Adam.__init__ is not orig_adam
    opt = torch.optim.AdamW(m1.parameters(), lr=1e-3)  # CPU parameters: torch's default, not fused
    assert not opt.defaults.get("fused")
    del m1, opt
    gc.collect()
    assert torch.optim.AdamW.__init__ is not orig_adamw  # m2 still alive
    del m2
    gc.collect()
    assert torch.optim.AdamW.__init__ is orig_adamw and torch.optim.Adam.__init__ is orig_adam
