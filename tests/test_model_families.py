"""HF interop beyond the notebook's SmolLM2: GPT-2 (``GPT2.from_hf``), Qwen2 (biased q/k/v),
Mistral (explicit head_dim) and Llama 3.x rope scaling — logits and loss equal to transformers'
on the same random weights (CPU, fp32), and cached generation equal to HF greedy generate."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from nbdistributed_amd.models import GPT2  # noqa: E402
from nbdistributed_amd.models.llama import from_hf  # noqa: E402

SMALL = dict(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=2, num_attention_heads=4,
             num_key_value_heads=2, max_position_embeddings=256)


def _eager(cfg):
    cfg._attn_implementation = "eager"
    return cfg


def _check_lm(hf, ours, V):
    ids = torch.randint(1, V, (2, 20), generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        out = hf(input_ids=ids, labels=ids)
        res = ours(ids, labels=ids) if not isinstance(ours, GPT2) else None
    if res is None:
        with torch.no_grad():
            logits, _ = ours(ids)
        loss = torch.nn.functional.cross_entropy(logits[:, :-1].reshape(-1, V), ids[:, 1:].reshape(-1))
    else:
        loss, logits = res
    torch.testing.assert_close(logits, out.logits, atol=5e-5, rtol=1e-4)
    assert abs(float(loss) - float(out.loss)) < 1e-5
    return ids


def _check_generate(hf, ours, ids):
    with torch.no_grad():
        ref = hf.generate(ids[:, :8], attention_mask=torch.ones_like(ids[:, :8]), max_new_tokens=6,
                          do_sample=False, pad_token_id=0)
    got = ours.generate(ids[:, :8], 6)
    assert torch.equal(got, ref)


def test_gpt2_from_hf():
    torch.manual_seed(0)
    hc = transformers.GPT2Config(vocab_size=256, n_positions=128, n_embd=128, n_layer=2, n_head=4)
    hf = transformers.GPT2LMHeadModel(_eager(hc)).eval()
    ours = GPT2.from_hf(hf).eval()
    ids = _check_lm(hf, ours, 256)
    _check_generate(hf, ours, ids)


def test_qwen2_from_hf_biased_qkv():
    torch.manual_seed(1)
    hf = transformers.Qwen2ForCausalLM(_eager(transformers.Qwen2Config(**SMALL))).eval()
    with torch.no_grad():  # HF initialises biases to zero: make them matter
        for layer in hf.model.layers:
            for proj in (layer.self_attn.q_proj, layer.self_attn.k_proj, layer.self_attn.v_proj):
                proj.bias.normal_(0, 0.5)
    ours = from_hf(hf).eval()
    assert ours.config.qkv_bias and not ours.config.o_bias
    ids = _check_lm(hf, ours, 256)
    _check_generate(hf, ours, ids)


def test_mistral_from_hf_explicit_head_dim():
    torch.manual_seed(2)
    hf = transformers.MistralForCausalLM(_eager(transformers.MistralConfig(head_dim=48, **SMALL))).eval()
    ours = from_hf(hf).eval()
    assert ours.config.head_dim == 48
    ids = _check_lm(hf, ours, 256)
    _check_generate(hf, ours, ids)


def test_llama3_rope_scaling_from_hf():
    torch.manual_seed(3)
    rp = {"rope_type": "llama3", "rope_theta": 500000.0, "factor": 8.0, "low_freq_factor": 1.0,
          "high_freq_factor": 4.0, "original_max_position_embeddings": 16}
    hf = transformers.LlamaForCausalLM(_eager(transformers.LlamaConfig(rope_parameters=rp, attention_bias=True,
                                                                       **SMALL))).eval()
    with torch.no_grad():
        for layer in hf.model.layers:
            layer.self_attn.o_proj.bias.normal_(0, 0.5)
    ours = from_hf(hf).eval()
    assert ours.config.rope_scaling is not None and ours.config.o_bias
    ids = _check_lm(hf, ours, 256)
    _check_generate(hf, ours, ids)


def test_unsupported_variants_raise():
    from nbdistributed_amd.models.llama import LlamaConfig

    with pytest.raises(NotImplementedError):
        LlamaConfig.from_hf(transformers.LlamaConfig(rope_parameters={"rope_type": "yarn", "factor": 2.0,
                                                                      "rope_theta": 1e4}, **SMALL))
    with pytest.raises(NotImplementedError):
        LlamaConfig.from_hf(transformers.LlamaConfig(mlp_bias=True, **SMALL))
