"""KV-cache generation (nbdistributed_amd/generation.py) on CPU: the decode path must reproduce
the full (cache-free) forward pass token for token, for both model families, ragged prompts."""
import pytest
import torch

from nbdistributed_amd import ops
from nbdistributed_amd.generation import KVCache, generate, sample
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.models.llama import LlamaConfig, LlamaForCausalLM


def _models():
    torch.manual_seed(0)
    return [GPT2(GPT2Config.tiny()).eval(), LlamaForCausalLM(LlamaConfig.tiny()).eval()]


def _logits(m, x):
    return m(x)[0] if isinstance(m, GPT2) else m(x)[1]


def _greedy_recompute(m, prompt, n):
    seq = list(prompt)
    with torch.no_grad():
        for _ in range(n):
            seq.append(int(_logits(m, torch.tensor([seq]))[0, -1].argmax()))
    return seq


@pytest.mark.parametrize("which", [0, 1], ids=["gpt2", "llama"])
def test_greedy_generate_matches_full_forward(which):
    m = _models()[which]
    ids = torch.randint(1, 512, (3, 10), generator=torch.Generator().manual_seed(1))
    lens = torch.tensor([10, 7, 4])
    out = m.generate(ids, 6, lengths=lens)
    assert out.shape == (3, 16)
    for b in range(3):
        L = int(lens[b])
        assert out[b, :L + 6].tolist() == _greedy_recompute(m, ids[b, :L].tolist(), 6)
        assert (out[b, L + 6:] == 0).all()  # pad after the new tokens


@pytest.mark.parametrize("which", [0, 1], ids=["gpt2", "llama"])
def test_decode_step_logits_match_full_forward(which):
    m = _models()[which]
    ids = torch.randint(1, 512, (2, 9), generator=torch.Generator().manual_seed(2))
    cache = KVCache.for_model(m, 2, 16)
    lens = torch.tensor([5, 5])
    m.prefill(ids[:, :5], cache, lens)
    for t in range(5, 9):
        lg = m.decode_step(ids[:, t], torch.full((2,), t), cache)
        ref = _logits(m, ids[:, :t + 1])[:, -1]
        torch.testing.assert_close(lg, ref, rtol=1e-4, atol=1e-4)


def test_decode_attention_reference_matches_masked_attention():
    torch.manual_seed(3)
    B, H, Hkv, D, Tmax = 2, 4, 2, 64, 12
    k = torch.randn(B, Hkv, Tmax, D)
    v = torch.randn(B, Hkv, Tmax, D)
    qkv = torch.randn(B, (H + 2 * Hkv) * D)
    pos = torch.tensor([3, 8])
    kc, vc = k.clone(), v.clone()
    o = ops.decode_attention(qkv, kc, vc, pos, H)
    for b in range(B):
        p = int(pos[b])
        kk, vv = k[b, :, :p + 1].clone(), v[b, :, :p + 1].clone()
        kk[:, p] = qkv[b, H * D:(H + Hkv) * D].view(Hkv, D)
        vv[:, p] = qkv[b, (H + Hkv) * D:].view(Hkv, D)
        q = qkv[b, :H * D].view(H, 1, D)
        ref = torch.nn.functional.scaled_dot_product_attention(q, kk.repeat_interleave(H // Hkv, 0),
                                                               vv.repeat_interleave(H // Hkv, 0))
        torch.testing.assert_close(o[b].view(H, D), ref.view(H, D), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(kc[b, :, p], kk[:, p])  # the new row was appended


def test_sampling_controls():
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(4, 50, generator=g)
    assert torch.equal(sample(logits), logits.argmax(-1))
    assert torch.equal(sample(logits, temperature=1.0, top_k=1, generator=g), logits.argmax(-1))
    assert torch.equal(sample(logits, temperature=1.0, top_p=1e-6, generator=g), logits.argmax(-1))
    s = torch.stack([sample(logits, temperature=1.0, top_k=5, generator=g) for _ in range(200)])
    top5 = logits.topk(5, -1).indices
    assert all(bool((top5[b] == s[:, b, None]).any(-1).all()) for b in range(4))
    a = sample(logits, temperature=0.7, generator=torch.Generator().manual_seed(5))
    b = sample(logits, temperature=0.7, generator=torch.Generator().manual_seed(5))
    assert torch.equal(a, b)


def test_eos_stops_and_pads_with_eos():
    m = _models()[0]
    ids = torch.randint(1, 512, (2, 6), generator=torch.Generator().manual_seed(4))
    free = m.generate(ids, 8)
    eos = int(free[0, 7])  # the second new token of row 0
    out = m.generate(ids, 8, eos_token_id=eos, sync_every=1)
    row = out[0, 6:].tolist()
    i = row.index(eos)
    assert all(t == eos for t in row[i:i + 1]) and row[:i + 1] == free[0, 6:6 + i + 1].tolist()


def test_generate_rejects_too_long():
    m = _models()[0]  # tiny GPT-2: 128 positions
    with pytest.raises(ValueError):
        m.generate(torch.ones(1, 100, dtype=torch.long), 40)


def test_sampled_generation_reproducible_with_generator():
    m = _models()[1]
    ids = torch.randint(1, 512, (2, 5), generator=torch.Generator().manual_seed(6))
    a = m.generate(ids, 7, temperature=0.9, top_k=40, generator=torch.Generator().manual_seed(7))
    b = m.generate(ids, 7, temperature=0.9, top_k=40, generator=torch.Generator().manual_seed(7))
    assert torch.equal(a, b) and torch.equal(a[:, :5], ids)


def test_generate_refuses_past_the_sliding_window():
    torch.manual_seed(0)
    m = LlamaForCausalLM(LlamaConfig.tiny(sliding_window=16)).eval()
    ids = torch.randint(1, 512, (1, 10))
    m.generate(ids, 6)  # 16 positions: inside the window
    with pytest.raises(NotImplementedError):
        m.generate(ids, 7)


def test_returned_cache_has_no_stale_key_bound():
    m = _models()[0]
    ids = torch.randint(1, 512, (2, 6), generator=torch.Generator().manual_seed(8))
    out, cache = m.generate(ids, 4, graph=False, return_cache=True)
    assert cache.kv_len_max is None
