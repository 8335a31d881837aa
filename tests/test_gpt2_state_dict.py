"""GPT-2's token table is stored padded (``GPT2Config.vocab_pad``: 512 with the hand-written LM
head, 128 with the library head, set from the environment): a state_dict saved under one padding
loads under the other, and an unpadded (HF-layout) table loads too."""
import pytest
import torch

from nbdistributed_amd.models import GPT2, GPT2Config


def _m(pad, V=50257):
    torch.manual_seed(0)
    return GPT2(GPT2Config(vocab_size=V, n_positions=32, n_embd=32, n_layer=1, n_head=1, vocab_pad=pad))


@pytest.mark.parametrize("src,dst", [(128, 512), (512, 128), (1, 512), (512, 1)])
def test_state_dict_loads_across_vocab_padding(src, dst):
    a, b = _m(src), _m(dst)
    assert a.wte.weight.shape[0] != b.wte.weight.shape[0]
    b.load_state_dict(a.state_dict())
    assert torch.equal(b.wte.weight[:50257], a.wte.weight[:50257])
    assert b.wte.weight.shape[0] == b.config.padded_vocab and not b.wte.weight[50257:].any()
    assert b.lm_head.weight is b.wte.weight  # still tied


def test_nonzero_pad_rows_are_refused():
    a, b = _m(512), _m(128)
    with torch.no_grad():
        a.wte.weight[50600] = 1.0  # a pad row that is not zero cannot be dropped silently
    with pytest.raises(RuntimeError, match="past the vocabulary"):
        b.load_state_dict(a.state_dict())
