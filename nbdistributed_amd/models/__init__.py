"""Model families used by the reference's workloads and the BASELINE configs.

* ``GPT2`` (``gpt2.py``) — GPT-2 small, 124,439,808 parameters (config 5).
* ``linear_4096`` — ``nn.Linear(4096, 4096)`` (configs 3 and 4).
* ``smollm2_135m_classifier`` — the reference notebook's model (SmolLM2-135M with a 2-way
  sequence-classification head, 134,516,160 parameters; ``00_accelerate.ipynb`` exec 22),
  random-init from its architecture config (no checkpoint download: no network).
* ``synthetic_mrpc`` — token/label batches shaped like the notebook's tokenized GLUE/MRPC
  (3,668 train samples, max_length 128).
"""
from __future__ import annotations

from typing import Optional

from .gpt2 import GPT2, GPT2Config

SMOLLM2_135M = dict(vocab_size=49152, hidden_size=576, intermediate_size=1536, num_hidden_layers=30,
                    num_attention_heads=9, num_key_value_heads=3, max_position_embeddings=8192,
                    rms_norm_eps=1e-5, rope_theta=100000.0, tie_word_embeddings=True, hidden_act="silu")


def linear_4096(bias: bool = True):
    import torch

    return torch.nn.Linear(4096, 4096, bias=bias)


def smollm2_135m_classifier(num_labels: int = 2, **overrides):
    """LlamaForSequenceClassification with SmolLM2-135M's architecture (random init)."""
    from transformers import LlamaConfig, LlamaForSequenceClassification

    cfg = dict(SMOLLM2_135M)
    cfg.update(overrides)
    conf = LlamaConfig(num_labels=num_labels, pad_token_id=0, **cfg)
    return LlamaForSequenceClassification(conf)


def synthetic_mrpc(n: int = 3668, seq_len: int = 128, vocab: int = 49152, seed: int = 0, device: Optional[str] = None):
    """(input_ids, attention_mask, labels) with MRPC's train-split shape; ~68% positive labels
    like MRPC.  Synthetic: the environment has no network for the real dataset."""
    import torch

    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1, vocab, (n, seq_len), generator=g)
    lengths = torch.randint(seq_len // 3, seq_len + 1, (n,), generator=g)
    mask = (torch.arange(seq_len)[None, :] < lengths[:, None]).long()
    ids = ids * mask
    labels = (torch.rand(n, generator=g) < 0.68).long()
    if device is not None:
        ids, mask, labels = ids.to(device), mask.to(device), labels.to(device)
    return ids, mask, labels


def native(hf_model, compute_dtype=None, **kw):
    """Swap an HF Llama-family model for the framework's native one (``llama.native``): same
    call signature and ``.loss`` / ``.logits`` outputs, fp32 master parameters, bf16 compute on
    the fused HIP path.  ``model = nbd.models.native(model)`` before creating the optimizer.
    Keywords (``fused_optimizer``, ``block_graphs``) go to ``llama.native``."""
    import torch

    from .llama import native as _native

    return _native(hf_model, compute_dtype=compute_dtype or torch.bfloat16, **kw)


__all__ = ["GPT2", "GPT2Config", "linear_4096", "smollm2_135m_classifier", "synthetic_mrpc", "SMOLLM2_135M", "native"]
