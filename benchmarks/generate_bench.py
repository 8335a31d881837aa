#!/usr/bin/env python3
"""Generation throughput: GPT-2 small (bf16, random init) decoding with the framework's KV cache
(graph-captured and eager) vs Hugging Face ``GPT2LMHeadModel.generate`` (its KV cache, eager) on
the same weights; plus the decode-attention kernel alone (achieved HBM bandwidth over the cache).

    python benchmarks/generate_bench.py [--batches 1,8,32] [--prompt 128] [--new 256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timed(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best


def kernel_bench(rows):
    from nbdistributed_amd import ops
    from nbdistributed_amd.ops.decode import partials_numel

    out = []
    for B, H, Hkv, T in rows:
        kc = torch.randn(B, Hkv, T, 64, device="cuda").to(torch.bfloat16)
        vc = torch.randn_like(kc)
        qkv = torch.randn(B, (H + 2 * Hkv) * 64, device="cuda").to(torch.bfloat16)
        pos = torch.full((B,), T - 1, device="cuda", dtype=torch.int64)
        ws = torch.empty(partials_numel(B, H, T), dtype=torch.float32, device="cuda")
        f = lambda: ops.decode_attention(qkv, kc, vc, pos, H, workspace=ws)  # noqa: E731
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        s.record()
        for _ in range(n):
            f()
        e.record()
        e.synchronize()
        us = s.elapsed_time(e) / n * 1e3
        gbs = 2 * kc.numel() * 2 / us / 1e3
        r = dict(B=B, H=H, Hkv=Hkv, T=T, us=round(us, 2), cache_GBps=round(gbs, 1))
        print(json.dumps(r), flush=True)
        out.append(r)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,8,32")
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--new", type=int, default=256)
    ap.add_argument("--no-hf", action="store_true")
    ap.add_argument("--model", default="gpt2", choices=["gpt2", "smollm2"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from nbdistributed_amd import ops
    from nbdistributed_amd.models import GPT2, GPT2Config

    ops.load_library()
    torch.manual_seed(0)
    hf = None
    if a.model == "smollm2":
        # SmolLM2-135M architecture (random init), built in HF and converted (models.llama.from_hf)
        from transformers import LlamaConfig as HLC, LlamaForCausalLM as HLM

        from nbdistributed_amd.models import SMOLLM2_135M
        from nbdistributed_amd.models.llama import from_hf

        cfg = dict(SMOLLM2_135M)
        cfg.pop("hidden_act", None)
        hf = HLM(HLC(**cfg)).to(torch.bfloat16)
        m = from_hf(hf).to("cuda").eval()
        hf = None if a.no_hf else hf.to("cuda").eval()
        vocab, name = cfg["vocab_size"], "SmolLM2-135M (random init)"
    else:
        m = GPT2(GPT2Config.small()).to("cuda", torch.bfloat16).eval()
        vocab, name = 50257, "gpt2-small (124M, random init)"
    if a.model == "gpt2" and not a.no_hf:
        try:
            from transformers import GPT2Config as HFC, GPT2LMHeadModel

            hf = GPT2LMHeadModel(HFC(n_embd=768, n_layer=12, n_head=12, n_positions=1024, vocab_size=50257))
            sd = {}
            for k, v in m.state_dict().items():  # nn.Linear [out, in] -> HF Conv1D [in, out]
                kk = "transformer." + k if not k.startswith("lm_head") else k
                if any(s in k for s in ("c_attn.weight", "c_proj.weight", "c_fc.weight")):
                    v = v.t()
                sd[kk] = v
            hf.load_state_dict(sd, strict=False)
            hf = hf.to("cuda", torch.bfloat16).eval()
        except Exception as e:  # pragma: no cover
            print("HF baseline unavailable:", e, flush=True)
    res = {"model": name, "dtype": "bf16", "prompt": a.prompt, "new_tokens": a.new, "runs": []}
    for B in [int(x) for x in a.batches.split(",")]:
        ids = torch.randint(1, vocab, (B, a.prompt), device="cuda")
        row = {"batch": B}
        g_out = None
        for name, kw in (("nbd_graph", dict(graph=True)), ("nbd_eager", dict(graph=False))):
            holder = {}
            t = timed(lambda: holder.__setitem__("o", m.generate(ids, a.new, **kw)))
            row[name + "_tok_per_s"] = round(B * a.new / t, 1)
            row[name + "_ms_per_token"] = round(t / a.new * 1e3, 3)
            if name == "nbd_graph":
                g_out = holder["o"]
        # steady-state decode cost: the marginal time per token between two lengths (prefill,
        # cache allocation and graph capture cancel out)
        t_short = timed(lambda: m.generate(ids, 32, graph=True))
        t_long = timed(lambda: m.generate(ids, 32 + a.new, graph=True))
        row["nbd_graph_marginal_ms_per_token"] = round((t_long - t_short) / a.new * 1e3, 3)
        row["nbd_graph_marginal_tok_per_s"] = round(B * a.new / (t_long - t_short), 1)
        if hf is not None:
            holder = {}
            t = timed(lambda: holder.__setitem__("o", hf.generate(ids, attention_mask=torch.ones_like(ids),
                                                                   max_new_tokens=a.new, min_new_tokens=a.new,
                                                                   do_sample=False, use_cache=True, pad_token_id=0)))
            row["hf_tok_per_s"] = round(B * a.new / t, 1)
            row["hf_ms_per_token"] = round(t / a.new * 1e3, 3)
            row["speedup_vs_hf"] = round(row["nbd_graph_tok_per_s"] / row["hf_tok_per_s"], 2)
            # greedy tokens agree until the first bf16 near-tie
            same = (holder["o"][:, a.prompt:] == g_out[:, a.prompt:]).float().cumprod(-1).sum(-1)
            row["tokens_agreeing_with_hf_mean"] = round(float(same.mean()), 1)
        print(json.dumps(row), flush=True)
        res["runs"].append(row)
    if a.model != "gpt2":
        if a.out:
            with open(a.out, "w") as f:
                json.dump(res, f, indent=1)
        return
    res["decode_kernel"] = kernel_bench([(1, 12, 12, 1024), (8, 12, 12, 1024), (32, 12, 12, 1024), (8, 32, 8, 8192),
                                         (1, 32, 8, 32768), (64, 12, 12, 2048)])
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
