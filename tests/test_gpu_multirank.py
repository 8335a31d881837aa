"""GPU, world size 2 on one MI355X: two workers share GPU 0 over the gloo backend (gloo stages
CUDA tensors through the host; RCCL refuses two ranks on one device).  This runs the
multi-rank DDP code with real HIP streams: the side-stream bucket pipeline, flat parameters,
FlatAdamW, the fused kernels — against torch DDP + torch AdamW on the same data."""
import pytest

from nbdistributed_amd.session import Session

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sess(require_gpu):
    s = Session(writer=lambda t: None)
    s.start(2, backend="gloo", gpu_ids=[0, 0], startup_timeout=600, timeout=600)
    yield s
    s.shutdown()


def test_two_ranks_share_gpu0(sess):
    r = sess.execute("(str(device), dist.get_backend(), world_size)", render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "('cuda:0', 'gloo', 2)", r.results[rank]


SETUP = """
import copy
import torch.nn as nn
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
from torch.nn.parallel import DistributedDataParallel as TorchDDP

class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(256, 512)
        self.b = nn.Linear(512, 512)
        self.c = nn.Linear(512, 64)
    def forward(self, x):
        return self.c(torch.relu(self.b(torch.relu(self.a(x)))))

torch.manual_seed(11 + rank)              # different init per rank: DDP broadcasts rank 0's
base = Net().to(device)
ref = TorchDDP(copy.deepcopy(base))
ours = NbdDDP(copy.deepcopy(base), bucket_cap_mb=0.5, first_bucket_mb=0.2, flat_params=True, grad_mode="bucket")
plain = NbdDDP(copy.deepcopy(base), bucket_cap_mb=0.5, first_bucket_mb=0.2)
opt_ref = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=0.01)
opt = FlatAdamW(ours, lr=1e-3, weight_decay=0.01)
(len(ours.buckets) > 1, ours.comm_stream is not None)
"""

TRAIN = """
g = torch.Generator(device="cpu").manual_seed(500 + rank)
for step in range(5):
    x = torch.randn(64, 256, generator=g).to(device)
    for model, o in ((ref, opt_ref), (ours, opt)):
        o.zero_grad(set_to_none=True)
        model(x).square().mean().backward()
        o.step()
    plain.zero_grad(set_to_none=True)
    plain(x).square().mean().backward()
    gerr = max(float((p.grad - q.grad).abs().max()) for p, q in zip(ref.module.parameters(), plain.module.parameters())) if step == 0 else 0.0
    if step == 0:
        g0 = gerr
torch.cuda.synchronize()
err = max(float((p - q).detach().abs().max()) for p, q in zip(ref.module.parameters(), ours.module.parameters()))
sig = torch.stack([p.detach().float().sum() for p in ours.module.parameters()])
other = sig.clone(); dist.broadcast(other, src=0)
(err < 1e-4, g0 < 1e-5, bool(torch.equal(sig, other)))
"""

GPT2 = """
from nbdistributed_amd.models import GPT2, GPT2Config
torch.manual_seed(3)
cfg = GPT2Config(vocab_size=2048, n_positions=256, n_embd=256, n_layer=2, n_head=4)
m = NbdDDP(GPT2(cfg).to(device, torch.bfloat16), flat_params=True, grad_mode="bucket")
o = FlatAdamW(m, lr=1e-3)
idx = torch.randint(0, 2048, (2, 256), generator=torch.Generator().manual_seed(rank)).to(device)
losses = []
for _ in range(6):
    loss = m(idx, idx, return_logits=False)[1]
    loss.backward()
    o.clip_grad_norm_(1.0)
    o.step()
    losses.append(float(loss.detach()))
sig = torch.stack([b.param_flat.float().sum() for b in m.buckets])
other = sig.clone(); dist.broadcast(other, src=0)
(losses[-1] < losses[0], bool(torch.equal(sig, other)))
"""


def test_ddp_flat_adamw_matches_torch_on_gpu_two_ranks(sess):
    r = sess.execute(SETUP, render=False)
    assert r.results[0]["echo"] == "(True, True)", r.results[0]
    r = sess.execute(TRAIN, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True, True)", r.results[rank]


def test_gpt2_hip_path_two_ranks_stay_in_sync(sess):
    r = sess.execute(GPT2, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True)", r.results[rank]


TP_GPT2 = """
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel.tensor import parallelize_gpt2
torch.manual_seed(5)                      # same init on both ranks: TP shards one replicated model
cfg = GPT2Config(vocab_size=512, n_positions=128, n_embd=256, n_layer=2, n_head=4)
ref = GPT2(cfg).to(device, torch.bfloat16)
tp = GPT2(cfg).to(device, torch.bfloat16)
tp.load_state_dict(ref.state_dict())
parallelize_gpt2(tp)
idx = torch.randint(0, 512, (2, 128), generator=torch.Generator().manual_seed(9)).to(device)
l_ref = ref(idx, idx)[1]; l_tp = tp(idx, idx)[1]
l_ref.backward(); l_tp.backward()
hid = slice(rank * 512, (rank + 1) * 512)
g_ref = ref.h[1].mlp.c_fc.weight.grad[hid].float(); g_tp = tp.h[1].mlp.c_fc.weight.grad.float()
gerr = ((g_tp - g_ref).abs().max() / g_ref.abs().max()).item()
w_err = ((tp.wte.weight.grad.float() - ref.wte.weight.grad.float()).abs().max()
         / ref.wte.weight.grad.float().abs().max()).item()
(abs(float(l_tp) - float(l_ref)) < 2e-2 * abs(float(l_ref)), gerr < 5e-2, w_err < 5e-2, tp.h[0].attn.n_head)
"""


def test_tensor_parallel_gpt2_hip_path_two_ranks(sess):
    """parallel.tensor: GPT-2 heads / MLP features split over 2 ranks (HIP GEMM + flash attention
    on the shards) = the unsharded bf16 model on the same rank."""
    r = sess.execute(TP_GPT2, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True, True, 2)", r.results[rank]


ULYSSES = """
from nbdistributed_amd.parallel.sequence import ulysses_attention, shard_sequence
torch.manual_seed(6)
q = torch.randn(1, 4, 256, 64, device=device, dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(1, 4, 256, 64, device=device, dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(1, 4, 256, 64, device=device, dtype=torch.bfloat16, requires_grad=True)
w = torch.randn(1, 4, 256, 64, device=device, dtype=torch.bfloat16)
ref = nbd.ops.flash_attention(q, k, v, causal=True)
(ref.float() * w.float()).sum().backward()
ql, kl, vl = (shard_sequence(t.detach(), dim=2).clone().requires_grad_() for t in (q, k, v))
out = ulysses_attention(ql, kl, vl, causal=True)
(out.float() * shard_sequence(w, dim=2).float()).sum().backward()
def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
(_rel(out, shard_sequence(ref.detach(), dim=2)) < 2e-2, _rel(kl.grad, shard_sequence(k.grad, dim=2)) < 5e-2)
"""


def test_ulysses_attention_hip_path_two_ranks(sess):
    """parallel.sequence: sequence split over 2 ranks, all-to-all to heads, HIP flash attention on the
    full sequence (T = 256), all-to-all back = flash attention on the unsplit sequence."""
    r = sess.execute(ULYSSES, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True)", r.results[rank]


MOE = """
from nbdistributed_amd.parallel.expert import MoE
torch.manual_seed(4)
moe = MoE(256, 512, 4, top_k=2).to(device, torch.bfloat16)
x = torch.randn(512, 256, generator=torch.Generator().manual_seed(rank)).to(device, torch.bfloat16)
x.requires_grad_()
y = moe(x)
y.float().square().mean().backward()
# every token gets exactly top_k expert outputs: compare to the dense gather over this rank's own experts
# on the other rank via a round trip of the weights (forward only)
parts = [torch.empty_like(moe.w1) for _ in range(2)]; dist.all_gather(parts, moe.w1.detach()); w1 = torch.cat(parts)
parts = [torch.empty_like(moe.w2) for _ in range(2)]; dist.all_gather(parts, moe.w2.detach()); w2 = torch.cat(parts)
idx, gates, _ = moe.route(x.detach())
ref = torch.zeros(512, 256, device=device)
for j in range(2):
    for e in range(4):
        m = idx[:, j] == e
        h = torch.nn.functional.gelu(x.detach()[m].float() @ w1[e].float().t(), approximate="tanh") @ w2[e].float().t()
        ref[m] += h * gates[m, j:j + 1]
err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
(err < 3e-2, moe.w1.grad is not None and bool(torch.isfinite(moe.w1.grad.float()).all()), bool(torch.isfinite(x.grad.float()).all()))
"""


def test_moe_expert_parallel_two_ranks(sess):
    """parallel.expert: 4 experts split over 2 ranks, variable-split all-to-all dispatch/combine of
    bf16 CUDA tokens = the dense top-2 mixture."""
    r = sess.execute(MOE, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True, True)", r.results[rank]


RING = """
from nbdistributed_amd.parallel.context import ring_attention, shard_context
torch.manual_seed(8)
q = torch.randn(1, 4, 512, 64, device=device, dtype=torch.bfloat16, requires_grad=True)
k = torch.randn(1, 2, 512, 64, device=device, dtype=torch.bfloat16, requires_grad=True)
v = torch.randn(1, 2, 512, 64, device=device, dtype=torch.bfloat16, requires_grad=True)
w = torch.randn(1, 4, 512, 64, device=device, dtype=torch.bfloat16)
ref = nbd.ops.flash_attention(q, k, v, causal=True)
(ref.float() * w.float()).sum().backward()
def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
oks = []
for layout in ("contiguous", "zigzag"):
    sh = lambda t: shard_context(t, dim=2, layout=layout)
    ql, kl, vl = (sh(t.detach()).clone().requires_grad_() for t in (q, k, v))
    out = ring_attention(ql, kl, vl, causal=True, layout=layout)
    (out.float() * sh(w).float()).sum().backward()
    oks.append(_rel(out, sh(ref.detach())) < 2e-2 and _rel(ql.grad, sh(q.grad)) < 5e-2
               and _rel(kl.grad, sh(k.grad)) < 5e-2 and _rel(vl.grad, sh(v.grad)) < 5e-2)
tuple(oks)
"""


def test_ring_attention_hip_path_two_ranks(sess):
    """parallel.context: a 512-token causal GQA sequence split over 2 ranks (contiguous: 256-token
    chunks, zigzag: 2 x 128), K/V passed round the ring, HIP flash kernels per block = flash
    attention on the unsplit sequence (outputs and q/k/v gradients)."""
    r = sess.execute(RING, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True)", r.results[rank]


CP_GPT2 = """
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel.context import parallelize_gpt2_context, shard_context
torch.manual_seed(3)
c = GPT2Config(vocab_size=512, n_positions=512, n_embd=128, n_layer=2, n_head=2)
ref = GPT2(c).to(device, torch.bfloat16)
cp = GPT2(c).to(device, torch.bfloat16)
cp.load_state_dict(ref.state_dict())
parallelize_gpt2_context(cp, layout="zigzag")
g = torch.Generator().manual_seed(4)
idx = torch.randint(0, 512, (2, 512), generator=g).to(device)
tgt = torch.randint(0, 512, (2, 512), generator=g).to(device)
_, lr_ = ref(idx, tgt)
lr_.backward()
_, l = cp(shard_context(idx, dim=1, layout="zigzag"), shard_context(tgt, dim=1, layout="zigzag"))
l.backward()
tot = l.detach().float().clone(); dist.all_reduce(tot)
gq = cp.h[0].attn.c_attn.weight.grad.float().clone(); dist.all_reduce(gq)
gr = ref.h[0].attn.c_attn.weight.grad.float()
(abs(tot.item() / 2 - lr_.item()) < 2e-2, ((gq / 2 - gr).abs().max() / gr.abs().max()).item() < 5e-2)
"""


def test_context_parallel_gpt2_hip_path_two_ranks(sess):
    """parallel.context: bf16 GPT-2 with each 512-token sequence zigzag-split over 2 ranks (HIP
    GEMM / LayerNorm / ring-attention blocks of 128 tokens) = the unsplit model (loss, c_attn grad)."""
    r = sess.execute(CP_GPT2, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True)", r.results[rank]


CP_LLAMA = """
from nbdistributed_amd.models.llama import LlamaConfig, LlamaModel
from nbdistributed_amd.parallel.context import parallelize_llama_context, shard_context
torch.manual_seed(5)
c = LlamaConfig.tiny()
ref = LlamaModel(c).to(device, torch.bfloat16)
cp = LlamaModel(c).to(device, torch.bfloat16)
cp.load_state_dict(ref.state_dict())
parallelize_llama_context(cp, layout="zigzag")
g = torch.Generator().manual_seed(6)
ids = torch.randint(0, 512, (2, 512), generator=g).to(device)
w = torch.randn(2, 512, 256, generator=g).to(device, torch.bfloat16)
h_ref = ref(ids)
(h_ref.float() * w.float()).sum().backward()
h = cp(shard_context(ids, dim=1, layout="zigzag"))
(h.float() * shard_context(w, dim=1, layout="zigzag").float()).sum().backward()
hs = shard_context(h_ref.detach(), dim=1, layout="zigzag")
gq = cp.layers[0].self_attn.qkv_proj.weight.grad.float().clone(); dist.all_reduce(gq)
gr = ref.layers[0].self_attn.qkv_proj.weight.grad.float()
(((h.float() - hs.float()).abs().max() / hs.float().abs().max()).item() < 3e-2,
 ((gq - gr).abs().max() / gr.abs().max()).item() < 5e-2)
"""


def test_context_parallel_llama_hip_path_two_ranks(sess):
    """parallel.context: bf16 native Llama (GQA, RoPE at global positions by nbd::rope_) with each
    512-token sequence zigzag-split over 2 ranks = the unsplit model (hidden states, qkv grad)."""
    r = sess.execute(CP_LLAMA, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True)", r.results[rank]


CP_DDP = """
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel import DistributedDataParallel, ParallelMesh
from nbdistributed_amd.parallel.context import parallelize_gpt2_context, shard_context
from nbdistributed_amd.optim import FlatAdamW
mesh = ParallelMesh(cp=world_size)
torch.manual_seed(0)
cfg = GPT2Config(vocab_size=1024, n_positions=2048, n_embd=256, n_layer=2, n_head=4)
model = GPT2(cfg).to(device, torch.bfloat16)
parallelize_gpt2_context(model, group=mesh.group('cp'), layout='zigzag')
ddp = DistributedDataParallel(model, flat_params=True, grad_mode='bucket')
opt = FlatAdamW(ddp, lr=1e-3)
g = torch.Generator().manual_seed(1)
idx = torch.randint(0, 1024, (2, 2048), generator=g)
tgt = torch.roll(idx, -1, 1)
x, y = (shard_context(t, dim=1, layout='zigzag').to(device) for t in (idx, tgt))
losses = []
for step in range(3):
    _, loss = ddp(x, y, return_logits=False)
    loss.backward()
    opt.step()
    opt.zero_grad(set_to_none=True)
    l = loss.detach().float(); dist.all_reduce(l); losses.append((l / world_size).item())
w = model.h[0].attn.c_attn.weight.detach().float().clone()
w0 = w.clone(); dist.broadcast(w0, 0)
(all(map(math.isfinite, losses)), losses[-1] < losses[0], torch.equal(w, w0))
"""


def test_context_parallel_ddp_training_two_ranks(sess):
    """examples/02_context_parallel.ipynb's loop: CP GPT-2 (zigzag ring attention over a mesh
    group) under nbd DDP (flat bucket grads) + FlatAdamW — finite, decreasing loss, replicas in sync."""
    r = sess.execute("import math\n" + CP_DDP, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True, True)", r.results[rank]


CP_LLAMA_LM = """
from nbdistributed_amd.models.llama import LlamaConfig, LlamaForCausalLM
from nbdistributed_amd.parallel.context import parallelize_llama_context, shard_context, shift_labels
torch.manual_seed(5)
c = LlamaConfig.tiny()
ref = LlamaForCausalLM(c).to(device, torch.bfloat16)
cp = LlamaForCausalLM(c).to(device, torch.bfloat16)
cp.load_state_dict(ref.state_dict())
parallelize_llama_context(cp, layout="zigzag")
g = torch.Generator().manual_seed(6)
ids = torch.randint(0, 512, (2, 512), generator=g)
labels = ids.clone(); labels[0, :200] = -100
ids, labels = ids.to(device), labels.to(device)
lr_, _ = ref(ids, labels)
lr_.backward()
sh = lambda t: shard_context(t, dim=1, layout="zigzag")
l, _ = cp(sh(ids), sh(shift_labels(labels)), return_logits=False)
l.backward()
tot = l.detach().float().clone(); dist.all_reduce(tot)
gq = cp.model.layers[0].self_attn.qkv_proj.weight.grad.float().clone(); dist.all_reduce(gq)
gr = ref.model.layers[0].self_attn.qkv_proj.weight.grad.float()
(abs(tot.item() / 2 - lr_.item()) < 2e-2, ((gq / 2 - gr).abs().max() / gr.abs().max()).item() < 5e-2)
"""


def test_context_parallel_llama_causal_lm_hip_path_two_ranks(sess):
    """parallel.context: bf16 LlamaForCausalLM, labels shifted on the full sequence and zigzag-
    sharded over 2 ranks, 200 ignored prompt tokens (uneven per shard) — averaged loss and qkv
    gradient = the unsplit model's (HIP cross-entropy with reduction='sum' + context_loss)."""
    r = sess.execute(CP_LLAMA_LM, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True)", r.results[rank]


ZERO_GPT2 = """
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel import DistributedDataParallel as NbdDDP
from nbdistributed_amd.optim import FlatAdamW
torch.manual_seed(3)
cfg = GPT2Config(vocab_size=2048, n_positions=256, n_embd=256, n_layer=2, n_head=4)
base = GPT2(cfg).to(device, torch.bfloat16)
import copy
mf = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", bucket_cap_mb=1.0)
mz = NbdDDP(copy.deepcopy(base), flat_params=True, grad_mode="bucket", bucket_cap_mb=1.0, shard=True)
of, oz = FlatAdamW(mf, lr=1e-3), FlatAdamW(mz, lr=1e-3)
idx = torch.randint(0, 2048, (2, 256), generator=torch.Generator().manual_seed(rank)).to(device)
lf, lz, nf, nz = [], [], [], []
for _ in range(4):
    for m, o, ls in ((mf, of, lf), (mz, oz, lz)):
        loss = m(idx, idx, return_logits=False)[1]
        loss.backward()
        (nf if o is of else nz).append(float(o.clip_grad_norm_(1e9)))  # the norm only: coefficient 1
        o.step()
        ls.append(float(loss.detach()))
mz.wait_params()
torch.cuda.synchronize()
err = max(float((p.float() - q.float()).abs().max()) for p, q in zip(mf.module.parameters(), mz.module.parameters()))
sig = torch.stack([b.param_flat.float().sum() for b in mz.buckets])
other = sig.clone(); dist.broadcast(other, src=0)
(err == 0.0, lf == lz, all(abs(a - b) <= 1e-6 * a for a, b in zip(nf, nz)), bool(torch.equal(sig, other)))
"""


def test_zero2_gpt2_matches_unsharded_two_ranks(sess):
    # the sharded update is the same kernel on a slice of the same averaged gradient: the
    # parameters stay bit-identical to the unsharded DDP + FlatAdamW (a clip coefficient < 1
    # would differ in its last bits — the norm's squares are summed in another order — and
    # Adam amplifies that on near-zero gradients, so the norm is compared, not clipped with)
    r = sess.execute(ZERO_GPT2, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, True, True, True)", r.results[rank]


TP_GENERATE = """
import copy
from nbdistributed_amd.models import GPT2, GPT2Config
from nbdistributed_amd.parallel.tensor import parallelize_gpt2
torch.manual_seed(6)
ref = GPT2(GPT2Config(vocab_size=512, n_positions=256, n_embd=256, n_layer=2, n_head=4)).to(device, torch.bfloat16).eval()
with torch.no_grad():
    ref.wte.weight.mul_(8.0)              # peaked logits: greedy tokens far from bf16 ties
tp = parallelize_gpt2(copy.deepcopy(ref))
ids = torch.randint(1, 512, (3, 40), generator=torch.Generator().manual_seed(4)).to(device)
lens = torch.tensor([40, 23, 7], device=device)
want = ref.generate(ids, 16, lengths=lens, graph=False)
got = tp.generate(ids, 16, lengths=lens, graph=False)   # gloo all-reduces: no graph capture
(bool(torch.equal(got, want)), tp.kv_layout()[1])
"""


def test_tensor_parallel_generation_two_ranks(sess):
    """Generation with heads / MLP features and the KV cache split over 2 ranks (decode kernels on
    the shards, one all-reduce per half block) = the unsharded bf16 model's tokens."""
    r = sess.execute(TP_GENERATE, render=False)
    for rank in (0, 1):
        assert r.results[rank]["echo"] == "(True, 2)", r.results[rank]
