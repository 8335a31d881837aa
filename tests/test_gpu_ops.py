"""GPU numerics: the HIP kernels (torch.ops.nbd.*) against plain PyTorch fp32 references."""
import math

import pytest
import torch

from nbdistributed_amd import ops

pytestmark = pytest.mark.gpu

DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


@pytest.fixture(scope="module")
def dev(require_gpu):
    assert ops.native_available(), ops._load_error
    return torch.device("cuda", 0)


def _tensors(dev, dtype, sizes, misalign=False):
    g = torch.Generator(device="cpu").manual_seed(0)
    out = []
    for i, n in enumerate(sizes):
        if misalign and i % 3 == 1:
            big = torch.randn(n + 1, generator=g).to(dev, dtype)
            out.append(big[1:])  # contiguous, data pointer not 16-B aligned
        else:
            out.append(torch.randn(n, generator=g).to(dev, dtype))
    return out


SIZES = [1, 7, 8, 9, 1000, 16383, 16384, 16385, 100003, 3 * 16384 + 5]


@pytest.mark.parametrize("src", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("dst", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("misalign", [False, True])
def test_bucket_flatten_matches_reference(dev, src, dst, misalign):
    ts = _tensors(dev, DT[src], SIZES, misalign)
    offsets, total = ops.plan_offsets([t.numel() for t in ts])
    if misalign:
        offsets = [o + (i % 2) for i, o in enumerate(offsets)]  # odd bucket offsets too
        total += 1
    b = torch.full((total,), 7.0, device=dev, dtype=DT[dst])
    ref = b.clone()
    ops.bucket_flatten(ts, b, offsets, scale=0.25)
    ops._ref_flatten(ts, ref, offsets, 0.25)
    torch.testing.assert_close(b.float(), ref.float(), rtol=0, atol=0)


@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("src,dst", [("bf16", "f32"), ("f32", "f32"), ("f32", "bf16"), ("f16", "f32")])
def test_bucket_unflatten_matches_reference(dev, src, dst, accumulate):
    sizes = SIZES + [5] * 70  # > 64 tensors: several launches
    offsets, total = ops.plan_offsets(sizes)
    bucket = torch.randn(total, device=dev).to(DT[src])
    outs = _tensors(dev, DT[dst], sizes)
    refs = [t.clone() for t in outs]
    ops.bucket_unflatten(bucket, outs, offsets, scale=1.0 / 8, accumulate=accumulate)
    ops._ref_unflatten(bucket, refs, offsets, 1.0 / 8, accumulate)
    tol = 0 if not accumulate else (1e-6 if dst == "f32" else 1e-2)
    for a, r in zip(outs, refs):
        torch.testing.assert_close(a.float(), r.float(), rtol=tol, atol=tol)


def test_flatten_unflatten_roundtrip_many_tensors(dev):
    ts = _tensors(dev, torch.float32, [(i * 37) % 5000 + 1 for i in range(200)])
    b, offs = ops.bucket_flatten(ts, dtype=torch.float32)
    outs = [torch.empty_like(t) for t in ts]
    ops.bucket_unflatten(b, outs, offs)
    for a, t in zip(outs, ts):
        assert torch.equal(a, t)


@pytest.mark.parametrize("k", [1, 2, 5, 16, 21])
@pytest.mark.parametrize("src,dst", [("bf16", "bf16"), ("f32", "f32"), ("bf16", "f32"), ("f16", "f16")])
def test_local_prereduce_matches_reference(dev, k, src, dst):
    n = 1_000_003
    xs = [torch.randn(n, device=dev).to(DT[src]) for _ in range(k)]
    out = torch.empty(n, device=dev, dtype=DT[dst])
    ops.local_prereduce(xs, out, scale=1.0 / k)
    ref = torch.stack([x.float() for x in xs]).sum(0) / k
    tol = 1e-5 if dst == "f32" else 1e-2
    torch.testing.assert_close(out.float(), ref, rtol=tol, atol=tol)


def _check_summary(x):
    got = ops.tensor_summary(x)
    ref = dict(zip(ops.SUMMARY_FIELDS, ops._ref_summary(x.cpu()).tolist()))
    n = x.numel()
    assert got["count"] == n
    assert got["nan"] == int(ref["nan"]) and got["inf"] == int(ref["inf"])
    if n == 0:
        return got
    scale = float(x.detach().double().abs().sum()) + 1e-12
    if got["nan"] == 0 and got["inf"] == 0:
        assert abs(got["sum"] - ref["sum"]) <= 2e-6 * scale + 1e-6
        assert math.isclose(got["norm"], ref["norm"], rel_tol=2e-5, abs_tol=1e-6)
        if n > 1:
            assert math.isclose(got["std"], ref["std"], rel_tol=1e-3, abs_tol=1e-6)
    assert got["min"] == ref["min"] and got["max"] == ref["max"] and got["absmax"] == ref["absmax"]
    return got


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("n", [0, 1, 511, 512, 513, 4099, 1_000_003, 50_000_017])
def test_tensor_summary_matches_reference(dev, dtype, n):
    x = (torch.randn(n, device=dev) * 3 + 0.5).to(DT[dtype])
    _check_summary(x)


@pytest.mark.parametrize("dtype", ["f32", "bf16", "f16"])
def test_tensor_summary_misaligned_and_nonfinite(dev, dtype):
    big = torch.randn(100_000, device=dev).to(DT[dtype])
    x = big[3:]  # misaligned start
    x[10] = float("nan")
    x[20] = float("inf")
    x[5000] = float("-inf")
    got = _check_summary(x)
    assert got["nan"] == 1 and got["inf"] == 2 and math.isnan(got["sum"])


def test_tensor_summary_large_mean_small_spread_f32(dev):
    x = 1000.0 + 1e-3 * torch.randn(4_000_000, device=dev)
    got = ops.tensor_summary(x)
    assert math.isclose(got["std"], float(x.double().std()), rel_tol=1e-3)


def test_tensor_summary_2d_noncontiguous(dev):
    x = torch.randn(1024, 2048, device=dev, dtype=torch.bfloat16).t()
    _check_summary(x)


@pytest.mark.parametrize("gdt", ["f32", "bf16"])
@pytest.mark.parametrize("pdt", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("n", [1, 7, 8, 1000, 16389, 1 << 20, (1 << 23) + 37])  # (the last: every thread runs its unrolled groups)
@pytest.mark.parametrize("clip", [False, True])
def test_adamw_flat_matches_reference(dev, gdt, pdt, n, clip):
    g = torch.Generator(device="cpu").manual_seed(n)
    master = torch.randn(n, generator=g)
    grads = [torch.randn(n, generator=g).to(DT[gdt]) for _ in range(3)]
    coef = torch.tensor([0.37]) if clip else None
    ref = [master.clone(), torch.zeros(n), torch.zeros(n), master.to(DT[pdt])]
    gpu = [t.clone().to(dev) for t in ref]
    for step, gr in enumerate(grads, 1):
        ops._ref_adamw(gr, ref[3], ref[0], ref[1], ref[2], 1e-3, 0.9, 0.95, 1e-8, 0.1, step, 0.5, coef)
        ops.adamw_flat(gr.to(dev), gpu[3], gpu[0], gpu[1], gpu[2], 1e-3, 0.9, 0.95, 1e-8, 0.1, step, 0.5,
                       coef.to(dev) if clip else None)
    torch.cuda.synchronize()
    for name, a, b in zip(("master", "exp_avg", "exp_avg_sq"), ref[:3], gpu[:3]):
        assert torch.allclose(b.cpu(), a, atol=1e-6, rtol=1e-5), name
    # the param copy is the master cast to its dtype (round-to-nearest both ways)
    assert torch.equal(gpu[3].cpu(), gpu[0].cpu().to(DT[pdt]))


@pytest.mark.parametrize("capturable", [False, True])
def test_adamw_flat_multi_one_launch_matches_per_bucket(dev, capturable):
    """adamw_flat_multi's single launch over all buckets (adamw_multi_kernel; sizes with and
    without a < 8-element tail, one bucket of 7 elements) bit-identical to one adamw_flat launch per
    bucket, incl. the device-side clip coefficient and the capturable step / lr scalars."""
    g = torch.Generator(device="cpu").manual_seed(5)
    sizes = [1 << 20, 7, 16389, 4096 + 3, (1 << 18) + 8]
    coef = torch.tensor([0.37], device=dev)
    sets = []
    for _ in range(2):
        bufs = []
        for n in sizes:
            master = torch.randn(n, generator=g).to(dev) if not sets else sets[0][len(bufs)][1].clone()
            bufs.append([None, master, torch.zeros(n, device=dev), torch.zeros(n, device=dev),
                         master.to(torch.bfloat16)])
        sets.append(bufs)
    grads = [[torch.randn(n, generator=g).to(dev, torch.bfloat16) for n in sizes] for _ in range(3)]
    st = [torch.zeros(1, device=dev) for _ in range(2)]
    lr_t = [torch.full((1,), 1e-3, device=dev) for _ in range(2)]
    for step, gr in enumerate(grads, 1):
        a, b = sets
        for t in st:
            t.add_(1.0)
        torch.ops.nbd.adamw_flat_multi(gr, [x[4] for x in a], [x[1] for x in a], [x[2] for x in a],
                                       [x[3] for x in a], 1e-3, 0.9, 0.95, 1e-8, 0.1, step, 0.5, coef,
                                       st[0] if capturable else None, lr_t[0] if capturable else None)
        for i, x in enumerate(b):
            ops.adamw_flat(gr[i], x[4], x[1], x[2], x[3], 1e-3, 0.9, 0.95, 1e-8, 0.1, step, 0.5, coef,
                           step_t=st[1] if capturable else None, lr_t=lr_t[1] if capturable else None)
    torch.cuda.synchronize()
    for x, y in zip(*sets):
        for u, v in zip(x[1:], y[1:]):
            assert torch.equal(u, v)


@pytest.mark.parametrize("dt", ["f32", "bf16", "f16"])
@pytest.mark.parametrize("V", [1, 7, 64, 1000, 50257])
@pytest.mark.parametrize("inplace", [False, True])
def test_cross_entropy_matches_reference(dev, dt, V, inplace):
    import torch.nn.functional as F

    g = torch.Generator(device="cpu").manual_seed(V)
    N = 67
    x32 = (torch.randn(N, V, generator=g) * 3).to(DT[dt]).float()
    tgt = torch.randint(0, V, (N,), generator=g)
    tgt[::5] = -100  # ignored rows
    ref_x = x32.clone().requires_grad_(True)
    ref = F.cross_entropy(ref_x, tgt)
    (ref * 2.5).backward()
    x = x32.to(dev, DT[dt]).requires_grad_(True)
    y = x * 1.0 if inplace else x  # in-place backward needs a non-leaf (it overwrites the storage)
    loss = ops.cross_entropy(y, tgt.to(dev), inplace_backward=inplace)
    (loss * 2.5).backward()
    torch.cuda.synchronize()
    tol = 1e-5 if dt == "f32" else 2e-2
    loss, ref = float(loss.detach()), float(ref.detach())
    assert abs(loss - ref) <= 1e-4 * max(1.0, abs(ref)), (loss, ref)
    gref = ref_x.grad
    assert torch.allclose(x.grad.float().cpu(), gref, atol=tol * float(gref.abs().max()) + 1e-7, rtol=tol)


def test_cross_entropy_strided_rows_and_sum(dev):
    import torch.nn.functional as F

    base = torch.randn(33, 1030, device=dev, dtype=torch.bfloat16)
    x = base[:, 3:1003]  # row stride 1030, misaligned start, unit column stride
    tgt = torch.randint(0, 1000, (33,), device=dev)
    got = ops.cross_entropy(x, tgt, reduction="sum")
    ref = F.cross_entropy(x.float(), tgt, reduction="sum")
    assert abs(float(got) - float(ref)) < 1e-3 * abs(float(ref))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding_tok_pos_matches_two_lookups(dtype):
    from nbdistributed_amd import ops

    g = torch.Generator(device="cuda").manual_seed(0)
    V, P, C, B, T = 1000, 256, 768, 3, 128
    wte = torch.randn(V, C, device="cuda", generator=g).to(dtype).requires_grad_()
    wpe = torch.randn(P, C, device="cuda", generator=g).to(dtype).requires_grad_()
    idx = torch.randint(0, V, (B, T), device="cuda", generator=g)
    idx[0, :40] = 7  # a frequent id
    pos = torch.arange(64, 64 + T, device="cuda")
    y = ops.embedding_tok_pos(idx, wte, pos, wpe)
    ref = torch.nn.functional.embedding(idx, wte) + torch.nn.functional.embedding(pos, wpe)
    assert torch.equal(y, ref)  # one fp32 add, one rounding: the same bits
    dy = torch.randn(B, T, C, device="cuda", generator=g).to(dtype)
    gt, gp = torch.autograd.grad(y, (wte, wpe), dy)
    rt, rp = torch.autograd.grad(ref, (wte, wpe), dy)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    assert (gt.float() - rt.float()).abs().max() <= tol * rt.float().abs().max()
    assert (gp.float() - rp.float()).abs().max() <= tol * rp.float().abs().max()
    assert float(gp[:64].float().abs().max()) == 0.0 and float(gp[64 + T:].float().abs().max()) == 0.0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_embedding_pos_bwd_op(dtype):
    """The position table's gradient in one launch: permuted positions covering every row (no
    zero fill), a partial cover (rows left zero), and accumulation into a given buffer — against
    fp32 sum + index_add."""
    g = torch.Generator(device="cuda").manual_seed(1)
    B, T, C = 4, 96, 256
    dy = torch.randn(B * T, C, device="cuda", generator=g).to(dtype)
    ref_rows = dy.float().view(B, T, C).sum(0)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    pos = torch.randperm(T, device="cuda", generator=g)
    got = torch.ops.nbd.embedding_pos_bwd(dy, pos, T)
    ref = torch.zeros(T, C, device="cuda").index_add_(0, pos, ref_rows)
    assert (got.float() - ref).abs().max() <= tol * ref.abs().max()
    P = 200
    pos2 = torch.arange(50, 50 + T, device="cuda")
    got2 = torch.ops.nbd.embedding_pos_bwd(dy, pos2, P)
    ref2 = torch.zeros(P, C, device="cuda").index_add_(0, pos2, ref_rows)
    assert (got2.float() - ref2).abs().max() <= tol * ref2.abs().max()
    assert float(got2[:50].float().abs().max()) == 0.0 and float(got2[50 + T:].float().abs().max()) == 0.0
    base = torch.randn(P, C, device="cuda", generator=g).to(dtype)
    acc = base.clone()
    torch.ops.nbd.embedding_pos_bwd(dy, pos2, P, acc, True)
    ref3 = base.float() + ref2
    assert (acc.float() - ref3).abs().max() <= 2 * tol * ref3.abs().max()
