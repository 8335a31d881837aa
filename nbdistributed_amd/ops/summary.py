"""One-pass device tensor summary (K4) used by the REPL echo and ``%dist_pull --summary``."""
from __future__ import annotations

from typing import Dict

from ._lib import _require


def _ref_summary(x):
    import torch

    xf = x.detach().reshape(-1).double()
    n = xf.numel()
    nan = torch.isnan(xf)
    inf = torch.isinf(xf)
    fin = xf[~nan]
    mn = float(fin.min()) if fin.numel() else float("inf")
    mx = float(fin.max()) if fin.numel() else float("-inf")
    amx = float(fin.abs().max()) if fin.numel() else 0.0
    s = float(xf.sum())
    mean = s / n if n else float("nan")
    std = float(xf.std()) if n > 1 else float("nan")
    norm = float(xf.square().sum().sqrt())
    return torch.tensor([n, s, mean, std, norm, mn, mx, amx, float(nan.sum()), float(inf.sum()),
                         n - float(nan.sum()) - float(inf.sum()), 0.0], dtype=torch.float64)


# ---------------------------------------------------------------- public API

SUMMARY_FIELDS = ("count", "sum", "mean", "std", "norm", "min", "max", "absmax", "nan", "inf", "finite", "shift")

def tensor_summary_raw(x):
    """float64[12] on x's device: see ``SUMMARY_FIELDS``."""
    import torch

    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16, torch.float16):
        _require()
        return torch.ops.nbd.tensor_summary(x.detach())
    if x.is_cuda:
        return _ref_summary(x).to(x.device)
    return _ref_summary(x)

def tensor_summary(x) -> Dict[str, float]:
    """One-pass statistics of ``x`` (HIP kernel on GPU); one 96-byte device->host copy."""
    import torch

    if not x.is_floating_point():
        x = x.float() if not x.is_cuda else x.to(torch.float32)
    raw = tensor_summary_raw(x).cpu().tolist()
    d = dict(zip(SUMMARY_FIELDS, raw))
    for k in ("count", "nan", "inf", "finite"):
        d[k] = int(d[k])
    d.pop("shift", None)
    return d

def tensor_summary_text(x) -> str:
    s = tensor_summary(x)
    shape = "x".join(str(d) for d in x.shape) or "scalar"
    parts = [f"mean={s['mean']:.6g}", f"std={s['std']:.6g}", f"min={s['min']:.6g}", f"max={s['max']:.6g}",
             f"norm={s['norm']:.6g}"]
    if s["nan"] or s["inf"]:
        parts.append(f"nan={s['nan']} inf={s['inf']}")
    return f"[{shape} {str(x.dtype).replace('torch.', '')} {x.device}] " + " ".join(parts)


__all__ = ["tensor_summary", "tensor_summary_text", "tensor_summary_raw", "SUMMARY_FIELDS"]
