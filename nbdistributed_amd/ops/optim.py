"""Fused flat AdamW over DDP buckets (K5)."""
from __future__ import annotations

from ._lib import _require


def _ref_adamw(grad, param, master, m, v, lr, beta1, beta2, eps, wd, step, grad_scale, grad_scale_t=None,
               step_t=None, lr_t=None):
    import math

    if step_t is not None:
        step, lr = float(step_t.reshape(())), float(lr_t.reshape(()))
    n = param.numel()
    g = grad.reshape(-1)[:n].float() * grad_scale
    if grad_scale_t is not None:
        g = g * grad_scale_t.float().reshape(())
    master.mul_(1 - lr * wd)
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    master.addcdiv_(m, denom, value=-lr / bc1)
    param.view(-1).copy_(master.to(param.dtype))

def adamw_flat(grad, param, master, exp_avg, exp_avg_sq, lr: float, beta1: float, beta2: float, eps: float,
               weight_decay: float, step: int, grad_scale: float = 1.0, grad_scale_t=None, step_t=None,
               lr_t=None) -> None:
    """One fused AdamW step over flat buffers (see csrc/kernels/optim.hip): fp32 master weights
    and moments, ``param`` (any float dtype) rewritten from the master copy.  The gradient is
    multiplied by ``grad_scale`` and, if given, by the 1-element device tensor ``grad_scale_t``
    (a clip coefficient computed on the GPU — no host sync).  ``step_t``/``lr_t`` (1-element
    float32 device tensors, together) override ``step``/``lr`` for HIP-graph replay."""
    import torch

    if param.is_cuda:
        _require()
        torch.ops.nbd.adamw_flat(grad, param, master, exp_avg, exp_avg_sq, float(lr), float(beta1), float(beta2),
                                 float(eps), float(weight_decay), int(step), float(grad_scale), grad_scale_t,
                                 step_t, lr_t)
    else:
        _ref_adamw(grad, param, master, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step, grad_scale,
                   grad_scale_t, step_t, lr_t)
