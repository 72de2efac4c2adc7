"""Fused optimizer kernels over flat buffers (GPU: gfx950 kernels; CPU: torch math).

Parity: reference adam / momentum / sgd ops (paddle/fluid/operators/adam_op.h:35-321,
momentum_op.cu:67, sgd_op.cu:73).  The GPU path updates a whole flat parameter
shard in one launch and writes the bf16 model copy in the same pass.
"""
from __future__ import annotations

import torch

from . import _native as N
from . import fused as _fused


def adamw_flat(param, grad, m, v, *, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
               step=1, param_out=None, decay_end=None, grad_scale=1.0, lr_tensor=None,
               beta1_pow=None, beta2_pow=None, grad_scale_tensor=None, lr_t_eps=False):
    """In-place AdamW on fp32 ``param`` (flat, contiguous) with fp32 moments.

    ``decay_end``: elements with index < decay_end get decoupled weight decay
    (the flat layout puts all decayed params first).  ``param_out``: optional
    bf16/fp32 copy written in the same pass.  ``lr_tensor``/``beta*_pow``:
    device scalars (static-graph adam op semantics, no host sync).  ``lr_t_eps``:
    Kingma/Paddle epsilon placement (adam_op.h): p -= lr*sqrt(1-b2^t)/(1-b1^t) * m/(sqrt(v)+eps).
    """
    n = param.numel()
    if decay_end is None:
        decay_end = n
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    if param.is_cuda:
        _fused.bump_weight_epoch()
        N.call("pa_adamw", N.dt(grad), (N.dt(param_out) if param_out is not None else -1), N.ptr(param),
               N.ptr(grad), N.ptr(m), N.ptr(v), N.ptr(param_out), n, float(lr), N.ptr(lr_tensor),
               float(beta1), float(beta2), float(eps), float(weight_decay), float(bc1), float(bc2),
               N.ptr(beta1_pow), N.ptr(beta2_pow), int(decay_end), float(grad_scale),
               N.ptr(grad_scale_tensor), int(lr_t_eps), N.stream())
        return param
    lr_ = float(lr_tensor.reshape(-1)[0]) if lr_tensor is not None else lr
    if beta1_pow is not None:
        bc1 = 1.0 - float(beta1_pow.reshape(-1)[0])
        bc2 = 1.0 - float(beta2_pow.reshape(-1)[0])
    gs = grad_scale * (float(grad_scale_tensor.reshape(-1)[0]) if grad_scale_tensor is not None else 1.0)
    g = grad.float() * gs
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    if weight_decay:
        idx = torch.arange(n, device=param.device) < decay_end
        param.mul_(torch.where(idx, 1 - lr_ * weight_decay, 1.0))
    e = eps / (bc2 ** 0.5) if lr_t_eps else eps
    param.addcdiv_(m / bc1, (v / bc2).sqrt_().add_(e), value=-lr_)
    if param_out is not None:
        param_out.copy_(param)
    return param


def momentum_flat(param, grad, velocity=None, *, lr, mu=0.9, nesterov=False, weight_decay=0.0,
                  grad_scale=1.0, lr_tensor=None):
    n = param.numel()
    if param.is_cuda:
        _fused.bump_weight_epoch()
        if param.dtype not in (torch.float32, torch.bfloat16) or not param.is_contiguous():
            raise TypeError(f"momentum_flat: contiguous fp32 / bf16 parameter required, got {param.dtype}")
        N.call("pa_momentum_p", N.dt(grad), N.dt(param), N.ptr(param), N.ptr(grad), N.ptr(velocity), n,
               float(lr), N.ptr(lr_tensor), float(mu), int(nesterov), float(weight_decay), float(grad_scale),
               N.stream())
        return param
    lr_ = float(lr_tensor.reshape(-1)[0]) if lr_tensor is not None else lr
    pf = param.float()
    g = grad.float() * grad_scale + weight_decay * pf
    if velocity is None:
        param.copy_(pf - lr_ * g)
        return param
    velocity.mul_(mu).add_(g)
    param.copy_(pf - (lr_ * (g + mu * velocity) if nesterov else lr_ * velocity))
    return param


def sumsq(x, out=None):
    """Sum of squares into a 1-element fp32 tensor (accumulates into ``out``)."""
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=x.device)
    if x.is_cuda:
        N.call("pa_sumsq", N.dt(x), N.ptr(x), x.numel(), N.ptr(out), N.stream())
    else:
        out += x.float().pow(2).sum()
    return out
