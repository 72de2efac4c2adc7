"""Hand-written backward rules (VJPs) of the eager engine (``autograd/engine.py``).

Each rule is called right after the op ran, with its output and arguments, and
returns ``(inputs, backward)``: ``backward(*grad_outputs)`` gives one gradient per
entry of ``inputs`` (None for non-tensors / non-differentiable ones).  "Forward
rules" (``fwd_rule``) also compute the forward themselves, for ops whose backward
needs a by-product the plain op does not return (dropout mask, pooling indices,
batch-norm batch statistics).  Backward math runs on raw tensors with torch
autograd off: ATen kernels on the CPU and, on the GPU, whatever kernel the op's
tensors dispatch to (the hot DyGraph layers call the HIP op library instead and
record its own Function.backward, engine.record_function).

Reference: the per-op grad kernels of paddle/fluid/operators (activation_op.h,
elementwise_*_op.h, matmul_op.h, reduce_*_op.h, conv_op.h, pool_op.h,
batch_norm_op.cc, layer_norm_op.h, softmax_op.h, cross_entropy_op.h, ...).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .engine import _FWD_RULES, _wrap, inplace, nondiff, passthrough, register

T = torch.Tensor
ATEN = torch.ops.aten


def _is_t(x):
    return isinstance(x, torch.Tensor)


def _unb(g, ref):
    """Sum ``g`` down to the shape of ``ref`` (broadcast inverse); ref may be a scalar."""
    if g is None or not _is_t(ref):
        return None
    shape = ref.shape
    if g.shape == shape:
        return g.to(ref.dtype) if g.dtype != ref.dtype else g
    nd = g.dim() - len(shape)
    if nd > 0:
        g = g.sum(dim=tuple(range(nd)))
    dims = tuple(i for i, s in enumerate(shape) if s == 1 and g.shape[i] != 1)
    if dims:
        g = g.sum(dim=dims, keepdim=True)
    g = g.reshape(shape)
    return g.to(ref.dtype) if g.dtype != ref.dtype else g


def fwd_rule(*funcs):
    def deco(r):
        for f in funcs:
            _FWD_RULES[f] = r
        return r

    return deco


# =========================================================================== elementwise
@register(torch.add, T.add, T.__add__, T.__radd__)
def _add(out, a, b, alpha=1, **kw):
    return (a, b), lambda g: (_unb(g, a), _unb(g if alpha == 1 else g * alpha, b))


@register(torch.sub, T.sub, T.__sub__, torch.subtract, T.subtract)
def _sub(out, a, b, alpha=1, **kw):
    return (a, b), lambda g: (_unb(g, a), _unb(-g if alpha == 1 else -g * alpha, b))


@register(T.__rsub__)
def _rsub_m(out, a, b, **kw):  # b - a
    return (a, b), lambda g: (_unb(-g, a), _unb(g, b))


@register(torch.rsub)
def _rsub(out, a, b, alpha=1, **kw):  # b - alpha * a
    return (a, b), lambda g: (_unb(-g * alpha, a), _unb(g, b))


@register(torch.mul, T.mul, T.__mul__, T.__rmul__, torch.multiply, T.multiply)
def _mul(out, a, b, **kw):
    return (a, b), lambda g: (_unb(g * b, a) if _is_t(a) else None, _unb(g * a, b) if _is_t(b) else None)


@register(torch.div, T.div, T.__truediv__, torch.true_divide, T.true_divide, torch.divide, T.divide)
def _div(out, a, b, rounding_mode=None, **kw):
    if rounding_mode is not None:
        return (a, b), lambda g: (None, None)
    return (a, b), lambda g: (_unb(g / b, a) if _is_t(a) else None,
                              _unb(-g * out / b, b) if _is_t(b) else None)


@register(T.__rtruediv__)
def _rdiv(out, a, b, **kw):  # b / a
    return (a, b), lambda g: (_unb(-g * out / a, a), _unb(g / a, b) if _is_t(b) else None)


@register(torch.pow, T.pow, T.__pow__)
def _pow(out, a, e, **kw):
    def bwd(g):
        ga = gb = None
        if _is_t(a):
            ga = _unb(g * e * torch.pow(a, e - 1), a) if not _is_t(e) else _unb(g * e * torch.pow(a, e - 1), a)
        if _is_t(e):
            base = a if _is_t(a) else torch.tensor(a, dtype=out.dtype, device=out.device)
            gb = _unb(g * out * torch.log(base), e)
        return ga, gb

    return (a, e), bwd


@register(T.__rpow__)
def _rpow(out, e, a, **kw):  # a ** e
    return (e, a), lambda g: (_unb(g * out * math.log(a) if not _is_t(a) else g * out * torch.log(a), e), None)


@register(torch.maximum, T.maximum, torch.fmax)
def _maximum(out, a, b, **kw):
    def bwd(g):
        m = (a >= b)
        return _unb(torch.where(m, g, 0.0), a), _unb(torch.where(m, 0.0, g), b)

    return (a, b), bwd


@register(torch.minimum, T.minimum, torch.fmin)
def _minimum(out, a, b, **kw):
    def bwd(g):
        m = (a <= b)
        return _unb(torch.where(m, g, 0.0), a), _unb(torch.where(m, 0.0, g), b)

    return (a, b), bwd


@register(torch.where, T.where)
def _where(out, cond, x=None, y=None, **kw):
    if x is None:
        return (), lambda g: ()
    return (cond, x, y), lambda g: (None, _unb(torch.where(cond, g, 0.0), x), _unb(torch.where(cond, 0.0, g), y))


@register(torch.neg, T.neg, T.__neg__, torch.negative)
def _neg(out, a, **kw):
    return (a,), lambda g: (-g,)


@register(torch.exp, T.exp)
def _exp(out, a, **kw):
    return (a,), lambda g: (g * out,)


@register(torch.expm1, T.expm1)
def _expm1(out, a, **kw):
    return (a,), lambda g: (g * (out + 1),)


@register(torch.log, T.log)
def _log(out, a, **kw):
    return (a,), lambda g: (g / a,)


@register(torch.log2, T.log2)
def _log2(out, a, **kw):
    return (a,), lambda g: (g / (a * math.log(2.0)),)


@register(torch.log10, T.log10)
def _log10(out, a, **kw):
    return (a,), lambda g: (g / (a * math.log(10.0)),)


@register(torch.log1p, T.log1p)
def _log1p(out, a, **kw):
    return (a,), lambda g: (g / (1 + a),)


@register(torch.sqrt, T.sqrt)
def _sqrt(out, a, **kw):
    return (a,), lambda g: (g * 0.5 / out,)


@register(torch.rsqrt, T.rsqrt)
def _rsqrt(out, a, **kw):
    return (a,), lambda g: (g * -0.5 * out / a,)


@register(torch.square, T.square)
def _square(out, a, **kw):
    return (a,), lambda g: (g * 2 * a,)


@register(torch.reciprocal, T.reciprocal)
def _recip(out, a, **kw):
    return (a,), lambda g: (-g * out * out,)


@register(torch.abs, T.abs, T.__abs__, torch.absolute)
def _abs(out, a, **kw):
    return (a,), lambda g: (g * torch.sign(a),)


@register(torch.sin, T.sin)
def _sin(out, a, **kw):
    return (a,), lambda g: (g * torch.cos(a),)


@register(torch.cos, T.cos)
def _cos(out, a, **kw):
    return (a,), lambda g: (-g * torch.sin(a),)


@register(torch.tan, T.tan)
def _tan(out, a, **kw):
    return (a,), lambda g: (g * (1 + out * out),)


@register(torch.erf, T.erf)
def _erf(out, a, **kw):
    return (a,), lambda g: (g * (2.0 / math.sqrt(math.pi)) * torch.exp(-a * a),)


@register(torch.atan, T.atan)
def _atan(out, a, **kw):
    return (a,), lambda g: (g / (1 + a * a),)


@register(torch.tanh, T.tanh, F.tanh)
def _tanh(out, a, **kw):
    return (a,), lambda g: (g * (1 - out * out),)


@register(torch.sigmoid, T.sigmoid, F.sigmoid)
def _sigmoid(out, a, **kw):
    return (a,), lambda g: (g * out * (1 - out),)


@register(torch.relu, T.relu, F.relu)
def _relu(out, a, inplace=False, **kw):
    return (a,), lambda g: (g * (out > 0).to(g.dtype),)


@register(F.relu6)
def _relu6(out, a, inplace=False, **kw):
    return (a,), lambda g: (g * ((a > 0) & (a < 6)).to(g.dtype),)


@register(F.leaky_relu)
def _leaky(out, a, negative_slope=0.01, inplace=False, **kw):
    return (a,), lambda g: (torch.where(a > 0, g, g * negative_slope),)


@register(F.elu)
def _elu(out, a, alpha=1.0, inplace=False, **kw):
    return (a,), lambda g: (torch.where(a > 0, g, g * (out + alpha)),)


@register(F.selu)
def _selu(out, a, inplace=False, **kw):
    sc, al = 1.0507009873554804934193349852946, 1.6732632423543772848170429916717
    return (a,), lambda g: (torch.where(a > 0, g * sc, g * (out + sc * al)),)


@register(F.celu)
def _celu(out, a, alpha=1.0, inplace=False, **kw):
    return (a,), lambda g: (torch.where(a > 0, g, g * torch.exp(a / alpha)),)


@register(F.gelu)
def _gelu(out, a, approximate="none", **kw):
    def bwd(g):
        if approximate == "tanh":
            k = math.sqrt(2.0 / math.pi)
            u = k * (a + 0.044715 * a * a * a)
            t = torch.tanh(u)
            return (g * (0.5 * (1 + t) + 0.5 * a * (1 - t * t) * k * (1 + 3 * 0.044715 * a * a)),)
        cdf = 0.5 * (1 + torch.erf(a / math.sqrt(2.0)))
        pdf = torch.exp(-0.5 * a * a) / math.sqrt(2 * math.pi)
        return (g * (cdf + a * pdf),)

    return (a,), bwd


@register(F.silu)
def _silu(out, a, inplace=False, **kw):
    def bwd(g):
        s = torch.sigmoid(a)
        return (g * s * (1 + a * (1 - s)),)

    return (a,), bwd


@register(F.mish)
def _mish(out, a, inplace=False, **kw):
    def bwd(g):
        sp = F.softplus(a)
        t = torch.tanh(sp)
        return (g * (t + a * (1 - t * t) * torch.sigmoid(a)),)

    return (a,), bwd


@register(F.softplus)
def _softplus(out, a, beta=1, threshold=20, **kw):
    return (a,), lambda g: (torch.where(a * beta > threshold, g, g * torch.sigmoid(a * beta)),)


@register(F.hardswish)
def _hardswish(out, a, inplace=False, **kw):
    return (a,), lambda g: (torch.where(a < -3, 0.0 * g, torch.where(a > 3, g, g * (2 * a + 3) / 6)),)


@register(F.hardsigmoid)
def _hardsigmoid(out, a, inplace=False, **kw):
    return (a,), lambda g: (g * ((a > -3) & (a < 3)).to(g.dtype) / 6,)


@register(F.hardtanh)
def _hardtanh(out, a, min_val=-1.0, max_val=1.0, inplace=False, **kw):
    return (a,), lambda g: (g * ((a > min_val) & (a < max_val)).to(g.dtype),)


@register(F.softsign)
def _softsign(out, a, **kw):
    return (a,), lambda g: (g / (1 + a.abs()) ** 2,)


@register(F.logsigmoid)
def _logsigmoid(out, a, **kw):
    return (a,), lambda g: (g * torch.sigmoid(-a),)


@register(F.tanhshrink)
def _tanhshrink(out, a, **kw):
    return (a,), lambda g: (g * torch.tanh(a) ** 2,)


@register(F.hardshrink)
def _hardshrink(out, a, lambd=0.5, **kw):
    return (a,), lambda g: (g * (a.abs() > lambd).to(g.dtype),)


@register(F.softshrink)
def _softshrink(out, a, lambd=0.5, **kw):
    return (a,), lambda g: (g * (a.abs() > lambd).to(g.dtype),)


@register(F.prelu)
def _prelu(out, a, w, **kw):
    def bwd(g):
        wb = w.reshape([1, -1] + [1] * (a.dim() - 2)) if a.dim() > 1 and w.numel() > 1 else w
        ga = torch.where(a > 0, g, g * wb)
        gw = _unb(torch.where(a > 0, 0.0 * g, g * a), wb).reshape(w.shape)
        return ga, gw

    return (a, w), bwd


@register(torch.clamp, T.clamp, torch.clip, T.clip)
def _clamp(out, a, min=None, max=None, **kw):
    def bwd(g):
        m = torch.ones_like(a, dtype=torch.bool)
        if min is not None:
            m = m & (a >= min)
        if max is not None:
            m = m & (a <= max)
        return (g * m.to(g.dtype), None if not _is_t(min) else None, None)

    return (a, min, max), bwd


# =========================================================================== matmul
def _mm_bwd(a, b, g):
    # autocast runs the product in a lower precision than the operands: differentiate
    # in the operands' dtype
    if g.dtype != a.dtype and a.dtype == b.dtype:
        g = g.to(a.dtype)
    a2 = a.unsqueeze(0) if a.dim() == 1 else a
    b2 = b.unsqueeze(-1) if b.dim() == 1 else b
    g2 = g
    if a.dim() == 1:
        g2 = g2.unsqueeze(-2)
    if b.dim() == 1:
        g2 = g2.unsqueeze(-1)
    ga = g2 @ b2.transpose(-1, -2)
    gb = a2.transpose(-1, -2) @ g2
    if a.dim() == 1:
        ga = ga.squeeze(-2)
    if b.dim() == 1:
        gb = gb.squeeze(-1)
    return _unb(ga, a), _unb(gb, b)


@register(torch.matmul, T.matmul, T.__matmul__, torch.mm, T.mm, torch.bmm, T.bmm)
def _matmul(out, a, b, **kw):
    return (a, b), lambda g: _mm_bwd(a, b, g)


@register(T.__rmatmul__)
def _rmatmul(out, a, b, **kw):  # b @ a
    return (a, b), lambda g: tuple(reversed(_mm_bwd(b, a, g)))


@register(torch.addmm, T.addmm)
def _addmm(out, inp, m1, m2, beta=1, alpha=1, **kw):
    def bwd(g):
        ga, gb = _mm_bwd(m1, m2, g * alpha if alpha != 1 else g)
        return _unb(g * beta if beta != 1 else g, inp), ga, gb

    return (inp, m1, m2), bwd


@register(F.linear)
def _linear(out, x, w, b=None, **kw):
    def bwd(g):
        if g.dtype != x.dtype and x.dtype == w.dtype:
            g = g.to(x.dtype)
        gx = g @ w
        gw = (g.reshape(-1, g.shape[-1]).t() @ x.reshape(-1, x.shape[-1])).to(w.dtype)
        gb = g.reshape(-1, g.shape[-1]).sum(0).to(b.dtype) if _is_t(b) else None
        return gx, gw, gb

    return (x, w, b), bwd


@register(F.bilinear)
def _bilinear(out, x1, x2, w, b=None, **kw):
    def bwd(g):
        gx1 = torch.einsum("bo,oij,bj->bi", g, w, x2)
        gx2 = torch.einsum("bo,oij,bi->bj", g, w, x1)
        gw = torch.einsum("bo,bi,bj->oij", g, x1, x2)
        return gx1, gx2, gw, (g.sum(0) if _is_t(b) else None)

    return (x1, x2, w, b), bwd


# =========================================================================== reductions
def _norm_dims(dim, nd):
    if dim is None:
        return tuple(range(nd))
    if isinstance(dim, int):
        dim = (dim,)
    return tuple(d % nd if nd else 0 for d in dim)


def _expand_back(g, a, dims, keepdim):
    if not keepdim and a.dim():
        for d in sorted(dims):
            g = g.unsqueeze(d)
    return g.expand(a.shape)


@register(torch.sum, T.sum)
def _sum(out, a, dim=None, keepdim=False, dtype=None, **kw):
    dims = _norm_dims(dim, a.dim())
    return (a,), lambda g: (_expand_back(g, a, dims, keepdim).to(a.dtype),)


@register(torch.mean, T.mean)
def _mean(out, a, dim=None, keepdim=False, dtype=None, **kw):
    dims = _norm_dims(dim, a.dim())
    n = 1
    for d in dims:
        n *= a.shape[d] if a.dim() else 1
    return (a,), lambda g: ((_expand_back(g, a, dims, keepdim) / max(n, 1)).to(a.dtype),)


def _minmax_rule(out, a, dim=None, keepdim=False, **kw):
    if dim is None and not isinstance(out, (tuple, list)):
        def bwd(g):
            m = (a == out).to(g.dtype)
            return (m * (g / m.sum()),)

        return (a,), bwd
    if not isinstance(out, (tuple, list)) or isinstance(dim, torch.Tensor):
        # torch.max(a, b): elementwise
        b = dim

        def bwd2(g):
            m = (a == out)
            return _unb(torch.where(m, g, 0.0), a), _unb(torch.where(m, 0.0, g), b)

        return (a, b), bwd2
    idx = out[1]

    def bwd3(g, gi=None):
        gg = g if keepdim else g.unsqueeze(dim)
        ii = idx if keepdim else idx.unsqueeze(dim)
        return (torch.zeros_like(a).scatter(dim, ii, gg),)

    return (a,), bwd3


register(torch.max, T.max, torch.min, T.min)(_minmax_rule)


@register(torch.amax, T.amax, torch.amin, T.amin)
def _amax(out, a, dim=(), keepdim=False, **kw):
    dims = _norm_dims(dim if dim != () else None, a.dim())

    def bwd(g):
        o = _expand_back(out, a, dims, keepdim)
        m = (a == o).to(g.dtype)
        cnt = m.sum(dim=dims, keepdim=True)
        return (m * _expand_back(g, a, dims, keepdim) / cnt,)

    return (a,), bwd


@register(torch.logsumexp, T.logsumexp)
def _lse(out, a, dim, keepdim=False, **kw):
    dims = _norm_dims(dim, a.dim())
    return (a,), lambda g: (_expand_back(g, a, dims, keepdim) * torch.exp(a - _expand_back(out, a, dims, keepdim)),)


@register(torch.var, T.var, torch.std, T.std)
def _var(out, a, dim=None, unbiased=None, keepdim=False, correction=None, **kw):
    if isinstance(dim, bool):  # var(unbiased)
        unbiased, dim = dim, None
    dims = _norm_dims(dim, a.dim())
    n = 1
    for d in dims:
        n *= a.shape[d]
    corr = correction if correction is not None else (0 if unbiased is False else 1)
    is_std = out is not None and kw.get("_std", False)

    def bwd(g):
        mu = a.mean(dim=dims, keepdim=True)
        gv = _expand_back(g, a, dims, keepdim) * 2 * (a - mu) / max(n - corr, 1)
        return (gv,)

    return (a,), bwd


@register(torch.std, T.std)
def _std(out, a, dim=None, unbiased=None, keepdim=False, correction=None, **kw):
    if isinstance(dim, bool):
        unbiased, dim = dim, None
    dims = _norm_dims(dim, a.dim())
    n = 1
    for d in dims:
        n *= a.shape[d]
    corr = correction if correction is not None else (0 if unbiased is False else 1)

    def bwd(g):
        mu = a.mean(dim=dims, keepdim=True)
        so = _expand_back(out, a, dims, keepdim)
        return (_expand_back(g, a, dims, keepdim) * (a - mu) / (max(n - corr, 1) * so),)

    return (a,), bwd


@register(torch.norm, T.norm, torch.linalg.vector_norm)
def _norm(out, a, p="fro", dim=None, keepdim=False, **kw):
    if "ord" in kw:
        p = kw["ord"]
    dims = _norm_dims(dim, a.dim())

    def bwd(g):
        o = _expand_back(out, a, dims, keepdim)
        ge = _expand_back(g, a, dims, keepdim)
        if p in ("fro", 2, 2.0, None):
            return (ge * a / o.clamp_min(1e-30),)
        if p in (1, 1.0):
            return (ge * torch.sign(a),)
        pp = float(p)
        return (ge * torch.sign(a) * a.abs() ** (pp - 1) / o.clamp_min(1e-30) ** (pp - 1),)

    return (a,), bwd


@register(torch.cumsum, T.cumsum)
def _cumsum(out, a, dim, **kw):
    return (a,), lambda g: (g.flip(dim).cumsum(dim).flip(dim),)


# =========================================================================== shape / views
def _reshape_rule(out, a, *args, **kw):
    return (a,), lambda g: (g.reshape(a.shape),)


register(torch.reshape, T.reshape, T.view, T.view_as, T.reshape_as, torch.flatten, T.flatten, T.unflatten,
         torch.squeeze, T.squeeze, torch.unsqueeze, T.unsqueeze, torch.ravel, T.ravel)(_reshape_rule)


@register(torch.permute, T.permute)
def _permute(out, a, *dims, **kw):
    if len(dims) == 1 and isinstance(dims[0], (list, tuple)):
        dims = dims[0]
    if not dims:
        dims = kw.get("dims")
    inv = [0] * len(dims)
    for i, d in enumerate(dims):
        inv[d % len(dims)] = i
    return (a,), lambda g: (g.permute(inv),)


@register(torch.transpose, T.transpose, torch.swapaxes, T.swapaxes)
def _transpose(out, a, d0, d1, **kw):
    return (a,), lambda g: (g.transpose(d0, d1),)


@register(torch.t, T.t)
def _t(out, a, **kw):
    return (a,), lambda g: (g.t() if g.dim() == 2 else g,)


@register(torch.movedim, T.movedim)
def _movedim(out, a, src, dst, **kw):
    return (a,), lambda g: (torch.movedim(g, dst, src),)


@register(T.expand, T.expand_as, torch.broadcast_to, T.broadcast_to)
def _expand(out, a, *args, **kw):
    return (a,), lambda g: (_unb(g, a),)


@register(T.repeat, torch.tile, T.tile)
def _repeat(out, a, *reps, **kw):
    if len(reps) == 1 and isinstance(reps[0], (list, tuple)):
        reps = tuple(reps[0])
    if not reps:
        reps = tuple(kw.get("dims") or kw.get("repeats"))

    def bwd(g):
        r = list(reps)
        shape = list(a.shape)
        if len(r) < len(shape):
            r = [1] * (len(shape) - len(r)) + r
        lead = len(r) - len(shape)
        shape = [1] * lead + shape
        gv = g.reshape([x for pair in zip(r, shape) for x in pair])
        gs = gv.sum(dim=tuple(range(0, 2 * len(r), 2)))
        return (gs.reshape(a.shape),)

    return (a,), bwd


@register(torch.repeat_interleave, T.repeat_interleave)
def _rep_il(out, a, repeats, dim=None, **kw):
    if _is_t(repeats) or dim is None:
        return (), lambda g: ()

    def bwd(g):
        s = list(a.shape)
        s.insert(dim + 1, repeats)
        return (g.reshape(s).sum(dim + 1),)

    return (a,), bwd


def _is_basic_index(idx):
    items = idx if isinstance(idx, tuple) else (idx,)
    return all(i is None or i is Ellipsis or isinstance(i, (int, slice)) for i in items)


@register(T.__getitem__)
def _getitem(out, a, idx, **kw):
    if _is_basic_index(idx):
        def bwd(g):
            z = torch.zeros_like(a, dtype=g.dtype)
            z[idx] = g
            return (z, None)

        return (a, idx), bwd

    def bwd_adv(g):
        # any advanced / mixed index: the flat positions the index selects, then one
        # index_add (duplicates accumulate)
        pos = torch.arange(a.numel(), device=a.device).reshape(a.shape)[idx]
        z = torch.zeros(a.numel(), dtype=g.dtype, device=g.device)
        z.index_add_(0, pos.reshape(-1), g.reshape(-1))
        return (z.reshape(a.shape), None)

    return (a, idx), bwd_adv


def setitem_outofplace(x, idx, v):
    """``x[idx] = v`` as a recorded out-of-place op (engine._dispatch_inplace)."""
    from .engine import _record

    res = x.clone()
    res[idx] = v
    res = _wrap(res)

    def bwd(g):
        gx = g.clone()
        gx[idx] = 0
        gv = _unb(g[idx], v) if _is_t(v) else None
        return gx, None, gv

    _record("setitem", bwd, (x, idx, v), [res])
    return res


@register(torch.cat, torch.concat, torch.concatenate)
def _cat(out, tensors, dim=0, **kw):
    sizes = [t.shape[dim] if t.dim() else 0 for t in tensors]

    def bwd(g):
        parts = torch.split(g, sizes, dim=dim)
        return tuple(p for p in parts)

    return tuple(tensors), bwd


@register(torch.stack)
def _stack(out, tensors, dim=0, **kw):
    return tuple(tensors), lambda g: tuple(torch.unbind(g, dim=dim))


def _multi_out_rule(dim_of):
    def rule(out, a, *args, **kw):
        dim = dim_of(args, kw)

        def bwd(*gs):
            parts = [g if g is not None else torch.zeros(o.shape, dtype=o.dtype, device=o.device)
                     for g, o in zip(gs, out)]
            return (torch.cat(parts, dim=dim),)

        return (a,), bwd

    return rule


register(torch.split, T.split, torch.chunk, T.chunk, torch.tensor_split, T.tensor_split)(
    _multi_out_rule(lambda args, kw: kw.get("dim", args[1] if len(args) > 1 else 0)))


@register(torch.unbind, T.unbind)
def _unbind(out, a, dim=0, **kw):
    def bwd(*gs):
        parts = [g if g is not None else torch.zeros(o.shape, dtype=o.dtype, device=o.device) for g, o in zip(gs, out)]
        return (torch.stack(parts, dim=dim),)

    return (a,), bwd


@register(torch.narrow, T.narrow)
def _narrow(out, a, dim, start, length, **kw):
    def bwd(g):
        z = torch.zeros_like(a, dtype=g.dtype)
        z.narrow(dim, start, length).copy_(g)
        return (z,)

    return (a,), bwd


@register(torch.select, T.select)
def _select(out, a, dim, index, **kw):
    def bwd(g):
        z = torch.zeros_like(a, dtype=g.dtype)
        z.select(dim, index).copy_(g)
        return (z,)

    return (a,), bwd


@register(torch.index_select, T.index_select)
def _index_select(out, a, dim, index, **kw):
    return (a,), lambda g: (torch.zeros_like(a, dtype=g.dtype).index_add_(dim, index, g),)


@register(torch.gather, T.gather)
def _gather(out, a, dim, index, **kw):
    return (a,), lambda g: (torch.zeros_like(a, dtype=g.dtype).scatter_add_(dim, index, g),)


@register(torch.take_along_dim, T.take_along_dim)
def _take_along(out, a, index, dim=None, **kw):
    if dim is None:
        return (a,), lambda g: (torch.zeros(a.numel(), dtype=g.dtype, device=g.device)
                                .scatter_add_(0, index.reshape(-1), g.reshape(-1)).reshape(a.shape),)
    return (a,), lambda g: (torch.zeros_like(a, dtype=g.dtype).scatter_add_(dim, index.expand_as(g), g),)


@register(torch.scatter, T.scatter)
def _scatter(out, a, dim, index, src=None, **kw):
    if "value" in kw or not _is_t(src):
        return (a,), lambda g: (g.scatter(dim, index, 0.0),)
    return (a, src), lambda g: (g.scatter(dim, index, 0.0), g.gather(dim, index))


@register(torch.masked_fill, T.masked_fill)
def _masked_fill(out, a, mask, value, **kw):
    return (a,), lambda g: (torch.where(mask, 0.0, g).to(g.dtype),)


@register(torch.flip, T.flip)
def _flip(out, a, dims, **kw):
    return (a,), lambda g: (g.flip(dims),)


@register(torch.roll, T.roll)
def _roll(out, a, shifts, dims=None, **kw):
    neg = tuple(-s for s in shifts) if isinstance(shifts, (list, tuple)) else -shifts
    return (a,), lambda g: (torch.roll(g, neg, dims),)


@register(torch.tril, T.tril)
def _tril(out, a, diagonal=0, **kw):
    return (a,), lambda g: (torch.tril(g, diagonal),)


@register(torch.triu, T.triu)
def _triu(out, a, diagonal=0, **kw):
    return (a,), lambda g: (torch.triu(g, diagonal),)


@register(F.pad)
def _pad(out, a, pad, mode="constant", value=None, **kw):
    if mode != "constant":
        return None

    def bwd(g):
        sl = [slice(None)] * a.dim()
        for i in range(len(pad) // 2):
            d = a.dim() - 1 - i
            lo, hi = pad[2 * i], pad[2 * i + 1]
            sl[d] = slice(lo, g.shape[d] - hi if hi else None) if lo >= 0 and hi >= 0 else slice(None)
        return (g[tuple(sl)],)

    return (a,), bwd


def _cast_rule(out, a, *args, **kw):
    return (a,), lambda g: (g.to(device=a.device, dtype=a.dtype),)


register(T.to, T.type, T.float, T.double, T.half, T.bfloat16, T.cuda, T.cpu, T.contiguous, torch.clone, T.clone,
         T.type_as, T.requires_grad_)(_cast_rule)


@register(T.copy_)
def _copy(out, dst, src, non_blocking=False, **kw):
    return (dst, src), lambda g: (None, _unb(g.to(src.dtype), src))


# =========================================================================== nn
@register(torch.softmax, T.softmax, F.softmax, torch.nn.functional.softmax)
def _softmax(out, a, dim=None, *args, **kw):
    dim = kw.get("dim", dim)
    if dim is None:
        dim = -1

    def bwd(g):
        o = out.to(g.dtype)
        return (o * (g - (g * o).sum(dim, keepdim=True)),)

    return (a,), bwd


@register(torch.log_softmax, T.log_softmax, F.log_softmax)
def _log_softmax(out, a, dim=None, *args, **kw):
    dim = kw.get("dim", dim)
    if dim is None:
        dim = -1
    return (a,), lambda g: (g - torch.exp(out) * g.sum(dim, keepdim=True),)


@fwd_rule(F.dropout, torch.dropout)
def _dropout(a, p=0.5, training=True, inplace=False, **kw):
    if "train" in kw:
        training = kw["train"]
    if not training or p == 0.0:
        return a.clone() if not inplace else a, (a,), lambda g: (g,)
    if p >= 1.0:
        return torch.zeros_like(a), (a,), lambda g: (torch.zeros_like(g),)
    mask = (torch.rand_like(a, dtype=torch.float32) >= p).to(a.dtype) / (1.0 - p)
    return a * mask, (a,), lambda g: (g * mask,)


@register(F.embedding)
def _embedding(out, ids, w, padding_idx=None, *args, **kw):
    def bwd(g):
        gw = torch.zeros_like(w, dtype=g.dtype)
        gw.index_add_(0, ids.reshape(-1), g.reshape(-1, w.shape[1]))
        if padding_idx is not None and padding_idx >= 0:
            gw[padding_idx] = 0
        return None, gw.to(w.dtype)

    return (ids, w), bwd


def _conv_bwd(nd, transposed):
    def rule(out, x, w, b=None, stride=1, padding=0, *rest, **kw):
        if transposed:
            output_padding = rest[0] if len(rest) > 0 else kw.get("output_padding", 0)
            groups = rest[1] if len(rest) > 1 else kw.get("groups", 1)
            dilation = rest[2] if len(rest) > 2 else kw.get("dilation", 1)
        else:
            dilation = rest[0] if len(rest) > 0 else kw.get("dilation", 1)
            groups = rest[1] if len(rest) > 1 else kw.get("groups", 1)
            output_padding = 0
        if isinstance(padding, str):
            return None
        tup = lambda v: [v] * nd if isinstance(v, int) else list(v)  # noqa: E731

        def bwd(g):
            gx, gw, gb = ATEN.convolution_backward(g, x, w, [w.shape[0 if not transposed else 1] * (groups if transposed else 1)] if _is_t(b) else None,
                                                   tup(stride), tup(padding), tup(dilation), transposed,
                                                   tup(output_padding), groups, [True, True, _is_t(b)])
            return gx, gw, gb

        return (x, w, b), bwd

    return rule


register(F.conv1d, torch.conv1d)(_conv_bwd(1, False))
register(F.conv2d, torch.conv2d)(_conv_bwd(2, False))
register(F.conv3d, torch.conv3d)(_conv_bwd(3, False))
register(F.conv_transpose1d, torch.conv_transpose1d)(_conv_bwd(1, True))
register(F.conv_transpose2d, torch.conv_transpose2d)(_conv_bwd(2, True))
register(F.conv_transpose3d, torch.conv_transpose3d)(_conv_bwd(3, True))


def _tuple(v, n):
    return [v] * n if isinstance(v, int) else list(v)


@fwd_rule(F.max_pool2d)
def _maxpool2d(x, kernel_size, stride=None, padding=0, dilation=1, ceil_mode=False, return_indices=False, **kw):
    k = _tuple(kernel_size, 2)
    s = _tuple(stride if stride not in (None, []) else kernel_size, 2)
    p, d = _tuple(padding, 2), _tuple(dilation, 2)
    out, idx = ATEN.max_pool2d_with_indices(x, k, s, p, d, ceil_mode)

    def bwd(g, gi=None):
        return (ATEN.max_pool2d_with_indices_backward(g, x, k, s, p, d, ceil_mode, idx),)

    return ((out, idx) if return_indices else out), (x,), bwd


@fwd_rule(F.max_pool1d)
def _maxpool1d(x, kernel_size, stride=None, padding=0, dilation=1, ceil_mode=False, return_indices=False, **kw):
    out = _maxpool2d(x.unsqueeze(-2), (1, kernel_size if isinstance(kernel_size, int) else kernel_size[0]),
                     (1, (stride if stride not in (None, []) else kernel_size) if isinstance(
                         stride if stride is not None else kernel_size, int) else stride[0]),
                     (0, padding if isinstance(padding, int) else padding[0]),
                     (1, dilation if isinstance(dilation, int) else dilation[0]), ceil_mode, True)
    (o, idx), _, b2 = out
    return ((o.squeeze(-2), idx.squeeze(-2)) if return_indices else o.squeeze(-2)), (x,), \
        lambda g, gi=None: (b2(g.unsqueeze(-2))[0].squeeze(-2),)


@register(F.avg_pool2d)
def _avgpool2d(out, x, kernel_size, stride=None, padding=0, ceil_mode=False, count_include_pad=True,
               divisor_override=None, **kw):
    k = _tuple(kernel_size, 2)
    s = _tuple(stride if stride not in (None, []) else kernel_size, 2)
    p = _tuple(padding, 2)
    return (x,), lambda g: (ATEN.avg_pool2d_backward(g, x, k, s, p, ceil_mode, count_include_pad, divisor_override),)


@register(F.avg_pool1d)
def _avgpool1d(out, x, kernel_size, stride=None, padding=0, ceil_mode=False, count_include_pad=True, **kw):
    k = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
    s = k if stride in (None, []) else (stride if isinstance(stride, int) else stride[0])
    p = padding if isinstance(padding, int) else padding[0]
    return (x,), lambda g: (ATEN.avg_pool2d_backward(g.unsqueeze(-2), x.unsqueeze(-2), [1, k], [1, s], [0, p],
                                                     ceil_mode, count_include_pad, None).squeeze(-2),)


@register(F.adaptive_avg_pool2d)
def _aap2d(out, x, output_size, **kw):
    return (x,), lambda g: (ATEN._adaptive_avg_pool2d_backward(g, x),)


@register(F.adaptive_avg_pool1d)
def _aap1d(out, x, output_size, **kw):
    return (x,), lambda g: (ATEN._adaptive_avg_pool2d_backward(g.unsqueeze(-2), x.unsqueeze(-2)).squeeze(-2),)


@fwd_rule(F.batch_norm)
def _batch_norm(x, running_mean, running_var, weight=None, bias=None, training=False, momentum=0.1, eps=1e-5,
                **kw):
    out, smean, sinv = ATEN.native_batch_norm(x, weight, bias, running_mean, running_var, training, momentum, eps)

    def bwd(g):
        gx, gw, gb = ATEN.native_batch_norm_backward(g, x, weight, running_mean, running_var, smean, sinv, training,
                                                     eps, [True, _is_t(weight), _is_t(bias)])
        return gx, None, None, gw, gb

    return out, (x, running_mean, running_var, weight, bias), bwd


@fwd_rule(F.layer_norm)
def _layer_norm(x, normalized_shape, weight=None, bias=None, eps=1e-5, **kw):
    ns = [normalized_shape] if isinstance(normalized_shape, int) else list(normalized_shape)
    out, mean, rstd = ATEN.native_layer_norm(x, ns, weight, bias, eps)

    def bwd(g):
        gx, gw, gb = ATEN.native_layer_norm_backward(g, x, ns, mean, rstd, weight, bias,
                                                     [True, _is_t(weight), _is_t(bias)])
        return gx, None, gw, gb

    return out, (x, ns, weight, bias), bwd


@fwd_rule(F.group_norm)
def _group_norm(x, num_groups, weight=None, bias=None, eps=1e-5, **kw):
    N, C = x.shape[0], x.shape[1]
    HxW = x.numel() // max(N * C, 1)
    out, mean, rstd = ATEN.native_group_norm(x, weight, bias, N, C, HxW, num_groups, eps)

    def bwd(g):
        gx, gw, gb = ATEN.native_group_norm_backward(g, x, mean, rstd, weight, N, C, HxW, num_groups,
                                                     [True, _is_t(weight), _is_t(bias)])
        return gx, None, gw, gb

    return out, (x, num_groups, weight, bias), bwd


# ---------------------------------------------------------------- losses
def _reduce_back(g, shape, reduction, n, dtype, device):
    if reduction == "mean":
        return (g / n).expand(shape) if g.dim() == 0 else g
    if reduction == "sum":
        return g.expand(shape)
    return g


@register(F.cross_entropy)
def _cross_entropy(out, inp, target, weight=None, size_average=None, ignore_index=-100, reduce=None,
                   reduction="mean", label_smoothing=0.0, **kw):
    if target.is_floating_point() or label_smoothing:
        return None  # soft labels / smoothing: fallback rule
    C = inp.shape[1] if inp.dim() > 1 else inp.shape[0]

    def bwd(g):
        x = inp.movedim(1, -1).reshape(-1, C) if inp.dim() > 2 else inp.reshape(-1, C)
        t = target.reshape(-1)
        ct = torch.float64 if x.dtype == torch.float64 else torch.float32
        p = torch.softmax(x.to(ct), dim=-1)
        valid = (t != ignore_index)
        tc = torch.where(valid, t, 0)
        w = weight[tc].to(ct) if _is_t(weight) else torch.ones_like(t, dtype=ct)
        w = w * valid.to(ct)
        oh = torch.zeros_like(p).scatter_(1, tc.unsqueeze(1), 1.0)
        gr = (p - oh) * w.unsqueeze(1)
        if reduction == "mean":
            gr = gr * (g.to(ct) / w.sum().clamp_min(1e-12))
        elif reduction == "sum":
            gr = gr * g.to(ct)
        else:
            gr = gr * g.reshape(-1, 1).to(ct)
        gr = gr.to(inp.dtype)
        if inp.dim() > 2:
            shp = list(inp.shape)
            gr = gr.reshape([shp[0]] + shp[2:] + [C]).movedim(-1, 1)
        return gr.reshape(inp.shape), None, None

    return (inp, target, weight), bwd


@register(F.nll_loss)
def _nll(out, inp, target, weight=None, size_average=None, ignore_index=-100, reduce=None, reduction="mean", **kw):
    C = inp.shape[1] if inp.dim() > 1 else inp.shape[0]

    def bwd(g):
        x = inp.movedim(1, -1).reshape(-1, C) if inp.dim() > 2 else inp.reshape(-1, C)
        t = target.reshape(-1)
        valid = (t != ignore_index)
        tc = torch.where(valid, t, 0)
        w = weight[tc].float() if _is_t(weight) else torch.ones_like(t, dtype=torch.float32)
        w = w * valid.float()
        gr = torch.zeros_like(x, dtype=torch.float32).scatter_(1, tc.unsqueeze(1), -w.unsqueeze(1))
        if reduction == "mean":
            gr = gr * (g.float() / w.sum().clamp_min(1e-12))
        elif reduction == "sum":
            gr = gr * g.float()
        else:
            gr = gr * g.reshape(-1, 1).float()
        gr = gr.to(inp.dtype)
        if inp.dim() > 2:
            shp = list(inp.shape)
            gr = gr.reshape([shp[0]] + shp[2:] + [C]).movedim(-1, 1)
        return gr.reshape(inp.shape), None, None

    return (inp, target, weight), bwd


def _pointwise_loss(dfn):
    def rule(out, a, b, size_average=None, reduce=None, reduction="mean", *args, **kw):
        def bwd(g):
            ga, gb = dfn(a, b, kw, *args)
            scale = g / a.numel() if reduction == "mean" else g
            return (_unb(ga * scale, a) if _is_t(a) else None, _unb(gb * scale, b) if _is_t(b) else None)

        return (a, b), bwd

    return rule


register(F.mse_loss)(_pointwise_loss(lambda a, b, kw: (2 * (a - b), -2 * (a - b))))
register(F.l1_loss)(_pointwise_loss(lambda a, b, kw: (torch.sign(a - b), -torch.sign(a - b))))


def _sl1(a, b, kw, beta=1.0):
    beta = kw.get("beta", beta)
    d = a - b
    gd = torch.where(d.abs() < beta, d / beta, torch.sign(d))
    return gd, -gd


register(F.smooth_l1_loss)(_pointwise_loss(_sl1))


def _huber(a, b, kw, delta=1.0):
    delta = kw.get("delta", delta)
    d = a - b
    gd = torch.where(d.abs() <= delta, d, delta * torch.sign(d))
    return gd, -gd


register(F.huber_loss)(_pointwise_loss(_huber))


@register(F.binary_cross_entropy)
def _bce(out, p, y, weight=None, size_average=None, reduce=None, reduction="mean", **kw):
    def bwd(g):
        eps = 1e-12
        gr = (p - y) / (p * (1 - p)).clamp_min(eps)
        if _is_t(weight):
            gr = gr * weight
        gr = gr * (g / p.numel() if reduction == "mean" else g)
        return gr, None, None

    return (p, y, weight), bwd


@register(F.binary_cross_entropy_with_logits)
def _bcel(out, x, y, weight=None, size_average=None, reduce=None, reduction="mean", pos_weight=None, **kw):
    def bwd(g):
        s = torch.sigmoid(x)
        if _is_t(pos_weight):
            gr = (pos_weight * y + 1 - y) * s - pos_weight * y
        else:
            gr = s - y
        if _is_t(weight):
            gr = gr * weight
        gr = gr * (g / x.numel() if reduction == "mean" else g)
        return gr, None, None, None

    return (x, y, weight, pos_weight), bwd


@register(F.kl_div)
def _kl(out, inp, target, size_average=None, reduce=None, reduction="mean", log_target=False, **kw):
    def bwd(g):
        gr = -torch.exp(target) if log_target else -target
        n = inp.numel() if reduction == "mean" else (inp.shape[0] if reduction == "batchmean" else 1)
        return gr * (g / n if reduction in ("mean", "batchmean") else g), None

    return (inp, target), bwd


@register(F.cosine_similarity)
def _cos_sim(out, a, b, dim=1, eps=1e-8, **kw):
    def bwd(g):
        na = a.norm(dim=dim, keepdim=True).clamp_min(eps)
        nb = b.norm(dim=dim, keepdim=True).clamp_min(eps)
        o = out.unsqueeze(dim)
        gg = g.unsqueeze(dim)
        ga = gg * (b / (na * nb) - o * a / (na * na))
        gb = gg * (a / (na * nb) - o * b / (nb * nb))
        return _unb(ga, a), _unb(gb, b)

    return (a, b), bwd


@register(F.normalize)
def _normalize(out, a, p=2.0, dim=1, eps=1e-12, **kw):
    def bwd(g):
        n = a.norm(p=p, dim=dim, keepdim=True)
        nc = n.clamp_min(eps)
        if p != 2.0:
            return None
        return (g / nc - out * (g * out).sum(dim, keepdim=True) / nc * (n > eps).to(g.dtype),)

    return (a,), bwd


# =========================================================================== non-differentiable
nondiff(T.detach, torch.detach, torch.zeros_like, torch.ones_like, torch.empty_like, torch.full_like,
        torch.rand_like, torch.randn_like, torch.randint_like, T.new_zeros, T.new_ones, T.new_empty, T.new_full,
        T.new_tensor, torch.sign, T.sign, torch.floor, T.floor, torch.ceil, T.ceil, torch.round, T.round,
        torch.trunc, T.trunc, torch.argmax, T.argmax, torch.argmin, T.argmin, torch.argsort, T.argsort,
        T.zero_, T.fill_, T.normal_, T.uniform_, T.bernoulli_, T.random_, T.exponential_,
        torch.bernoulli, torch.multinomial, T.__eq__, T.__ne__, T.__lt__, T.__le__, T.__gt__, T.__ge__,
        torch.isnan, torch.isinf, torch.isfinite, torch.nonzero, T.nonzero, torch.histc, torch.bucketize,
        T.__floordiv__, T.__rfloordiv__, T.__mod__, torch.remainder, torch.floor_divide,
        torch.full, torch.arange, torch.linspace)
passthrough(T.numpy, T.tolist, T.item, T.data_ptr, T.dim, T.size, T.numel, T.stride, T.element_size,
            T.is_contiguous, T.__len__, T.__bool__, T.__int__, T.__float__, T.__index__, T.__format__,
            T.storage_offset, T.untyped_storage, T.nelement, T.ndimension, T.get_device, T.is_floating_point,
            T.is_complex, T.__hash__, T.__reduce_ex__, T.__setstate__, T.__deepcopy__, T.register_hook,
            T.record_stream, T.share_memory_, T.is_shared, T.is_pinned, T.__array__,
            T.shape.__get__, T.dtype.__get__, T.device.__get__, T.is_cuda.__get__, T.ndim.__get__,
            T.requires_grad.__get__, T.is_leaf.__get__, T.data.__set__,
            T.grad.__get__, T.grad.__set__, T._version.__get__, T.layout.__get__, T.names.__get__,
            T.grad_fn.__get__, T.requires_grad.__set__)
nondiff(T.data.__get__)

# torch.Tensor.T / mT are views: grad is the transpose back
register(T.T.__get__, T.mT.__get__)(lambda out, a, *r, **k: ((a,), lambda g: (g.transpose(-1, -2) if g.dim() >= 2
                                                                                else g,)))
register(T.real.__get__)(lambda out, a, *r, **k: ((a,), lambda g: (g,)))

# in-place variants run out of place then copy into the target (engine._dispatch_inplace)
inplace({T.add_: T.add, T.__iadd__: T.__add__, T.sub_: T.sub, T.__isub__: T.__sub__, T.mul_: T.mul,
         T.__imul__: T.__mul__, T.div_: T.div, T.__itruediv__: T.__truediv__, T.clamp_: T.clamp, T.clip_: T.clip,
         T.relu_: T.relu, T.sigmoid_: T.sigmoid, T.tanh_: T.tanh, T.exp_: T.exp, T.pow_: T.pow,
         T.masked_fill_: T.masked_fill, T.neg_: T.neg, T.sqrt_: T.sqrt, T.abs_: T.abs, T.log_: T.log,
         T.scatter_: T.scatter, T.index_add_: T.index_add, T.unsqueeze_: T.unsqueeze, T.squeeze_: T.squeeze,
         T.t_: T.t, T.transpose_: T.transpose, torch.relu_: torch.relu, F.relu_: F.relu})


@register(torch.index_add, T.index_add)
def _index_add(out, a, dim, index, src, alpha=1, **kw):
    return (a, src), lambda g: (g, g.index_select(dim, index) * alpha)
