"""Python side of csrc/kernels/fluid_ops.hip: the Fluid operator-library rows
(activations + their grads, softmax_with_cross_entropy with the Softmax output,
cast, n-d strided gather = transpose / reverse / slice / expand / tile, Philox
uniform / gaussian random, the pointwise loss family, LoD sequence softmax).

Every function takes device tensors and returns device tensors (operands are made
contiguous and 16-byte aligned first); callers use them for CUDA places and keep
their torch formulas for CPUPlace.  Reference rows: see fluid_ops.hip's header.
"""
from __future__ import annotations

import ctypes

import torch

from ..framework import mixed_vector as _mv

from . import _native as N

ACTS = ["relu", "sigmoid", "logsigmoid", "exp", "tanh", "tanh_shrink", "softshrink", "sqrt", "rsqrt", "abs", "ceil",
        "floor", "cos", "sin", "round", "reciprocal", "log", "square", "softplus", "softsign", "brelu", "leaky_relu",
        "soft_relu", "elu", "relu6", "pow", "stanh", "hard_shrink", "thresholded_relu", "hard_sigmoid", "swish",
        "gelu", "silu"]
ACT_ID = {n: i for i, n in enumerate(ACTS)}
LOSSES = {"hinge_loss": 0, "huber_loss": 1, "smooth_l1": 2, "log_loss": 3, "modified_huber_loss": 4,
          "sigmoid_cross_entropy_with_logits": 5}
_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3, torch.int32: 4, torch.int64: 5,
       torch.uint8: 6, torch.bool: 6, torch.int8: 7, torch.int16: 8}


def ok(*ts) -> bool:
    """Device tensors of a dtype the kernels cover (fp32 / bf16)."""
    return all(t is not None and t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) for t in ts)


def _d(t):
    t = t.contiguous()
    if t.data_ptr() % 16:
        t = t.clone()
    return t


def act_fwd(name, x, a=0.0, b=0.0):
    x = _d(x)
    y = torch.empty_like(x)
    N.call("pa_act_fwd", ACT_ID[name], N.dt(x), N.ptr(x), N.ptr(y), x.numel(), float(a), float(b), N.stream())
    return y


def _same(ref, *ts):
    for t in ts:
        if t is not None and t.numel() != ref.numel():
            raise ValueError(f"fluid kernel operand of {t.numel()} elements, expected {ref.numel()}")


def act_bwd(name, dy, x=None, y=None, a=0.0, b=0.0):
    _same(dy, x, y)
    dy = _d(dy)
    x = _d(x) if x is not None else None
    y = _d(y) if y is not None else None
    dx = torch.empty_like(dy)
    N.call("pa_act_bwd", ACT_ID[name], N.dt(dy), N.ptr(x), N.ptr(y), N.ptr(dy), N.ptr(dx), dy.numel(), float(a),
           float(b), N.stream())
    return dx


def softmax_ce(logits, label=None, soft=None, ignore_index=-100):
    """Rows of ``logits`` [.., V] -> (softmax [.., V], loss [.., 1]); hard int64
    ``label`` [.., 1] or soft ``soft`` [.., V]."""
    V = logits.shape[-1]
    rows = logits.numel() // max(V, 1)
    if label is not None and label.numel() != rows:
        raise ValueError(f"softmax_ce: {label.numel()} labels for {rows} rows")
    _same(logits, soft)
    x = _d(logits)
    prob = torch.empty_like(x)
    loss = torch.empty(x.shape[:-1] + (1,), dtype=x.dtype, device=x.device)
    lab = _d(label.reshape(-1).long()) if label is not None else None
    sf = _d(soft.to(x.dtype)) if soft is not None else None
    N.call("pa_softmax_ce_prob_fwd", N.dt(x), N.ptr(x), N.ptr(lab), N.ptr(sf), N.ptr(prob), N.ptr(loss),
           x.numel() // max(V, 1), V, int(ignore_index), N.stream())
    return prob, loss


def softmax_ce_grad(prob, dloss, label=None, soft=None, ignore_index=-100):
    V = prob.shape[-1]
    rows = prob.numel() // max(V, 1)
    if dloss.numel() != rows or (label is not None and label.numel() != rows):
        raise ValueError(f"softmax_ce_grad: {dloss.numel()} grads / labels for {rows} rows")
    _same(prob, soft)
    p = _d(prob)
    g = _d(dloss.to(p.dtype).reshape(-1))
    dx = torch.empty_like(p)
    lab = _d(label.reshape(-1).long()) if label is not None else None
    sf = _d(soft.to(p.dtype)) if soft is not None else None
    N.call("pa_softmax_ce_prob_bwd", N.dt(p), N.ptr(p), N.ptr(lab), N.ptr(sf), N.ptr(g), N.ptr(dx),
           p.numel() // max(V, 1), V, int(ignore_index), N.stream())
    return dx


def cast(x, dtype):
    if x.dtype == dtype:
        return x.clone()
    if x.dtype not in _DT or dtype not in _DT or x.dtype in (torch.complex64, torch.complex128):
        return x.to(dtype)
    x = _d(x)
    y = torch.empty(x.shape, dtype=dtype, device=x.device)
    N.call("pa_cast_any", _DT[x.dtype], _DT[dtype], N.ptr(x), N.ptr(y), x.numel(), int(dtype == torch.bool),
           N.stream())
    return y


def _la(v):
    return (ctypes.c_long * max(1, len(v)))(*[int(x) for x in v])


def gather(x, sizes, strides, base=0):
    """out (dense, shape ``sizes``) [i] = x.flat[base + sum_d i_d * strides[d]]; the
    reachable offsets are checked against x before launch."""
    x = _d(x)
    sizes, strides = list(sizes), list(strides)
    if not sizes:
        sizes, strides = [1], [0]
    if len(sizes) > 8:
        raise ValueError("strided gather: at most 8 dims")
    lo = base + sum(min(0, (s - 1) * st) for s, st in zip(sizes, strides) if s > 0)
    hi = base + sum(max(0, (s - 1) * st) for s, st in zip(sizes, strides) if s > 0)
    out = torch.empty(sizes, dtype=x.dtype, device=x.device)
    if out.numel() == 0:
        return out
    if lo < 0 or hi >= x.numel():
        raise IndexError(f"strided gather reaches [{lo}, {hi}] of a {x.numel()}-element source")
    N.call("pa_strided_gather", x.element_size(), N.ptr(x), N.ptr(out), len(sizes), _la(sizes), _la(strides),
           int(base), N.stream())
    return out


def _cstrides(shape):
    st, acc = [], 1
    for s in reversed(shape):
        st.append(acc)
        acc *= s
    return list(reversed(st))


def permute(x, perm):
    st = _cstrides(x.shape)
    return gather(x, [x.shape[p] for p in perm], [st[p] for p in perm])


def flip(x, dims):
    st = _cstrides(x.shape)
    base = 0
    strides = list(st)
    for d in dims:
        d %= x.dim()
        base += (x.shape[d] - 1) * st[d]
        strides[d] = -st[d]
    return gather(x, list(x.shape), strides, base)


def slice_(x, axes, starts, ends):
    st = _cstrides(x.shape)
    sizes = list(x.shape)
    base = 0
    for a, s, e in zip(axes, starts, ends):
        n = x.shape[a]
        s = max(0, min(n, s + n if s < 0 else s))
        e = max(0, min(n, e + n if e < 0 else e))
        sizes[a] = max(0, e - s)
        base += s * st[a]
    return gather(x, sizes, st, base)


def expand(x, shape):
    """Broadcast ``x`` to ``shape`` (size-1 dims stride 0)."""
    lead = len(shape) - x.dim()
    st = [0] * lead + _cstrides(x.shape)
    src = [1] * lead + list(x.shape)
    return gather(x, list(shape), [0 if s == 1 and t != 1 else st[i] for i, (s, t) in enumerate(zip(src, shape))])


def tile(x, reps):
    """Fluid expand (expand_times): out[.., i, ..] = x[.., i % n, ..]."""
    reps = list(reps)
    st = _cstrides(x.shape)
    sizes, strides = [], []
    for n, r, s in zip(x.shape, reps, st):
        sizes += [r, n]
        strides += [0, s]
    return gather(x, sizes, strides).reshape([n * r for n, r in zip(x.shape, reps)])


def random(shape, kind, a, b, seed, dtype=torch.float32, device="cuda"):
    out = torch.empty(list(shape), dtype=dtype, device=device)
    N.call("pa_random", N.dt(out), N.ptr(out), out.numel(), 0 if kind == "uniform" else 1, float(a), float(b),
           ctypes.c_ulonglong(int(seed) & 0xFFFFFFFFFFFFFFFF), N.stream())
    return out


def loss_fwd(name, x, y, a=0.0, want_res=False):
    _same(x, y)
    x, y = _d(x), _d(y.to(x.dtype))
    out = torch.empty_like(x)
    res = torch.empty_like(x) if want_res else None
    N.call("pa_loss_fwd", LOSSES[name], N.dt(x), N.ptr(x), N.ptr(y), N.ptr(out), N.ptr(res), x.numel(), float(a),
           N.stream())
    return out, res


def loss_bwd(name, x, y, g, res=None, a=0.0):
    """dx = g (one value per row of x.numel() / g.numel() elements) * dloss/dx."""
    _same(x, y, res)
    if g.numel() == 0 or x.numel() % g.numel():
        raise ValueError(f"loss grad: {g.numel()} upstream values do not tile {x.numel()} elements")
    x, y = _d(x), _d(y.to(x.dtype))
    g = _d(g.to(x.dtype))
    res = _d(res) if res is not None else None
    dx = torch.empty_like(x)
    N.call("pa_loss_bwd", LOSSES[name], N.dt(x), N.ptr(x), N.ptr(y), N.ptr(res), N.ptr(g), N.ptr(dx), x.numel(),
           max(1, x.numel() // max(1, g.numel())), float(a), N.stream())
    return dx


def _check_off(offsets, n):
    offsets = [int(o) for o in offsets]
    if len(offsets) < 2 or offsets[0] < 0 or offsets[-1] > n or any(b < a for a, b in zip(offsets, offsets[1:])):
        raise ValueError(f"bad LoD offsets {offsets[:8]} for {n} elements")


def seq_softmax(x, offsets):
    _check_off(offsets, x.numel())
    x = _d(x)
    off = _mv.device_offsets(offsets, x.device, torch.int64)
    y = torch.empty_like(x)
    N.call("pa_seq_softmax_fwd", N.dt(x), N.ptr(x), N.ptr(off), N.ptr(y), len(offsets) - 1, N.stream())
    return y


def seq_softmax_grad(y, dy, offsets):
    _check_off(offsets, y.numel())
    _same(y, dy)
    y, dy = _d(y), _d(dy)
    off = _mv.device_offsets(offsets, y.device, torch.int64)
    dx = torch.empty_like(y)
    N.call("pa_seq_softmax_bwd", N.dt(y), N.ptr(y), N.ptr(dy), N.ptr(off), N.ptr(dx), len(offsets) - 1, N.stream())
    return dx
