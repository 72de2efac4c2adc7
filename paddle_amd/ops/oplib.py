"""Python side of the general GPU operator library (csrc/kernels/oplib.hip).

Each function takes torch tensors, runs the HIP kernel for CUDA fp32 / bf16 inputs
and returns ``None`` when the kernel does not cover the case (other dtypes, CPU
tensors, shapes past the kernel limits), so operator kernels can write
``out = oplib.binary(...)`` and fall back to the reference torch expression only
where the native path is not defined.  On a GPU box the covered cases never fall
back silently: a missing library raises (``_native.lib``).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from ..framework import mixed_vector as _mv

from . import _native as N
from ..autograd import tape as _tape

_ENABLED = os.environ.get("PADDLE_AMD_OPLIB", "1") != "0"
_DT = {torch.float32: 0, torch.bfloat16: 1}
_BIN = {"add": 0, "sub": 1, "mul": 2, "div": 3, "max": 4, "min": 5, "pow": 6}
_RED = {"sum": 0, "mean": 1, "max": 2, "min": 3, "prod": 4}
_POOL = {"SUM": 0, "AVERAGE": 1, "SQRT": 2, "MAX": 3, "LAST": 4, "FIRST": 5}


def _ok(*ts):
    return _ENABLED and all(t is not None and t.is_cuda and t.dtype in _DT for t in ts)


def _larr(vals):
    a = (ctypes.c_long * max(len(vals), 1))(*[int(v) for v in vals])
    return a


# ------------------------------------------------------------------ binary


def fill_(t, value):
    """t[...] = value on the elementwise kernel of tensor_ops.hip (any device dtype
    and layout the kernel covers; else torch's fill).  The kernel takes the value as a
    double: integer fills beyond 2**53 (int64 sentinels) take torch's exact fill."""
    exact = not (not t.dtype.is_floating_point and not t.dtype.is_complex and isinstance(value, int)
                 and abs(value) > 2 ** 53)
    if t.is_cuda and t.numel() and exact:
        from . import _native as N
        from . import aten_native as A

        F = N.fastops()
        if F is not None and F.fill_(t, float(value)):
            return t

        if t.dtype in A._DT and A._launch(A.U["fill"], t, [], a=float(value), cdt=A._cdt(t.dtype)):
            return t
    return t.fill_(value)


def add_(a, b):
    """a += b in place on the elementwise kernel (same shape; b's dtype may differ):
    a direct launch, no pass through the ATen dispatcher or the native-dispatch mode."""
    if a.is_cuda and b.is_cuda and a.shape == b.shape and a.numel():
        from . import _native as N
        from . import aten_native as A

        F = N.fastops()
        if F is not None and F.add_(a, b, 1.0):
            return a

        if a.dtype in A._DT and b.dtype in A._DT and A._launch(A.B["add"], a, [a, b], a=1.0,
                                                                 cdt=A._cdt(a.dtype)):
            return a
    return a.add_(b)


def full_like(t, value):
    """A new tensor shaped like ``t`` filled with ``value`` (native fill)."""
    return fill_(torch.empty_like(t, memory_format=torch.contiguous_format), value)


def binary(op, x, y):
    """out = x (op) y with y already broadcast-compatible (expandable) to x's shape."""
    if not _ok(x, y) or x.dtype != y.dtype or op not in _BIN or x.dim() > 6:
        return None
    shape = tuple(x.shape)
    try:
        yb = y.expand(shape)
    except RuntimeError:
        return None
    x = x.contiguous()
    out = torch.empty(shape, dtype=x.dtype, device=x.device)
    n = x.numel()
    if n == 0:
        return out
    same = tuple(y.shape) == shape and y.is_contiguous() and x.data_ptr() % 32 == 0 and y.data_ptr() % 32 == 0
    nd = max(x.dim(), 1)
    size = list(shape) or [1]
    sx = list(x.stride()) or [1]
    sy = list(yb.stride()) or [0]
    N.call("pa_binary", _DT[x.dtype], _BIN[op], N.ptr(x), N.ptr(yb if same else y), N.ptr(out), n, nd,
           _larr(size), _larr(sx), _larr(sy), int(same), N.stream())
    return out


# ------------------------------------------------------------------ reduce


def reduce(op, x, dims, keep_dim=False):
    """Reduction over ``dims`` (list of ints).  Native when the reduced axes form one
    contiguous block (any tensor after a permute does): x -> [pre, R, post]."""
    if not _ok(x) or op not in _RED or x.numel() == 0:
        return None
    nd = x.dim()
    dims = sorted({d % nd for d in dims}) if nd else []
    if not dims:
        return None
    if dims != list(range(dims[0], dims[-1] + 1)):
        keep = [d for d in range(nd) if d not in dims]
        xp = x.permute(keep + dims).contiguous()
        out = reduce(op, xp, list(range(len(keep), nd)))
        if out is None:
            return None
        if keep_dim:
            shp = [1 if d in dims else x.shape[d] for d in range(nd)]
            out = out.reshape(shp)
        return out
    x = x.contiguous()
    pre = int(np.prod(x.shape[:dims[0]])) if dims[0] > 0 else 1
    R = int(np.prod([x.shape[d] for d in dims]))
    post = int(np.prod(x.shape[dims[-1] + 1:])) if dims[-1] + 1 < nd else 1
    oshape = [x.shape[d] for d in range(nd) if d not in dims] if not keep_dim else \
        [1 if d in dims else x.shape[d] for d in range(nd)]
    out = torch.empty(oshape, dtype=x.dtype, device=x.device)
    N.call("pa_reduce", _DT[x.dtype], _RED[op], N.ptr(x), N.ptr(out), pre, R, post, N.stream())
    return out


# ------------------------------------------------------------------ dropout

_PHILOX = {"offset": 0}


def dropout(x, p, seed=None, upscale=False):
    """Philox4x32-10 dropout: returns (out, mask uint8).  ``seed`` None draws one from
    torch's generator; each call advances a per-process counter offset."""
    if not _ok(x):
        return None
    x = x.contiguous()
    if seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    off = _PHILOX["offset"]
    n = x.numel()
    _PHILOX["offset"] += (n + 3) // 4
    out = torch.empty_like(x)
    mask = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    scale = 1.0 / (1.0 - p) if (upscale and p < 1.0) else 1.0
    N.call("pa_dropout", _DT[x.dtype], N.ptr(x), N.ptr(out), N.ptr(mask), n, float(p), float(scale),
           ctypes.c_ulonglong(seed), ctypes.c_ulonglong(off), N.stream())
    return out, mask


def mask_mul(d, mask, scale=1.0):
    if not _ok(d) or mask.dtype != torch.uint8:
        return None
    d = d.contiguous()
    out = torch.empty_like(d)
    mask = mask.contiguous()  # bound: a temporary passed to ptr() is freed before the launch
    N.call("pa_mask_mul", _DT[d.dtype], N.ptr(d), N.ptr(mask), N.ptr(out), d.numel(), float(scale),
           N.stream())
    return out


# ------------------------------------------------------------------ top-k


def topk(x, k):
    """Top-k along the last axis -> (values, int64 indices); k <= 64."""
    if not _ok(x) or x.dim() == 0 or k <= 0 or k > 64 or k > x.shape[-1]:
        return None
    x = x.contiguous()
    n = x.shape[-1]
    rows = x.numel() // n
    vals = torch.empty(*x.shape[:-1], k, dtype=x.dtype, device=x.device)
    idx = torch.empty(*x.shape[:-1], k, dtype=torch.int64, device=x.device)
    N.call("pa_topk", _DT[x.dtype], N.ptr(x), N.ptr(vals), N.ptr(idx), rows, n, k, N.stream())
    return vals, idx


# ------------------------------------------------------------------ optimizers


def _lr(lr, dev):
    return lr.float().contiguous() if torch.is_tensor(lr) else torch.tensor([float(lr)], device=dev)


def sgd_(p, g, lr):
    if not _ok(p, g) or p.dtype != g.dtype or not p.is_contiguous():
        return None
    g, lr_t = g.contiguous(), _lr(lr, p.device)
    N.call("pa_sgd", _DT[p.dtype], N.ptr(p), N.ptr(g), N.ptr(lr_t), p.numel(), N.stream())
    return p


def sgd_sparse_(p, rows, values, lr):
    """Param[rows] -= lr * values (duplicate rows accumulate)."""
    if not (_ok(p, values) and p.dtype == torch.float32 and values.dtype == torch.float32 and p.is_contiguous()):
        return None
    rows = torch.as_tensor(rows, dtype=torch.int64).to(p.device)
    D = p.numel() // p.shape[0]
    values, lr_t = values.contiguous(), _lr(lr, p.device)
    N.call("pa_sgd_sparse", N.ptr(p), N.ptr(rows), N.ptr(values), N.ptr(lr_t),
           rows.numel(), D, N.stream())
    return p


def adagrad_(p, g, m, lr, eps):
    if not (_ok(p, g, m) and p.dtype == g.dtype == m.dtype == torch.float32 and p.is_contiguous()
            and m.is_contiguous()):
        return None
    g, lr_t = g.contiguous(), _lr(lr, p.device)
    N.call("pa_adagrad", N.ptr(p), N.ptr(g), N.ptr(m), N.ptr(lr_t), p.numel(), float(eps),
           N.stream())
    return p


# ------------------------------------------------------------------ rows


def gather_rows(src, idx, fill=0.0):
    """out[i] = src[idx[i]] (idx < 0: ``fill``); src viewed as [rows, D]."""
    if not _ok(src) or src.dim() == 0:
        return None
    src = src.contiguous()
    D = src.numel() // max(src.shape[0], 1)
    idx = torch.as_tensor(np.asarray(idx, dtype=np.int32)).to(src.device) if not torch.is_tensor(idx) \
        else idx.to(device=src.device, dtype=torch.int32)
    out = torch.empty((idx.numel(),) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    N.call("pa_gather_rows", _DT[src.dtype], N.ptr(src), N.ptr(idx), N.ptr(out), idx.numel(), D, float(fill),
           N.stream())
    return out


def scatter_add_rows(v, idx, nrows):
    """out[idx[i]] += v[i] into a zero fp32 [nrows, ...] (idx < 0 skipped)."""
    if not _ok(v):
        return None
    v32 = v.float().contiguous()
    D = v32.numel() // max(v32.shape[0], 1)
    idx = torch.as_tensor(np.asarray(idx, dtype=np.int32)).to(v.device) if not torch.is_tensor(idx) \
        else idx.to(device=v.device, dtype=torch.int32)
    out = torch.zeros((nrows,) + tuple(v.shape[1:]), dtype=torch.float32, device=v.device)
    N.call("pa_scatter_add_rows", N.ptr(v32), N.ptr(idx), N.ptr(out), idx.numel(), D, N.stream())
    return out.to(v.dtype)


def merge_rows(rows, values):
    """SelectedRows MergeAdd: unique rows (sorted) and the summed values."""
    if not _ok(values):
        return None
    r = torch.as_tensor(np.asarray(rows, dtype=np.int64))
    uniq, inv = torch.unique(r, sorted=True, return_inverse=True)
    return uniq.tolist(), scatter_add_rows(values, inv.to(torch.int32), uniq.numel())


# ------------------------------------------------------------------ sequences


def seq_pool(x, offsets, pooltype, pad_value=0.0):
    """x [T, ...] grouped by host offsets -> (out [nseq, ...], maxindex int32 or None)."""
    t = _POOL.get(pooltype.upper())
    if not _ok(x) or t is None or x.dim() == 0:
        return None
    x = x.contiguous()
    nseq = len(offsets) - 1
    D = x.numel() // max(x.shape[0], 1)
    off = _mv.device_offsets(offsets, x.device, torch.int32)
    out = torch.empty((nseq,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    maxi = torch.empty((nseq,) + tuple(x.shape[1:]), dtype=torch.int32, device=x.device) if t == 3 else None
    N.call("pa_seq_pool", _DT[x.dtype], N.ptr(x), N.ptr(off), N.ptr(out), N.ptr(maxi), nseq, D, t, float(pad_value),
           N.stream())
    return out, maxi


def seq_pool_grad(dout, offsets, pooltype, maxi, nrows):
    t = _POOL.get(pooltype.upper())
    if not _ok(dout) or t is None:
        return None
    dout = dout.contiguous()
    nseq = len(offsets) - 1
    D = dout.numel() // max(nseq, 1)
    off = _mv.device_offsets(offsets, dout.device, torch.int32)
    dx = torch.zeros((nrows,) + tuple(dout.shape[1:]), dtype=dout.dtype, device=dout.device)
    N.call("pa_seq_pool_grad", _DT[dout.dtype], N.ptr(dout), N.ptr(off), N.ptr(maxi), N.ptr(dx), nseq, D, t,
           N.stream())
    return dx


# ------------------------------------------------------------------ GRU gates


class _GruGateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ur, h):
        ur, h = ur.contiguous(), h.contiguous()
        B, D = h.shape
        u, r, rh = (torch.empty_like(h) for _ in range(3))
        N.call("pa_gru_gate", N.ptr(ur), N.ptr(h), N.ptr(u), N.ptr(r), N.ptr(rh), B, D, N.stream())
        ctx.save_for_backward(u, r, h)
        return u, r, rh

    @staticmethod
    def backward(ctx, du, dr, drh):
        u, r, h = ctx.saved_tensors
        B, D = h.shape
        du = torch.zeros_like(u) if du is None else du.contiguous()
        drh = torch.zeros_like(u) if drh is None else drh.contiguous()
        dur = torch.empty(B, 2 * D, dtype=h.dtype, device=h.device)
        dh = torch.zeros_like(h)
        N.call("pa_gru_gate_bwd", N.ptr(du), N.ptr(drh), N.ptr(u), N.ptr(r), N.ptr(h), N.ptr(dur), N.ptr(dh), B, D,
               N.stream())
        if dr is not None:  # r is also an output: its direct gradient joins through sigmoid'
            dur[:, D:] += dr * r * (1 - r)
        return dur, dh


class _GruOutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cpre, u, h):
        cpre, u, h = cpre.contiguous(), u.contiguous(), h.contiguous()
        c, hn = torch.empty_like(h), torch.empty_like(h)
        N.call("pa_gru_out", N.ptr(cpre), N.ptr(u), N.ptr(h), N.ptr(c), N.ptr(hn), h.numel(), N.stream())
        ctx.save_for_backward(u, h, c)
        return hn, c

    @staticmethod
    def backward(ctx, dhn, dc):
        u, h, c = ctx.saved_tensors
        dhn = torch.zeros_like(h) if dhn is None else dhn.contiguous()
        dcpre, du, dh = (torch.empty_like(h) for _ in range(3))
        N.call("pa_gru_out_bwd", N.ptr(dhn), N.ptr(u), N.ptr(h), N.ptr(c), N.ptr(dcpre), N.ptr(du), N.ptr(dh),
               h.numel(), N.stream())
        if dc is not None:
            dcpre = dcpre + dc * (1 - c * c)
        return dcpre, du, dh


def gru_step(g, h, W, D):
    """One GRU step with sigmoid gates / tanh candidate on the fused kernels:
    returns (h_new, u, r, c, rh) like operators.rnn_ops._gru_step."""
    if not (_ENABLED and g.is_cuda and g.dtype == torch.float32 and h.dtype == torch.float32):
        return None
    ur = g[:, :2 * D] + h @ W[:, :2 * D]
    u, r, rh = _tape.apply(_GruGateFn, ur, h)
    hn, c = _tape.apply(_GruOutFn, g[:, 2 * D:] + rh @ W[:, 2 * D:], u, h)
    return hn, u, r, c, rh


# ------------------------------------------------------------------ autograd-aware entry points
# Operator kernels run under autograd when the executor stashes their graph for the
# automatic VJP (framework/registry.py), so the native paths are autograd Functions
# whose backward passes run on the same kernels.

_NEG1 = {}


def _neg1(dev, dt):
    k = (dev, dt)
    if k not in _NEG1:
        _NEG1[k] = torch.full((1,), -1.0, dtype=dt, device=dev)
    return _NEG1[k]


def _sum_to(g, shape):
    """Sum a full-shape gradient down to a broadcast operand's ``shape`` (same rank)."""
    if tuple(g.shape) == tuple(shape):
        return g
    dims = [d for d in range(g.dim()) if shape[d] == 1 and g.shape[d] != 1]
    r = reduce("sum", g, dims, keep_dim=True) if dims else g
    return r if r is not None else g.sum(dims, keepdim=True)


class _BinaryFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, op, x, y):
        ctx.op = op
        ctx.save_for_backward(x, y)
        return binary(op, x, y)

    @staticmethod
    def backward(ctx, d):
        x, y = ctx.saved_tensors
        op = ctx.op
        d = d.contiguous()
        m1 = _neg1(d.device, d.dtype)
        if op == "add":
            dx, dy = d, d
        elif op == "sub":
            dx, dy = d, binary("mul", d, m1)
        elif op == "mul":
            dx, dy = binary("mul", d, y), binary("mul", d, x)
        else:  # div
            dx = binary("div", d, y)
            dy = binary("mul", binary("mul", dx, binary("div", x, y)), m1)
        gx = dx if ctx.needs_input_grad[1] else None
        gy = _sum_to(dy, y.shape) if ctx.needs_input_grad[2] else None
        return None, gx, gy


def ew(op, x, y):
    """Elementwise x (op) y with y broadcast to x (same rank, size-1 dims broadcast);
    None when the native path does not apply."""
    if not _ok(x, y) or x.dtype != y.dtype or x.dim() != y.dim() or x.dim() > 6:
        return None
    if any(b != a and b != 1 for a, b in zip(x.shape, y.shape)):
        return None
    if op in ("add", "sub", "mul", "div") and (x.requires_grad or y.requires_grad):
        return _tape.apply(_BinaryFn, op, x, y)
    if x.requires_grad or y.requires_grad:
        return None  # max / min / pow gradients stay on the torch reference
    return binary(op, x, y)


class _ReduceFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, op, x, dims, keep_dim):
        ctx.op, ctx.shape = op, x.shape
        ctx.dims = sorted({d % max(x.dim(), 1) for d in dims})
        ctx.keep = keep_dim
        return reduce(op, x, dims, keep_dim)

    @staticmethod
    def backward(ctx, g):
        shp = [1 if d in ctx.dims else ctx.shape[d] for d in range(len(ctx.shape))]
        g = g.reshape(shp)
        if ctx.op == "mean":
            R = int(np.prod([ctx.shape[d] for d in ctx.dims]))
            g = g / R
        return None, g.expand(ctx.shape).contiguous(), None, None


def reduce_op(op, x, dims, keep_dim=False):
    if not _ok(x) or op not in _RED or x.numel() == 0 or not dims:
        return None
    if x.requires_grad:
        if op not in ("sum", "mean"):
            return None
        return _tape.apply(_ReduceFn, op, x, list(dims), keep_dim)
    return reduce(op, x, dims, keep_dim)


class _TopkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k):
        vals, idx = topk(x, k)
        ctx.save_for_backward(idx)
        ctx.shape = x.shape
        ctx.mark_non_differentiable(idx)
        return vals, idx

    @staticmethod
    def backward(ctx, gv, gi):
        (idx,) = ctx.saved_tensors
        dx = torch.zeros(ctx.shape, dtype=gv.dtype, device=gv.device)
        return dx.scatter_(-1, idx, gv), None


def topk_op(x, k):
    if not _ok(x) or x.dim() == 0 or k <= 0 or k > 64 or k > x.shape[-1]:
        return None
    return _tape.apply(_TopkFn, x, k)


class _SeqPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, offsets, pooltype):
        out, maxi = seq_pool(x, offsets, pooltype)
        ctx.offsets, ctx.pooltype, ctx.nrows = offsets, pooltype, x.shape[0]
        ctx.save_for_backward(maxi if maxi is not None else torch.empty(0, device=x.device))
        return out, (maxi if maxi is not None else torch.zeros(out.shape, dtype=torch.int32, device=x.device))

    @staticmethod
    def backward(ctx, g, _gi):
        (maxi,) = ctx.saved_tensors
        return seq_pool_grad(g, ctx.offsets, ctx.pooltype, maxi if maxi.numel() else None, ctx.nrows), None, None


def seq_pool_op(x, offsets, pooltype):
    """-> (out, maxindex int32) or None."""
    if not _ok(x) or pooltype.upper() not in _POOL or x.dim() == 0:
        return None
    return _tape.apply(_SeqPoolFn, x, list(offsets), pooltype)


class _GatherRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, idx, fill):
        ctx.save_for_backward(idx)
        ctx.nrows = src.shape[0]
        return gather_rows(src, idx, fill)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        return scatter_add_rows(g.contiguous(), idx, ctx.nrows), None, None


def gather_rows_op(src, idx, fill=0.0):
    """Row gather with a scatter-add backward (sequence expand / pad / unpad)."""
    if not _ok(src) or src.dim() == 0:
        return None
    idx = torch.as_tensor(np.asarray(idx, dtype=np.int32)).to(src.device) if not torch.is_tensor(idx) \
        else idx.to(device=src.device, dtype=torch.int32)
    return _tape.apply(_GatherRowsFn, src, idx, float(fill))


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed, upscale):
        out, mask = dropout(x, p, seed, upscale)
        ctx.save_for_backward(mask)
        ctx.scale = 1.0 / (1.0 - p) if (upscale and p < 1.0) else 1.0
        ctx.mark_non_differentiable(mask)
        return out, mask

    @staticmethod
    def backward(ctx, g, _gm):
        (mask,) = ctx.saved_tensors
        return mask_mul(g, mask, ctx.scale), None, None, None


def dropout_op(x, p, seed=None, upscale=False):
    """-> (out, uint8 mask) on the Philox kernel, or None."""
    if not _ok(x):
        return None
    return _tape.apply(_DropoutFn, x, float(p), seed, bool(upscale))


# ------------------------------------------------------------------ misc Fluid kernels (misc.hip)


def one_hot(x, depth):
    """x int64 [...] -> float32 [..., depth]; raises on out-of-range ids."""
    if not (_ENABLED and x.is_cuda):
        return None
    xl = x.to(torch.int64).contiguous()
    out = torch.empty(tuple(x.shape) + (depth,), dtype=torch.float32, device=x.device)
    bad = torch.zeros(1, dtype=torch.int32, device=x.device)
    N.call("pa_one_hot", N.ptr(xl), N.ptr(out), xl.numel(), int(depth), N.ptr(bad), N.stream())
    if int(bad.item()):
        raise ValueError(f"one_hot: an id is outside [0, {depth})")
    return out


_PAD_MODE = {"constant": 0, "reflect": 1, "edge": 2}


class _Pad2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pads, mode, value, nhwc):
        x = x.contiguous()
        if nhwc:
            Nn, H, W, C = x.shape
        else:
            Nn, C, H, W = x.shape
        t, b, l, r = pads
        shape = (Nn, H + t + b, W + l + r, C) if nhwc else (Nn, C, H + t + b, W + l + r)
        y = torch.empty(shape, dtype=x.dtype, device=x.device)
        N.call("pa_pad2d", _DT[x.dtype], N.ptr(x), N.ptr(y), Nn, C, H, W, t, b, l, r, _PAD_MODE[mode], float(value),
               int(nhwc), N.stream())
        ctx.meta = (Nn, C, H, W, t, b, l, r, _PAD_MODE[mode], int(nhwc), x.shape, x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        Nn, C, H, W, t, b, l, r, mode, nhwc, shape, dt = ctx.meta
        dy = dy.contiguous()
        dx = torch.zeros(shape, dtype=torch.float32, device=dy.device)
        N.call("pa_pad2d_bwd", _DT[dy.dtype], N.ptr(dy), N.ptr(dx), Nn, C, H, W, t, b, l, r, mode, nhwc, N.stream())
        return dx.to(dt), None, None, None, None


def pad2d_op(x, pads, mode="constant", value=0.0, nhwc=False):
    if not _ok(x) or x.dim() != 4 or mode not in _PAD_MODE:
        return None
    H, W = (x.shape[1], x.shape[2]) if nhwc else (x.shape[2], x.shape[3])
    t, b, l, r = pads
    if mode == "reflect" and (t >= H or b >= H or l >= W or r >= W):
        return None
    return _tape.apply(_Pad2dFn, x, tuple(int(v) for v in pads), mode, float(value), bool(nhwc))


class _LrnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, n, k, alpha, beta):
        x = x.contiguous()
        Nn, C = x.shape[0], x.shape[1]
        HW = x.numel() // max(Nn * C, 1)
        out = torch.empty_like(x)
        mid = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        N.call("pa_lrn_fwd", _DT[x.dtype], N.ptr(x), N.ptr(out), N.ptr(mid), Nn, C, HW, int(n), float(k),
               float(alpha), float(beta), N.stream())
        ctx.save_for_backward(x, mid)
        ctx.args = (Nn, C, HW, int(n), float(alpha), float(beta))
        ctx.mark_non_differentiable(mid)
        return out, mid

    @staticmethod
    def backward(ctx, dout, dmid):
        x, mid = ctx.saved_tensors
        Nn, C, HW, n, alpha, beta = ctx.args
        dout = dout.contiguous()
        dx = torch.empty_like(x)
        N.call("pa_lrn_bwd", _DT[x.dtype], N.ptr(x), N.ptr(dout), N.ptr(mid), N.ptr(dx), Nn, C, HW, n, alpha, beta,
               N.stream())
        return dx, None, None, None, None


def lrn_op(x, n, k, alpha, beta):
    """(out, mid) of cross-channel LRN (NCHW) or None."""
    if not _ok(x) or x.dim() < 2:
        return None
    return _tape.apply(_LrnFn, x, n, k, alpha, beta)


class _RowConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, seq_start, seq_end):
        x, w = x.contiguous(), w.contiguous()
        rows, D = x.shape[0], x.numel() // max(x.shape[0], 1)
        out = torch.empty_like(x)
        N.call("pa_row_conv_fwd", _DT[x.dtype], N.ptr(x), N.ptr(w), N.ptr(seq_end), N.ptr(out), rows, D, w.shape[0],
               N.stream())
        ctx.save_for_backward(x, w, seq_start, seq_end)
        return out

    @staticmethod
    def backward(ctx, dy):
        x, w, seq_start, seq_end = ctx.saved_tensors
        dy = dy.contiguous()
        rows, D = x.shape[0], x.numel() // max(x.shape[0], 1)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty(w.shape, dtype=torch.float32, device=w.device) if ctx.needs_input_grad[1] else None
        N.call("pa_row_conv_bwd", _DT[x.dtype], N.ptr(dy), N.ptr(x), N.ptr(w), N.ptr(seq_start), N.ptr(seq_end),
               N.ptr(dx), N.ptr(dw), rows, D, w.shape[0], N.stream())
        return dx, (dw.to(w.dtype) if dw is not None else None), None, None


def row_conv_op(x, w, offsets):
    """Lookahead row convolution over LoD sequences ``offsets`` (level-0 offsets)."""
    if not _ok(x, w) or x.dtype != w.dtype:
        return None
    rows = x.shape[0]
    start = np.zeros(rows, dtype=np.int32)
    end = np.zeros(rows, dtype=np.int32)
    for s, e in zip(offsets[:-1], offsets[1:]):
        start[s:e], end[s:e] = s, e
    st = torch.as_tensor(start).to(x.device)
    en = torch.as_tensor(end).to(x.device)
    return _tape.apply(_RowConvFn, x, w, st, en)


def argsort_op(x, axis=-1, descending=False):
    """(sorted values, int64 indices) along the last axis for rows of <= 2048."""
    if not _ok(x) or x.dim() == 0:
        return None
    ax = axis % x.dim()
    if ax != x.dim() - 1 or x.shape[-1] > 2048 or x.shape[-1] == 0:
        return None
    xc = x.detach().contiguous()
    n = xc.shape[-1]
    rows = xc.numel() // n
    vals = torch.empty_like(xc)
    idx = torch.empty(xc.shape, dtype=torch.int64, device=x.device)
    N.call("pa_argsort_rows", _DT[xc.dtype], N.ptr(xc), N.ptr(vals), N.ptr(idx), rows, n, int(descending), N.stream())
    return vals, idx


def accuracy_op(indices, label):
    """(accuracy float32[1], correct int32[1], total int32[1])."""
    if not (_ENABLED and indices.is_cuda):
        return None
    ind = indices.to(torch.int64).contiguous()
    lab = label.reshape(-1).to(torch.int64).contiguous()
    rows, k = ind.shape[0], ind.numel() // max(ind.shape[0], 1)
    correct = torch.empty(1, dtype=torch.int32, device=ind.device)
    total = torch.empty(1, dtype=torch.int32, device=ind.device)
    acc = torch.empty(1, dtype=torch.float32, device=ind.device)
    N.call("pa_accuracy", N.ptr(ind), N.ptr(lab), rows, k, N.ptr(correct), N.ptr(acc), N.ptr(total), N.stream())
    return acc, correct, total


def _cat_into(xs, axis, out):
    pre = int(np.prod(out.shape[:axis])) if axis else 1
    post = int(np.prod(out.shape[axis + 1:])) if axis + 1 < out.dim() else 1
    es = out.element_size()
    dpitch = out.shape[axis] * post * es
    off = 0
    for x in xs:
        w = x.shape[axis] * post * es
        N.call("pa_copy2d", ctypes.c_void_p(out.data_ptr() + off), dpitch, N.ptr(x), w, w, pre, N.stream())
        off += w


class _ConcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, axis, *xs):
        xs = [x.contiguous() for x in xs]
        shape = list(xs[0].shape)
        shape[axis] = sum(x.shape[axis] for x in xs)
        out = torch.empty(shape, dtype=xs[0].dtype, device=xs[0].device)
        _cat_into(xs, axis, out)
        ctx.axis, ctx.sizes = axis, [x.shape[axis] for x in xs]
        return out

    @staticmethod
    def backward(ctx, g):
        return (None,) + tuple(split_op(g, ctx.sizes, ctx.axis))


class _SplitFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, axis, sizes):
        x = x.contiguous()
        pre = int(np.prod(x.shape[:axis])) if axis else 1
        post = int(np.prod(x.shape[axis + 1:])) if axis + 1 < x.dim() else 1
        es = x.element_size()
        spitch = x.shape[axis] * post * es
        outs, off = [], 0
        for s in sizes:
            shape = list(x.shape)
            shape[axis] = s
            o = torch.empty(shape, dtype=x.dtype, device=x.device)
            w = s * post * es
            N.call("pa_copy2d", N.ptr(o), w, ctypes.c_void_p(x.data_ptr() + off), spitch, w, pre, N.stream())
            outs.append(o)
            off += w
        ctx.axis = axis
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        gs = [g if g is not None else None for g in gs]
        if any(g is None for g in gs):
            return None, None, None
        return concat_op(list(gs), ctx.axis), None, None


def concat_op(xs, axis=0):
    if not xs or not all(_ok(x) for x in xs) or len({x.dtype for x in xs}) != 1:
        return None
    axis = axis % xs[0].dim()
    return _tape.apply(_ConcatFn, axis, *xs)


def split_op(x, sizes, axis=0):
    if not _ok(x):
        return None
    axis = axis % x.dim()
    return list(_tape.apply(_SplitFn, x, axis, list(sizes)))


# ------------------------------------------------ sequence / detection / metric (seqdet.hip)


def _i32(vals, dev):
    return torch.as_tensor(np.asarray(vals, dtype=np.int32)).to(dev)


class _CtcFn(torch.autograd.Function):
    """CTC loss with the warp-ctc gradient contract (warpctc_op.h): the loss is the
    plain -log p; ``norm_by_times`` only scales the gradient by 1/T_n."""

    @staticmethod
    def forward(ctx, logits, labels, xoff, loff, blank, norm_by_times):
        x = logits.detach().float().contiguous()
        T, C = x.shape
        n = len(xoff) - 1
        lens = [b - a for a, b in zip(loff[:-1], loff[1:])]
        smax = 2 * max(lens + [0]) + 1
        dev = x.device
        xo, lo = _i32(xoff, dev), _i32(loff, dev)
        lab = labels.reshape(-1).to(torch.int32).contiguous()
        if lab.numel() == 0:
            lab = torch.zeros(1, dtype=torch.int32, device=dev)
        lse = torch.empty(max(T, 1), dtype=torch.float32, device=dev)
        alpha = torch.empty(max(T, 1) * smax, dtype=torch.float32, device=dev)
        beta = torch.empty_like(alpha)
        loss = torch.empty(n, dtype=torch.float32, device=dev)
        grad = torch.empty_like(x)
        N.call("pa_ctc_loss", N.ptr(x), N.ptr(xo), N.ptr(lab), N.ptr(lo), n, T, C, smax, int(blank), N.ptr(lse),
               N.ptr(alpha), N.ptr(beta), N.ptr(loss), N.ptr(grad), N.stream())
        tl = torch.as_tensor([b - a for a, b in zip(xoff[:-1], xoff[1:])], dtype=torch.float32)
        seq = torch.repeat_interleave(torch.arange(n), tl.long()).to(dev)
        ctx.save_for_backward(grad, seq, tl.to(dev))
        ctx.norm, ctx.dt, ctx.xoff = norm_by_times, logits.dtype, xoff
        return loss.reshape(n, 1).to(logits.dtype)

    @staticmethod
    def backward(ctx, dloss):
        grad, seq, tl = ctx.saved_tensors
        w = dloss.reshape(-1).float()
        if ctx.norm:
            w = w / tl.clamp(min=1)
        g = seq_scale_op(grad, ctx.xoff, w)  # sequence_scale.cu: row *= w[sequence(row)]
        return g.to(ctx.dt), None, None, None, None, None


def ctc_loss_op(logits, labels, xoff, loff, blank=0, norm_by_times=False):
    """Per-sequence CTC loss [N, 1] over LoD-packed logits [T_total, C] (softmax inside)."""
    if not (_ENABLED and logits.is_cuda and logits.dim() == 2 and logits.dtype in _DT):
        return None
    if 2 * max([b - a for a, b in zip(loff[:-1], loff[1:])] + [0]) + 1 > 8192:
        return None
    return _tape.apply(_CtcFn, logits, labels, list(xoff), list(loff), int(blank), bool(norm_by_times))


class _RoiPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rois, bid, ph, pw, scale):
        xc = x.float().contiguous()
        B, C, H, W = xc.shape
        R = rois.shape[0]
        out = torch.empty(R, C, ph, pw, dtype=torch.float32, device=x.device)
        am = torch.empty(R, C, ph, pw, dtype=torch.int64, device=x.device)
        r = rois.float().contiguous()
        N.call("pa_roi_pool_fwd", N.ptr(xc), N.ptr(r), N.ptr(bid), R, C, H, W, ph, pw, float(scale), N.ptr(out),
               N.ptr(am), N.stream())
        ctx.save_for_backward(am, bid)
        ctx.shape, ctx.dt = (B, C, H, W), x.dtype
        ctx.mark_non_differentiable(am)
        return out.to(x.dtype), am

    @staticmethod
    def backward(ctx, dy, _dam):
        am, bid = ctx.saved_tensors
        B, C, H, W = ctx.shape
        R, _, ph, pw = am.shape
        dx = torch.zeros(B, C, H, W, dtype=torch.float32, device=am.device)
        d = dy.float().contiguous()
        N.call("pa_roi_pool_bwd", N.ptr(d), N.ptr(am), N.ptr(bid), R, C, H, W, ph, pw, N.ptr(dx), N.stream())
        return dx.to(ctx.dt), None, None, None, None, None


def roi_pool_op(x, rois, batch_ids, pooled_h, pooled_w, scale):
    """(Out [R, C, ph, pw], Argmax int64) with roi_pool_op.cu's bin boundaries."""
    if not (_ENABLED and x.is_cuda and x.dim() == 4 and x.dtype in _DT):
        return None
    bid = _i32(batch_ids if len(batch_ids) else [0], x.device)
    return _tape.apply(_RoiPoolFn, x, rois, bid, int(pooled_h), int(pooled_w), float(scale))


def edit_distance_op(hyps, refs, hoff, roff, normalized=False):
    """Levenshtein distance per (hyp, ref) sequence pair, float32 [N, 1]."""
    if not (_ENABLED and hyps.is_cuda):
        return None
    n = len(hoff) - 1
    if n <= 0:
        return None
    dev = hyps.device
    h = hyps.reshape(-1).to(torch.int64).contiguous()
    r = refs.reshape(-1).to(torch.int64).contiguous()
    h = h if h.numel() else torch.zeros(1, dtype=torch.int64, device=dev)
    r = r if r.numel() else torch.zeros(1, dtype=torch.int64, device=dev)
    wsw = max(b - a for a, b in zip(roff[:-1], roff[1:])) + 1
    ws = torch.empty(n * 2 * wsw, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    ho, ro = _i32(hoff, dev), _i32(roff, dev)  # held: a freed temporary's block would be reused
    N.call("pa_edit_distance", N.ptr(h), N.ptr(ho), N.ptr(r), N.ptr(ro), n, wsw, N.ptr(ws),
           int(normalized), N.ptr(out), N.stream())
    return out.reshape(n, 1)


def ctc_align_op(x, offsets, blank=0, merge_repeated=True):
    """(int64 [M, 1] aligned tokens, new level-0 offsets); one -1 when all were removed."""
    if not (_ENABLED and x.is_cuda):
        return None
    n = len(offsets) - 1
    if n <= 0:
        return None
    dev = x.device
    xi = x.reshape(-1).to(torch.int64).contiguous()
    if xi.numel() == 0:
        return None
    out = torch.empty_like(xi)
    counts = torch.empty(n, dtype=torch.int32, device=dev)
    off = _i32(offsets, dev)
    N.call("pa_ctc_align", N.ptr(xi), N.ptr(off), n, int(blank), int(merge_repeated), N.ptr(out),
           N.ptr(counts), N.stream())
    cnt = counts.cpu().tolist()
    if sum(cnt) == 0:
        return torch.full((1, 1), -1, dtype=torch.int64, device=dev), [0, 1]
    idx = torch.cat([torch.arange(s, s + c) for s, c in zip(offsets[:-1], cnt)]).to(dev)
    new_off = np.concatenate([[0], np.cumsum(cnt)]).astype(int).tolist()
    return out.index_select(0, idx).reshape(-1, 1), new_off


def mean_iou_hist(pred, label, num_classes):
    """(correct int32 [C], wrong int32 [C]) class histograms of mean_iou_op.cu."""
    if not (_ENABLED and pred.is_cuda):
        return None
    p, l = pred.reshape(-1).contiguous(), label.reshape(-1).contiguous()
    if p.dtype not in (torch.int32, torch.int64) or l.dtype != p.dtype or p.numel() != l.numel():
        return None
    correct = torch.zeros(num_classes, dtype=torch.int32, device=p.device)
    wrong = torch.zeros(num_classes, dtype=torch.int32, device=p.device)
    N.call("pa_mean_iou_hist", N.ptr(p), N.ptr(l), p.numel(), int(num_classes), int(p.dtype == torch.int64),
           N.ptr(correct), N.ptr(wrong), N.stream())
    return correct, wrong


def fake_quant_op(x, bit_length=8, in_scale=None, use_in_scale=False, clip=False):
    """(round(x / s * (2^(b-1) - 1)), s): s = |x|max (abs_max), max(|x|max, in_scale)
    (range_abs_max training, with clip) or in_scale (is_test)."""
    if not (_ENABLED and x.is_cuda and x.dtype == torch.float32):
        return None
    xc = x.contiguous()
    amax = torch.zeros(1, dtype=torch.int32, device=x.device)
    out = torch.empty_like(xc)
    s = torch.empty(1, dtype=torch.float32, device=x.device)
    ins = in_scale.reshape(1).float().contiguous() if in_scale is not None else None
    N.call("pa_fake_quant", N.ptr(xc), xc.numel(), int(bit_length), N.ptr(ins), int(use_in_scale), int(clip),
           N.ptr(amax), N.ptr(out), N.ptr(s), N.stream())
    return out, s


def isfinite_op(x, bad=None):
    """bool [1]: every element finite.  With ``bad`` (int32 [1] on the device) the
    check only ORs into that flag (no host sync), so a caller can test many tensors and
    read one flag; returns False when the kernel does not cover ``x``."""
    if not _ok(x):
        return None if bad is None else False
    xc = x.contiguous()
    flag = torch.zeros(1, dtype=torch.int32, device=x.device) if bad is None else bad
    N.call("pa_isfinite", N.ptr(xc), xc.numel(), _DT[x.dtype], N.ptr(flag), N.stream())
    return (flag == 0) if bad is None else True


def seq_pad_op(x, offsets, maxlen, pad_value):
    """LoD rows [T_total, ...] -> [N, maxlen, ...]; pad_value scalar or one row."""
    if not _ok(x) or x.dim() < 1:
        return None
    n = len(offsets) - 1
    xc = x.contiguous()
    D = xc.numel() // max(xc.shape[0], 1) if xc.shape[0] else int(np.prod(xc.shape[1:]))
    pv = torch.as_tensor(pad_value, dtype=x.dtype).reshape(-1).to(x.device).contiguous()
    if pv.numel() not in (1, D):
        return None
    out = torch.empty((n, maxlen) + tuple(xc.shape[1:]), dtype=x.dtype, device=x.device)
    off = _i32(offsets, x.device)
    N.call("pa_seq_pad", N.ptr(xc), N.ptr(off), n, int(maxlen), D, N.ptr(pv), pv.numel(),
           xc.element_size(), N.ptr(out), N.stream())
    return out


def seq_unpad_op(p, offsets):
    """[N, maxlen, ...] -> LoD rows [T_total, ...]."""
    if not _ok(p) or p.dim() < 2:
        return None
    n, maxlen = p.shape[0], p.shape[1]
    pc = p.contiguous()
    D = int(np.prod(pc.shape[2:])) if pc.dim() > 2 else 1
    rows = offsets[-1]
    out = torch.empty((rows,) + tuple(pc.shape[2:]), dtype=p.dtype, device=p.device)
    off = _i32(offsets, p.device)
    N.call("pa_seq_unpad", N.ptr(pc), N.ptr(off), n, maxlen, D, rows, pc.element_size(),
           N.ptr(out), N.stream())
    return out


def seq_scale_op(x, offsets, scales):
    """x[row] * scales[sequence(row)] (sequence_scale.cu), returned as a new tensor."""
    if not _ok(x):
        return None
    out = x.contiguous().clone()
    n = len(offsets) - 1
    D = out.numel() // max(out.shape[0], 1)
    sc = torch.as_tensor(scales, dtype=torch.float32).reshape(-1).to(x.device).contiguous()
    off = _i32(offsets, x.device)
    N.call("pa_seq_scale", N.ptr(out), N.ptr(off), n, D, out.shape[0], N.ptr(sc), _DT[x.dtype],
           N.stream())
    return out


# ------------------------------------------------------------------ optimizers (optim_ext.hip)


def opt_update_(kind, p, g, states, lr, **h):
    """In-place fp32 update of ``p`` and its ``states`` (list; ``None`` entries are
    optional states such as RMSProp's MeanGrad).  ``kind``: adamax (h: bp1, b1, b2,
    eps), decayed_adagrad (decay, eps), adadelta (rho, eps), rmsprop (rho, mu, eps),
    ftrl (l1, l2, lr_power), proximal (l1, l2), lars (mu, coeff, wd).  Returns None
    when the kernel does not cover the tensors (then the caller runs its torch path)."""
    ts = [p, g] + [s for s in states if s is not None]
    if not (_ENABLED and all(t.is_cuda and t.dtype == torch.float32 for t in ts)):
        return None
    if not (p.is_contiguous() and all(s is None or s.is_contiguous() for s in states)):
        return None
    n = p.numel()
    if any(t.numel() != n for t in ts):
        return None
    g = g.contiguous()
    lr_t = _lr(lr, p.device).reshape(-1)[:1].contiguous() if lr is not None else None
    st = [N.ptr(s) for s in states]
    if kind == "adamax":
        bp1 = _lr(h["bp1"], p.device).reshape(-1)[:1].contiguous()
        N.call("pa_opt_adamax", N.ptr(p), N.ptr(g), *st, N.ptr(lr_t), N.ptr(bp1), h["b1"], h["b2"], h["eps"], n,
               N.stream())
    elif kind == "decayed_adagrad":
        N.call("pa_opt_decayed_adagrad", N.ptr(p), N.ptr(g), *st, N.ptr(lr_t), h["decay"], h["eps"], n, N.stream())
    elif kind == "adadelta":
        N.call("pa_opt_adadelta", N.ptr(p), N.ptr(g), *st, h["rho"], h["eps"], n, N.stream())
    elif kind == "rmsprop":
        N.call("pa_opt_rmsprop", N.ptr(p), N.ptr(g), *st, N.ptr(lr_t), h["rho"], h["mu"], h["eps"], n, N.stream())
    elif kind == "ftrl":
        N.call("pa_opt_ftrl", N.ptr(p), N.ptr(g), *st, N.ptr(lr_t), h["l1"], h["l2"], h["lr_power"], n, N.stream())
    elif kind == "proximal":
        m = st[0] if st else None  # proximal_gd has no Moment
        N.call("pa_opt_proximal", N.ptr(p), N.ptr(g), m, N.ptr(lr_t), h["l1"], h["l2"], n, N.stream())
    elif kind == "lars":
        acc = torch.zeros(2, dtype=torch.float32, device=p.device)
        N.call("pa_opt_lars", N.ptr(p), N.ptr(g), *st, N.ptr(lr_t), N.ptr(acc), h["mu"], h["coeff"], h["wd"], n,
               N.stream())
    else:
        raise ValueError(kind)
    return p


# ------------------------------------------------------------------ fused_elemwise_activation (fused_ew.hip)


class _FusedEwActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, mode, bop, uop, scale, post, want_inter):
        x, y = x.contiguous(), y.contiguous()
        out = torch.empty_like(x)
        inter = torch.empty_like(x) if want_inter else None
        N.call("pa_fused_ew_act", _DT[x.dtype], mode, bop, uop, float(scale), N.ptr(x), N.ptr(y), N.ptr(out),
               N.ptr(inter), x.numel(), y.numel(), post, N.stream())
        ctx.save_for_backward(x, y)
        ctx.conf = (mode, bop, uop, float(scale), post)
        if inter is not None:
            ctx.mark_non_differentiable(inter)
        return out, inter

    @staticmethod
    def backward(ctx, dout, _dinter):
        x, y = ctx.saved_tensors
        mode, bop, uop, scale, post = ctx.conf
        dout = dout.contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dyf = torch.empty(x.shape, dtype=torch.float32, device=x.device) if ctx.needs_input_grad[1] else None
        N.call("pa_fused_ew_act_bwd", _DT[x.dtype], mode, bop, uop, scale, N.ptr(x), N.ptr(y), N.ptr(dout),
               N.ptr(dx), N.ptr(dyf), x.numel(), y.numel(), post, N.stream())
        dy = None
        if dyf is not None:
            ny = y.numel()
            dy = dyf.view(-1, ny, post).sum((0, 2)) if dyf.numel() != ny else dyf.view(-1)
            dy = dy.reshape(y.shape).to(y.dtype)
        return dx, dy, None, None, None, None, None, None


def fused_ew_act(x, y, functors, axis=-1, scale=0.0, want_inter=False):
    """(Out, IntermediateOut or None) of fused_elemwise_activation for
    functors in {elementwise_add, elementwise_mul} x {relu, scale}; None if uncovered."""
    f0, f1 = functors
    bops = {"elementwise_add": 0, "elementwise_mul": 1}
    uops = {"relu": 0, "scale": 1}
    if f0 in bops and f1 in uops:
        mode, bop, uop = 0, bops[f0], uops[f1]
    elif f0 in uops and f1 in bops:
        mode, bop, uop = 1, bops[f1], uops[f0]
    else:
        return None
    if not _ok(x, y) or x.dtype != y.dtype or y.numel() == 0:
        return None
    if tuple(y.shape) == tuple(x.shape):
        post = 1
        yv = y
    else:
        ax = axis if axis >= 0 else x.dim() - y.dim()
        ys = list(y.shape)
        while ys and ys[-1] == 1 and len(ys) > 1:  # trailing 1s (Paddle trims them)
            ys.pop()
        if ax < 0 or ax + len(ys) > x.dim() or list(x.shape[ax:ax + len(ys)]) != ys:
            return None
        post = int(np.prod(x.shape[ax + len(ys):])) if ax + len(ys) < x.dim() else 1
        yv = y
    return _tape.apply(_FusedEwActFn, x, yv, mode, bop, uop, scale, post, bool(want_inter))


# ------------------------------------------------------------------ detection (detect.hip)


def _f32c(t):
    return t.float().contiguous()


def iou_matrix_op(a, b, normalized=True):
    """[Na, Nb] IoU of box sets a [Na, 4], b [Nb, 4] (iou_similarity_op.h)."""
    if not (_ENABLED and a.is_cuda and b.is_cuda and a.dim() == 2 and b.dim() == 2):
        return None
    a, b = _f32c(a), _f32c(b)
    out = torch.empty(a.shape[0], b.shape[0], dtype=torch.float32, device=a.device)
    N.call("pa_iou_matrix", N.ptr(a), N.ptr(b), a.shape[0], b.shape[0], int(normalized), N.ptr(out), N.stream())
    return out


def box_coder_op(decode, prior, var, target, normalized=True):
    """encode_center_size: target [N, 4] -> [N, M, 4]; decode_center_size: target
    [N, M, 4] (or [N, 4] as [N, 1, 4] against M == 1 ...) -> boxes [N, M, 4]."""
    if not (_ENABLED and prior.is_cuda and target.is_cuda):
        return None
    pr = _f32c(prior)
    M = pr.shape[0]
    v = _f32c(var) if var is not None else None
    if v is not None and v.numel() != M * 4:
        return None
    t = _f32c(target)
    if decode:
        if t.dim() == 2:
            t = t.unsqueeze(1)
        if t.dim() != 3 or t.shape[1] != M:
            return None
        n = t.shape[0]
    else:
        if t.dim() != 2:
            return None
        n = t.shape[0]
    out = torch.empty(n, M, 4, dtype=torch.float32, device=t.device)
    N.call("pa_box_coder", int(decode), N.ptr(pr), N.ptr(v), N.ptr(t), n, M, int(normalized), N.ptr(out), N.stream())
    return out


def multiclass_nms_op(boxes, scores, background, score_thr, nms_top_k, nms_thr, keep_top_k, normalized=True):
    """(rows [R, 6] = (label, score, x1, y1, x2, y2), level-0 offsets) of
    multiclass_nms_op.cc for boxes [N, M, 4], scores [N, C, M]; per-class greedy NMS
    on the device (bitmask kernel).  None when uncovered (top-K > 512)."""
    if not (_ENABLED and boxes.is_cuda and scores.is_cuda and boxes.dim() == 3 and scores.dim() == 3):
        return None
    Nn, C, M = scores.shape
    K = M if nms_top_k is None or nms_top_k < 0 else min(int(nms_top_k), M)
    if K <= 0 or K > 512 or boxes.shape[1] != M:
        return None
    dev = scores.device
    s = scores.float()
    valid = s > score_thr
    masked = torch.where(valid, s, torch.full_like(s, -float("inf")))
    ss, order = torch.sort(masked, dim=-1, descending=True, stable=True)
    ss, order = ss[..., :K].contiguous(), order[..., :K].to(torch.int32).contiguous()
    count = valid.sum(-1).clamp(max=K).to(torch.int32)
    if 0 <= background < C:
        count[:, background] = 0
    count = count.contiguous()
    keep = torch.empty(Nn, C, K, dtype=torch.uint8, device=dev)
    bx = _f32c(boxes)
    N.call("pa_nms_bitmask", N.ptr(bx), N.ptr(order), N.ptr(count), Nn * C, C, M, K, float(nms_thr), int(normalized),
           N.ptr(keep), N.stream())
    kept = keep.bool()
    flat = torch.where(kept, ss, torch.full_like(ss, -float("inf"))).reshape(Nn, C * K)
    fs, fi = torch.sort(flat, dim=-1, descending=True, stable=True)  # class-major, then score: as the host loop
    nkeep = kept.reshape(Nn, -1).sum(-1)
    if keep_top_k is not None and keep_top_k > -1:
        nkeep = nkeep.clamp(max=int(keep_top_k))
    T = int(nkeep.max().item()) if Nn else 0
    counts = nkeep.cpu().tolist()
    if T == 0:
        return torch.full((1, 6), -1.0, dtype=torch.float32, device=dev), [0, 1]
    fs, fi = fs[:, :T], fi[:, :T]
    cls = (fi // K).float()
    bidx = order.reshape(Nn, C * K).gather(1, fi).long()
    bsel = bx.gather(1, bidx.unsqueeze(-1).expand(Nn, T, 4))
    rows = torch.cat([cls.unsqueeze(-1), fs.unsqueeze(-1), bsel], -1)  # [N, T, 6]
    sel = torch.arange(T, device=dev).unsqueeze(0) < torch.as_tensor(counts, device=dev).unsqueeze(1)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(int).tolist()
    return rows[sel], off


# ------------------------------------------------------------------ box generators / target_assign (detect.hip)


def _farr(vals):
    import ctypes

    return (ctypes.c_float * len(vals))(*[float(v) for v in vals])


def prior_box_op(feat, H, W, IH, IW, sizes, variances, step_w, step_h, offset, clip):
    """boxes, variances [H, W, P, 4] (fp32) from the per-prior (w, h) list, or None."""
    if not (_ENABLED and feat.is_cuda) or not sizes:
        return None
    dev = feat.device
    bw = torch.tensor([s[0] for s in sizes], dtype=torch.float32, device=dev)
    bh = torch.tensor([s[1] for s in sizes], dtype=torch.float32, device=dev)
    P = len(sizes)
    boxes = torch.empty(H, W, P, 4, dtype=torch.float32, device=dev)
    var = torch.empty_like(boxes)
    N.call("pa_prior_box", N.ptr(bw), N.ptr(bh), N.ptr(boxes), N.ptr(var), H, W, P, float(IW), float(IH),
           float(step_w), float(step_h), float(offset), int(bool(clip)), _farr(variances), N.stream())
    return boxes, var


def anchor_generator_op(feat, H, W, ws, hs, variances, sw, sh, offset):
    if not (_ENABLED and feat.is_cuda) or not ws:
        return None
    dev = feat.device
    aw = torch.tensor(ws, dtype=torch.float32, device=dev)
    ah = torch.tensor(hs, dtype=torch.float32, device=dev)
    anchors = torch.empty(H, W, len(ws), 4, dtype=torch.float32, device=dev)
    var = torch.empty_like(anchors)
    N.call("pa_anchor_generator", N.ptr(aw), N.ptr(ah), N.ptr(anchors), N.ptr(var), H, W, len(ws), float(sw),
           float(sh), float(offset), _farr(variances), N.stream())
    return anchors, var


def polygon_box_transform_op(x):
    if not (_ENABLED and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4):
        return None
    x = x.contiguous()
    y = torch.empty_like(x)
    Nn, C, H, W = x.shape
    N.call("pa_polygon_box_transform", N.ptr(x), N.ptr(y), Nn * C, C, H, W, N.stream())
    return y


def target_assign_op(x, xoff, match, neg=None, neg_off=None, mismatch=0.0):
    """x [R, Pw, K] rows of all images (LoD offsets ``xoff``), match [N, P] int64 ->
    (out [N, P, K], weight [N, P, 1]), or None."""
    if not (_ENABLED and x.is_cuda and x.dtype == torch.float32):
        return None
    dev = x.device
    Nn, P = match.shape
    xs = x.reshape(x.shape[0], -1, x.shape[-1]).contiguous()
    Pw, K = xs.shape[1], xs.shape[2]
    xo = torch.tensor(list(xoff), dtype=torch.int32, device=dev)
    m = match.to(torch.int64).contiguous()
    out = torch.empty(Nn, P, K, dtype=torch.float32, device=dev)
    wt = torch.empty(Nn, P, 1, dtype=torch.float32, device=dev)
    nneg = 0
    ng = ni = None
    if neg is not None:
        ng = neg.reshape(-1).to(torch.int64).contiguous()
        nneg = ng.numel()
        img = [b for b in range(len(neg_off) - 1) for _ in range(neg_off[b + 1] - neg_off[b])]
        ni = torch.tensor(img, dtype=torch.int32, device=dev)
    N.call("pa_target_assign", N.ptr(xs), N.ptr(xo), N.ptr(m), N.ptr(ng), N.ptr(ni), N.ptr(out), N.ptr(wt), Nn, P,
           Pw, K, nneg, float(mismatch), N.stream())
    return out, wt
