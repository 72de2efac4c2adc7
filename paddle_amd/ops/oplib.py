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

from . import _native as N

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
    N.call("pa_mask_mul", _DT[d.dtype], N.ptr(d), N.ptr(mask.contiguous()), N.ptr(out), d.numel(), float(scale),
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
    N.call("pa_sgd", _DT[p.dtype], N.ptr(p), N.ptr(g.contiguous()), N.ptr(_lr(lr, p.device)), p.numel(), N.stream())
    return p


def sgd_sparse_(p, rows, values, lr):
    """Param[rows] -= lr * values (duplicate rows accumulate)."""
    if not (_ok(p, values) and p.dtype == torch.float32 and values.dtype == torch.float32 and p.is_contiguous()):
        return None
    rows = torch.as_tensor(rows, dtype=torch.int64).to(p.device)
    D = p.numel() // p.shape[0]
    N.call("pa_sgd_sparse", N.ptr(p), N.ptr(rows), N.ptr(values.contiguous()), N.ptr(_lr(lr, p.device)),
           rows.numel(), D, N.stream())
    return p


def adagrad_(p, g, m, lr, eps):
    if not (_ok(p, g, m) and p.dtype == g.dtype == m.dtype == torch.float32 and p.is_contiguous()
            and m.is_contiguous()):
        return None
    N.call("pa_adagrad", N.ptr(p), N.ptr(g.contiguous()), N.ptr(m), N.ptr(_lr(lr, p.device)), p.numel(), float(eps),
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
    off = torch.as_tensor(np.asarray(offsets, dtype=np.int32)).to(x.device)
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
    off = torch.as_tensor(np.asarray(offsets, dtype=np.int32)).to(dout.device)
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
    u, r, rh = _GruGateFn.apply(ur, h)
    hn, c = _GruOutFn.apply(g[:, 2 * D:] + rh @ W[:, 2 * D:], u, h)
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
        return _BinaryFn.apply(op, x, y)
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
        return _ReduceFn.apply(op, x, list(dims), keep_dim)
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
    return _TopkFn.apply(x, k)


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
    return _SeqPoolFn.apply(x, list(offsets), pooltype)


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
    return _GatherRowsFn.apply(src, idx, float(fill))


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
    return _DropoutFn.apply(x, float(p), seed, bool(upscale))
