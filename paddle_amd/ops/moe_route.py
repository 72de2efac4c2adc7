"""MoE token dispatch / combine (csrc/kernels/moe.hip) as autograd functions.

``routing(flat_e, T, k, keep)`` turns the gate's expert choice per (token, slot)
into the expert-sorted order of the kept slots: ``src`` (token of each sorted
row), ``pos`` (sorted row of each slot, -1 if dropped) and the sorted experts.
``dispatch`` gathers token rows into that order; ``combine`` sums each token's k
expert outputs weighted by the gate.  Both backward passes are gathers over
``pos`` -- no atomics, no sort-based ``index_put`` -- and the combine backward
produces the gate-weight gradient in the same pass.  CPU tensors take the
equivalent torch indexing path.
"""
from __future__ import annotations

import torch

from . import _native as N
from ..autograd import tape as _tape


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def routing(flat_e, T, k, keep=None):
    """-> (slot_sorted [R] long, src [R] int32, pos [T*k] int32, e_sorted [R] long)."""
    if keep is None:
        slots = torch.argsort(flat_e, stable=True)
    else:
        sel = keep.nonzero().squeeze(-1)
        slots = sel[torch.argsort(flat_e[sel], stable=True)]
    R = slots.numel()
    pos = torch.full((T * k,), -1, dtype=torch.int32, device=flat_e.device)
    pos[slots] = torch.arange(R, dtype=torch.int32, device=flat_e.device)
    src = torch.div(slots, k, rounding_mode="floor").to(torch.int32)
    return slots, src, pos, flat_e[slots]


def _route_native_ok(flat_e, E):
    return flat_e.is_cuda and flat_e.dtype == torch.int64 and 0 < E <= 1024 and flat_e.numel() > 0


def _route_ws(n, E, device):
    """int32 workspace of pa_moe_route: per 1024-slot block the expert counts and
    running bases, plus the expert row offsets."""
    nb = (n + 1023) // 1024
    return torch.empty(2 * nb * E + E, dtype=torch.int32, device=device)


def _rank_in_expert(flat_e):
    """Rank of every slot among the slots of its expert, in slot order (torch path)."""
    order = torch.argsort(flat_e, stable=True)
    se = flat_e[order]
    first = torch.searchsorted(se, se, right=False)
    rank = torch.empty_like(order)
    rank[order] = torch.arange(se.numel(), device=flat_e.device) - first
    return rank


def route(flat_e, T, k, E, cap=None):
    """Expert-sorted layout of the kept slots -> (src [R] int32, pos [T*k] int32,
    e_sorted [R] int64, counts [E] int64).  ``cap``: keep only the first ``cap`` slots
    of each expert (slot order; rows stay compact).  On the GPU one workgroup of
    ``pa_moe_route`` (a stable counting sort: no argsort, no index_put, no
    histogram atomics on global memory); with ``cap`` the kept-row count is read back
    to size the outputs (the torch path syncs on it the same way)."""
    n = flat_e.numel()
    if _route_native_ok(flat_e, E):
        dev = flat_e.device
        flat_e = _c(flat_e)
        pos = torch.empty(n, dtype=torch.int32, device=dev)
        src = torch.empty(n, dtype=torch.int32, device=dev)
        e_sorted = torch.empty(n, dtype=torch.int64, device=dev)
        counts = torch.empty(E, dtype=torch.int64, device=dev)
        ws = _route_ws(n, E, dev)
        N.call("pa_moe_route", N.ptr(flat_e), n, E, k, 0 if cap is None else 2, -1 if cap is None else int(cap),
               N.ptr(pos), N.ptr(src), N.ptr(e_sorted), N.ptr(counts), N.ptr(ws), N.stream())
        if cap is not None:
            R = int(counts.sum())
            src, e_sorted = src[:R], e_sorted[:R]
        return src, pos, e_sorted, counts
    keep = None if cap is None else _rank_in_expert(flat_e) < cap
    _, src, pos, e_sorted = routing(flat_e, T, k, keep)
    counts = torch.zeros(E, dtype=torch.int64, device=flat_e.device).index_add_(0, e_sorted,
                                                                                torch.ones_like(e_sorted))
    return src, pos, e_sorted, counts


def _native_ok(x):
    return x.is_cuda and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0


class _DispatchFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, src, pos, k):
        x = _c(x)
        T, H = x.shape
        out = torch.empty(src.numel(), H, dtype=x.dtype, device=x.device)
        N.call("pa_moe_gather", N.ptr(x), N.ptr(src), N.ptr(out), src.numel(), H, N.stream())
        ctx.save_for_backward(pos)
        ctx.k, ctx.T = k, T
        return out

    @staticmethod
    def backward(ctx, ds):
        (pos,) = ctx.saved_tensors
        ds = _c(ds)
        dx = torch.empty(ctx.T, ds.shape[1], dtype=ds.dtype, device=ds.device)
        N.call("pa_moe_reduce", N.ptr(ds), N.ptr(pos), None, N.ptr(dx), ctx.T, ctx.k, ds.shape[1], N.stream())
        return dx, None, None, None


class _CombineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ys, w, pos, k, padded=False):
        ys = _c(ys)
        ctx.wshape = w.shape  # [T * k] or [T, k]
        w = _c(w.float())
        T, H = pos.numel() // k, ys.shape[1]
        y = torch.empty(T, H, dtype=ys.dtype, device=ys.device)
        N.call("pa_moe_reduce", N.ptr(ys), N.ptr(pos), N.ptr(w), N.ptr(y), T, k, H, N.stream())
        ctx.save_for_backward(ys, w, pos)
        ctx.k, ctx.padded = k, padded
        return y

    @staticmethod
    def backward(ctx, dy):
        ys, w, pos = ctx.saved_tensors
        dy = _c(dy)
        k, H = ctx.k, ys.shape[1]
        T = pos.numel() // k
        # padded (capacity) layouts have rows no slot references: their gradient is 0
        dys = torch.zeros_like(ys) if ctx.padded else torch.empty_like(ys)
        dw = torch.empty(T * k, dtype=torch.float32, device=dy.device)
        N.call("pa_moe_combine_bwd", N.ptr(dy), N.ptr(ys), N.ptr(pos), N.ptr(w), N.ptr(dys), N.ptr(dw), T, k, H,
               N.stream())
        return dys, dw.view(ctx.wshape), None, None, None


def dispatch(x, src, pos, k):
    """x [T, H] -> rows in sorted order [R, H]."""
    if _native_ok(x):
        return _tape.apply(_DispatchFn, x, src, pos, k)
    return _tape.apply(_DispatchRefFn, x, src, pos, k)


class _DispatchRefFn(torch.autograd.Function):
    """Host dispatch (row gather) with its scatter-add backward."""

    @staticmethod
    def forward(ctx, x, src, pos, k):
        ctx.save_for_backward(src)
        ctx.T = x.shape[0]
        return x[src.long()]

    @staticmethod
    def backward(ctx, g):
        (src,) = ctx.saved_tensors
        dx = torch.zeros(ctx.T, g.shape[1], dtype=g.dtype, device=g.device).index_add_(0, src.long(), g)
        return dx, None, None, None


def capacity_routing(flat_e, T, k, E, cap):
    """Fixed-capacity (GShard) layout, no host sync: slot s of expert e = flat_e[s]
    goes to row e * cap + (its rank among e's slots, in slot order) when that rank
    is below ``cap``, else it is dropped (pos = -1).  -> (src [E*cap] int32: token of
    each row, 0 for padding rows; pos [T*k] int32).  Kept slots match ``routing``
    with keep = rank < cap, in the same within-expert order."""
    dev = flat_e.device
    if _route_native_ok(flat_e, E):
        flat_e = _c(flat_e)
        pos = torch.empty(T * k, dtype=torch.int32, device=dev)
        src = torch.empty(E * cap, dtype=torch.int32, device=dev)  # the kernel zero-fills padding rows
        counts = torch.empty(E, dtype=torch.int64, device=dev)
        ws = _route_ws(T * k, E, dev)
        N.call("pa_moe_route", N.ptr(flat_e), T * k, E, k, 1, int(cap), N.ptr(pos), N.ptr(src), None, N.ptr(counts),
               N.ptr(ws), N.stream())
        return src, pos
    rank = _rank_in_expert(flat_e)
    keep = rank < cap
    row = flat_e * cap + rank
    pos = torch.where(keep, row, torch.full_like(row, -1)).to(torch.int32)
    src = torch.zeros(E * cap, dtype=torch.int32, device=dev)
    slots = torch.arange(T * k, device=dev)
    src.index_put_((row[keep],), torch.div(slots[keep], k, rounding_mode="floor").to(torch.int32))
    return src, pos


def combine(ys, w, pos, k, padded=False):
    """ys [R, H] (sorted order), w [T*k] gate weights -> y [T, H].  ``padded``: some
    rows of ys are referenced by no slot (capacity layout; their gradient is 0)."""
    if _native_ok(ys):
        return _tape.apply(_CombineFn, ys, w, pos, k, padded)
    return _tape.apply(_CombineRefFn, ys, w, pos, k)


class _CombineRefFn(torch.autograd.Function):
    """Host combine: y[t] = sum_j w[t, j] ys[pos[t, j]] (dropped slots: pos -1), with
    its backward (dys = scatter of w dy, dw = <dy, ys> per slot)."""

    @staticmethod
    def forward(ctx, ys, w, pos, k):
        T = pos.numel() // k
        wf = w.reshape(-1)
        keep = pos >= 0
        slots = keep.nonzero().squeeze(-1)
        rows = pos[slots].long()
        tok = torch.div(slots, k, rounding_mode="floor")
        y = torch.zeros(T, ys.shape[1], dtype=ys.dtype, device=ys.device)
        y.index_add_(0, tok, ys[rows] * wf[slots].unsqueeze(-1).to(ys.dtype))
        ctx.save_for_backward(ys, wf, slots, rows, tok)
        ctx.wshape = w.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        ys, wf, slots, rows, tok = ctx.saved_tensors
        dys = torch.zeros_like(ys)
        dys.index_add_(0, rows, dy[tok] * wf[slots].unsqueeze(-1).to(dy.dtype))
        dw = torch.zeros(wf.numel(), dtype=wf.dtype, device=wf.device)
        dw[slots] = (dy[tok].float() * ys[rows].float()).sum(-1).to(wf.dtype)
        return dys, dw.view(ctx.wshape), None, None
