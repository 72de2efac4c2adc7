"""Autograd wrappers of ``csrc/kernels/nnmisc.hip``: cos_sim, bilinear / nearest
interpolation, conv_shift and lstm_unit on the device (forward + hand-written
backward kernels).  Each returns None when the inputs are not eligible (CPU,
unsupported dtype) so the Fluid operator falls back to its host expression.

Reference: operators/cos_sim_op.h, math/cos_sim_functor.cu, bilinear_interp_op.cu,
conv_shift_op.cu, lstm_unit_op.cu.
"""
from __future__ import annotations

import os

import torch

from . import _native as N
from ..autograd import tape as _tape

_ENABLED = os.environ.get("PADDLE_AMD_OPLIB", "1") != "0"
_DT = {torch.float32: 0, torch.bfloat16: 1}


def _ok(*ts):
    return _ENABLED and all(t is not None and t.is_cuda and t.dtype in _DT for t in ts)


class _CosSimFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y):
        x2, y2 = x.reshape(x.shape[0], -1).contiguous(), y.reshape(y.shape[0], -1).contiguous()
        rows, D = x2.shape
        yr = y2.shape[0]
        out = torch.empty(rows, 1, dtype=x.dtype, device=x.device)
        xn = torch.empty(rows, 1, dtype=torch.float32, device=x.device)
        yn = torch.empty(rows, 1, dtype=torch.float32, device=x.device)
        N.call("pa_cos_sim", _DT[x.dtype], N.ptr(x2), N.ptr(y2), N.ptr(out), N.ptr(xn), N.ptr(yn), rows, D, yr,
               N.stream())
        ctx.save_for_backward(x2, y2, out, xn, yn)
        ctx.shapes = (x.shape, y.shape)
        ctx.mark_non_differentiable(xn, yn)
        return out, xn, yn

    @staticmethod
    def backward(ctx, dout, _dxn, _dyn):
        x2, y2, out, xn, yn = ctx.saved_tensors
        xs, ys = ctx.shapes
        rows, D = x2.shape
        yr = y2.shape[0]
        d = dout.contiguous().to(x2.dtype)
        dx = torch.empty_like(x2) if ctx.needs_input_grad[0] else None
        dy = (torch.zeros(y2.shape, dtype=torch.float32, device=x2.device) if ctx.needs_input_grad[1] else None)
        N.call("pa_cos_sim_bwd", _DT[x2.dtype], N.ptr(x2), N.ptr(y2), N.ptr(out), N.ptr(xn), N.ptr(yn), N.ptr(d),
               N.ptr(dx), N.ptr(dy), rows, D, yr, N.stream())
        return (dx.reshape(xs) if dx is not None else None,
                dy.to(y2.dtype).reshape(ys) if dy is not None else None)


def cos_sim(x, y):
    """-> (out [rows, 1], |x| [rows, 1], |y| [rows, 1]) or None."""
    if not _ok(x, y) or x.dtype != y.dtype or x.shape[0] == 0:
        return None
    if y.shape[0] not in (1, x.shape[0]) or x[0].numel() != y[0].numel():
        return None
    return _tape.apply(_CosSimFn, x, y)


class _InterpFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow, nearest, align):
        x = x.contiguous()
        Nn, C, H, W = x.shape
        y = torch.empty(Nn, C, oh, ow, dtype=x.dtype, device=x.device)
        N.call("pa_interp", _DT[x.dtype], 0, N.ptr(x), N.ptr(y), Nn * C, H, W, oh, ow, int(nearest), int(align),
               N.stream())
        ctx.conf = (x.shape, x.dtype, oh, ow, int(nearest), int(align))
        return y

    @staticmethod
    def backward(ctx, dy):
        (Nn, C, H, W), dt, oh, ow, nearest, align = ctx.conf
        d = dy.contiguous().to(dt)
        dx = torch.zeros(Nn, C, H, W, dtype=torch.float32, device=dy.device)
        N.call("pa_interp", _DT[dt], 1, N.ptr(d), N.ptr(dx), Nn * C, H, W, oh, ow, nearest, align, N.stream())
        return dx.to(dt), None, None, None, None


def interpolate(x, oh, ow, mode="bilinear", align_corners=True):
    if not _ok(x) or x.dim() != 4 or oh <= 0 or ow <= 0 or mode not in ("bilinear", "nearest"):
        return None
    return _tape.apply(_InterpFn, x, int(oh), int(ow), mode == "nearest", bool(align_corners))


class _ConvShiftFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y):
        x, y = x.contiguous(), y.contiguous()
        B, M = x.shape
        Nn = y.shape[1]
        out = torch.empty_like(x)
        N.call("pa_conv_shift", _DT[x.dtype], N.ptr(x), N.ptr(y), None, N.ptr(out), None, None, B, M, Nn, N.stream())
        ctx.save_for_backward(x, y)
        return out

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        B, M = x.shape
        Nn = y.shape[1]
        g = g.contiguous().to(x.dtype)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dy = torch.empty_like(y) if ctx.needs_input_grad[1] else None
        N.call("pa_conv_shift", _DT[x.dtype], N.ptr(x), N.ptr(y), N.ptr(g), None, N.ptr(dx), N.ptr(dy), B, M, Nn,
               N.stream())
        return dx, dy


def conv_shift(x, y):
    if not _ok(x, y) or x.dtype != y.dtype or x.dim() != 2 or y.dim() != 2 or x.shape[0] != y.shape[0]:
        return None
    if y.shape[1] > x.shape[1] or y.shape[1] % 2 == 0:
        return None
    return _tape.apply(_ConvShiftFn, x, y)


class _LstmUnitFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cp, fb):
        x, cp = x.contiguous(), cp.contiguous()
        B, D = cp.shape
        c, h = torch.empty_like(cp), torch.empty_like(cp)
        N.call("pa_lstm_unit", _DT[x.dtype], 0, N.ptr(x), N.ptr(cp), N.ptr(c), N.ptr(h), None, None, None, None, B, D,
               float(fb), N.stream())
        ctx.save_for_backward(x, cp, c)
        ctx.fb = float(fb)
        return c, h

    @staticmethod
    def backward(ctx, dc, dh):
        x, cp, c = ctx.saved_tensors
        B, D = cp.shape
        dcc = dc.contiguous().to(x.dtype) if dc is not None else None
        dhc = dh.contiguous().to(x.dtype) if dh is not None else None
        dx = torch.empty_like(x)
        dcp = torch.empty_like(cp)
        N.call("pa_lstm_unit", _DT[x.dtype], 1, N.ptr(x), N.ptr(cp), N.ptr(c), None, N.ptr(dcc), N.ptr(dhc), N.ptr(dx),
               N.ptr(dcp), B, D, ctx.fb, N.stream())
        return dx, dcp, None


def lstm_unit(x, c_prev, forget_bias=0.0):
    """-> (c, h) or None.  x [B, 4D] gates in (i, f, o, g) order."""
    if not _ok(x, c_prev) or x.dtype != c_prev.dtype or x.dim() != 2 or c_prev.dim() != 2:
        return None
    if x.shape[1] != 4 * c_prev.shape[1] or x.shape[0] != c_prev.shape[0]:
        return None
    return _tape.apply(_LstmUnitFn, x, c_prev, forget_bias)


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, label, soft, ignore):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        rows, D = x2.shape
        y = torch.empty(rows, 1, dtype=x.dtype, device=x.device)
        lab = label.reshape(-1).to(torch.int64).contiguous() if not soft else None
        sl = label.reshape(rows, D).to(x.dtype).contiguous() if soft else None
        N.call("pa_cross_entropy", _DT[x.dtype], 0, N.ptr(x2), N.ptr(lab), N.ptr(sl), None, N.ptr(y), rows, D,
               int(ignore), N.stream())
        ctx.save_for_backward(x2, lab if lab is not None else sl)
        ctx.conf = (soft, int(ignore), tuple(x.shape))
        return y.reshape(tuple(x.shape[:-1]) + (1,))

    @staticmethod
    def backward(ctx, dy):
        x2, lab = ctx.saved_tensors
        soft, ignore, shape = ctx.conf
        rows, D = x2.shape
        d = dy.reshape(rows).contiguous().to(x2.dtype)
        dx = torch.empty_like(x2)
        N.call("pa_cross_entropy", _DT[x2.dtype], 1, N.ptr(x2), None if soft else N.ptr(lab),
               N.ptr(lab) if soft else None, N.ptr(d), N.ptr(dx), rows, D, ignore, N.stream())
        return dx.reshape(shape), None, None, None


def cross_entropy(x, label, soft_label=False, ignore_index=-100):
    """-log(x[label]) / -sum(label * log x) over the last axis of a probability tensor, or None."""
    if not _ok(x) or not label.is_cuda or x.dim() < 1 or x.shape[-1] == 0:
        return None
    if soft_label and label.shape != x.shape:
        return None
    if not soft_label and label.numel() != x.numel() // x.shape[-1]:
        return None
    return _tape.apply(_XentFn, x, label, bool(soft_label), int(ignore_index))
