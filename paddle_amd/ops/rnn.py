"""Persistent-kernel LSTM (``csrc/kernels/rnn.hip``) with autograd.

One launch runs all T recurrent steps (W_hh resident in VGPRs across the grid,
hidden state exchanged through a grid barrier); the input projection, dW_ih,
dW_hh, db and dx are single large GEMMs outside the recurrence.  Variable
lengths (LoD / packed sequences) freeze (h, c) past each sequence's end, so
``hs[T-1]`` holds every sequence's last state.

Reference behaviour: operators/lstm_op.h (LoD batch LSTM), the gate math of
operators/math/detail/lstm_kernel.h; gate order here is torch's (i, f, g, o).
"""
from __future__ import annotations

import torch

from . import _native as N

_SUPPORTED_H = (128, 256, 512, 1024)


def persistent_ok(x, H, B):
    return x.is_cuda and H in _SUPPORTED_H and 1 <= B <= 128


def _bp(B):
    # padded batch rows of the kernel's exchange buffers (row tiles of 16: 1, 2, 4, 8)
    return 16 if B <= 16 else 32 if B <= 32 else 64 if B <= 64 else 128


def _lens_dev(lens, T, B, device):
    if lens is None:
        return torch.full((B,), T, dtype=torch.int32, device=device)
    return lens.to(device=device, dtype=torch.int32).contiguous()


class _LstmFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lens, w_ih, w_hh, b, h0, c0):
        T, B, I = x.shape
        H = w_hh.shape[0]
        dev = x.device
        x2 = x.reshape(T * B, I)
        xp = torch.matmul(x2, w_ih.to(x2.dtype)).float()
        if b is not None:
            xp = xp + b.float()
        xp = xp.contiguous()
        whh = w_hh.detach().to(torch.bfloat16).contiguous()
        BP = _bp(B)
        hbuf = torch.zeros(2, BP, H, dtype=torch.bfloat16, device=dev)
        if h0 is not None:
            hbuf[0, :B] = h0.to(torch.bfloat16)
        hs = torch.empty(T, B, H, dtype=torch.float32, device=dev)
        cs = torch.empty_like(hs)
        gates = torch.empty(T, B, 4 * H, dtype=torch.bfloat16, device=dev)
        ws = torch.zeros(32, dtype=torch.int32, device=dev)
        h0f = h0.float().contiguous() if h0 is not None else None
        c0f = c0.float().contiguous() if c0 is not None else None
        N.call("pa_lstm_persistent", 0, N.ptr(xp), N.ptr(whh), N.ptr(lens), N.ptr(hbuf), N.ptr(hs), N.ptr(cs),
               N.ptr(gates), N.ptr(h0f), N.ptr(c0f), None, None, None, None, None, None, N.ptr(ws), T, B, H,
               N.stream())
        ctx.save_for_backward(x, lens, w_ih, whh, hs, cs, gates, h0f, c0f)
        ctx.flags = (b is not None, h0 is not None, c0 is not None, x.dtype, w_ih.dtype)
        ctx.ws = ws
        return hs.to(x.dtype), hs[-1].clone().to(x.dtype), cs[-1].clone().to(x.dtype)

    @staticmethod
    def backward(ctx, dhs, dh_last, dc_last):
        x, lens, w_ih, whh, hs, cs, gates, h0f, c0f = ctx.saved_tensors
        has_b, has_h0, has_c0, xdt, wdt = ctx.flags
        T, B, I = x.shape
        H = whh.shape[0]
        dev = x.device
        BP = _bp(B)
        dgates = torch.empty(T, BP, 4 * H, dtype=torch.bfloat16, device=dev)
        dh0 = torch.empty(B, H, dtype=torch.float32, device=dev)
        dc0 = torch.empty_like(dh0)
        f = lambda t: t.float().contiguous() if t is not None else None  # noqa: E731
        N.call("pa_lstm_persistent", 1, None, N.ptr(whh), N.ptr(lens), None, N.ptr(hs), N.ptr(cs), N.ptr(gates),
               N.ptr(h0f), N.ptr(c0f), N.ptr(f(dhs)), N.ptr(f(dh_last)), N.ptr(f(dc_last)), N.ptr(dgates),
               N.ptr(dh0), N.ptr(dc0), N.ptr(ctx.ws), T, B, H, N.stream())
        dG = dgates[:, :B].reshape(T * B, 4 * H)
        hprev = torch.empty(T, B, H, dtype=torch.bfloat16, device=dev)
        hprev[0] = h0f.to(torch.bfloat16) if h0f is not None else 0
        hprev[1:] = hs[:-1].to(torch.bfloat16)
        hp2 = hprev.reshape(T * B, H)
        dw_hh = (torch.matmul(hp2.t().float(), dG.float()) if wdt == torch.float32 else torch.matmul(hp2.t(), dG))
        x2 = x.reshape(T * B, I)
        dGx = dG.to(x2.dtype)
        dx = torch.matmul(dGx, w_ih.to(x2.dtype).t()).view(T, B, I) if ctx.needs_input_grad[0] else None
        dw_ih = torch.matmul(x2.t(), dGx).to(wdt) if ctx.needs_input_grad[2] else None
        db = dG.float().sum(0) if has_b else None
        return (dx, None, dw_ih, dw_hh.to(wdt), db, dh0.to(xdt) if has_h0 else None,
                dc0.to(xdt) if has_c0 else None)


def lstm(x, w_ih, w_hh, b=None, h0=None, c0=None, lens=None, time_major=True):
    """Single-layer unidirectional LSTM.

    x [T, B, I] (or [B, T, I] with ``time_major=False``), w_ih [I, 4H], w_hh [H, 4H],
    b [4H] (= b_ih + b_hh), gate order (i, f, g, o); ``lens`` [B] valid lengths.
    Returns (hs [T, B, H] (batch-major if input was), h_last [B, H], c_last [B, H]);
    past a sequence's end its (h, c) stay frozen, so h_last is its final state.
    """
    if not time_major:
        x = x.transpose(0, 1)
    T, B, _ = x.shape
    H = w_hh.shape[0]
    if not persistent_ok(x, H, B):
        hs, h, c = _lstm_ref(x, w_ih, w_hh, b, h0, c0, lens)
    else:
        hs, h, c = _LstmFn.apply(x.contiguous(), _lens_dev(lens, T, B, x.device), w_ih, w_hh, b, h0, c0)
    if not time_major:
        hs = hs.transpose(0, 1)
    return hs, h, c


def _lstm_ref(x, w_ih, w_hh, b=None, h0=None, c0=None, lens=None):
    """Plain PyTorch recurrence with the same length-freezing semantics (CPU path
    and numerics reference)."""
    T, B, _ = x.shape
    H = w_hh.shape[0]
    dt = x.dtype
    h = h0.to(dt) if h0 is not None else x.new_zeros(B, H)
    c = c0.to(dt) if c0 is not None else x.new_zeros(B, H)
    xp = x.reshape(T * B, -1) @ w_ih.to(dt)
    if b is not None:
        xp = xp + b.to(dt)
    xp = xp.view(T, B, 4 * H)
    L = lens.to(x.device) if lens is not None else None
    out = []
    for t in range(T):
        g = xp[t] + h @ w_hh.to(dt)
        i, f, gg, o = g.chunk(4, 1)
        cn = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        hn = torch.sigmoid(o) * torch.tanh(cn)
        if L is not None:
            m = (t < L).to(dt).unsqueeze(1)
            cn = m * cn + (1 - m) * c
            hn = m * hn + (1 - m) * h
        h, c = hn, cn
        out.append(h)
    return torch.stack(out), h, c


def reverse_padded(x, lens, time_major=True):
    """Reverse every sequence within its own length (for the backward direction)."""
    if lens is None:
        return x.flip(0 if time_major else 1)
    xt = x if time_major else x.transpose(0, 1)
    T, B = xt.shape[:2]
    t = torch.arange(T, device=x.device).unsqueeze(1)
    L = lens.to(x.device).long().unsqueeze(0)
    idx = torch.where(t < L, L - 1 - t, t)                       # [T, B]
    out = xt.gather(0, idx.view(T, B, *([1] * (xt.dim() - 2))).expand_as(xt))
    return out if time_major else out.transpose(0, 1)
