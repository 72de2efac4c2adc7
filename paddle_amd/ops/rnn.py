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
from ..autograd import tape as _tape  # noqa: E402

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
        # w_ih None: x already holds the gate pre-activations (Fluid's lstm op input)
        xp = x2.float() if w_ih is None else torch.matmul(x2, w_ih.to(x2.dtype)).float()
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
        ws = torch.zeros(128, dtype=torch.int32, device=dev)  # err + per-row-block counters
        h0f = h0.float().contiguous() if h0 is not None else None
        c0f = c0.float().contiguous() if c0 is not None else None
        N.call("pa_lstm_persistent", 0, N.ptr(xp), N.ptr(whh), N.ptr(lens), N.ptr(hbuf), N.ptr(hs), N.ptr(cs),
               N.ptr(gates), N.ptr(h0f), N.ptr(c0f), None, None, None, None, None, None, None, N.ptr(ws), T, B,
               H, N.stream())
        ctx.save_for_backward(x, lens, w_ih, whh, hs, cs, gates, h0f, c0f)
        ctx.flags = (b is not None, h0 is not None, c0 is not None, x.dtype, w_ih.dtype if w_ih is not None else None)
        ctx.ws = ws
        return hs.to(x.dtype), hs[-1].clone().to(x.dtype), cs[-1].clone().to(x.dtype), cs.to(x.dtype)

    @staticmethod
    def backward(ctx, dhs, dh_last, dc_last, dcs):
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
        # keep the converted gradients referenced until the launch: a temporary freed
        # inside the argument list can be handed straight to the next conversion
        dhs_, dcs_, dhl_, dcl_ = f(dhs), f(dcs), f(dh_last), f(dc_last)
        N.call("pa_lstm_persistent", 1, None, N.ptr(whh), N.ptr(lens), None, N.ptr(hs), N.ptr(cs), N.ptr(gates),
               N.ptr(h0f), N.ptr(c0f), N.ptr(dhs_), N.ptr(dcs_), N.ptr(dhl_), N.ptr(dcl_), N.ptr(dgates),
               N.ptr(dh0), N.ptr(dc0), N.ptr(ctx.ws), T, B, H, N.stream())
        dG = dgates[:, :B].reshape(T * B, 4 * H)
        hprev = torch.empty(T, B, H, dtype=torch.bfloat16, device=dev)
        hprev[0] = h0f.to(torch.bfloat16) if h0f is not None else 0
        hprev[1:] = hs[:-1].to(torch.bfloat16)
        hp2 = hprev.reshape(T * B, H)
        dw_hh = (torch.matmul(hp2.t(), dG) if wdt == torch.bfloat16 else torch.matmul(hp2.t().float(), dG.float()))
        x2 = x.reshape(T * B, I)
        dGx = dG.to(x2.dtype)
        wdt_hh = wdt if wdt is not None else xdt
        if w_ih is None:
            dx, dw_ih = (dGx.view(T, B, I) if ctx.needs_input_grad[0] else None), None
        else:
            dx = torch.matmul(dGx, w_ih.to(x2.dtype).t()).view(T, B, I) if ctx.needs_input_grad[0] else None
            dw_ih = torch.matmul(x2.t(), dGx).to(wdt) if ctx.needs_input_grad[2] else None
        db = dG.float().sum(0) if has_b else None
        return (dx, None, dw_ih, dw_hh.to(wdt_hh), db, dh0.to(xdt) if has_h0 else None,
                dc0.to(xdt) if has_c0 else None)


def lstm(x, w_ih, w_hh, b=None, h0=None, c0=None, lens=None, time_major=True, return_cells=False):
    """Single-layer unidirectional LSTM.

    x [T, B, I] (or [B, T, I] with ``time_major=False``), w_ih [I, 4H] (None: x is
    already the [.., 4H] gate pre-activation), w_hh [H, 4H],
    b [4H] (= b_ih + b_hh), gate order (i, f, g, o); ``lens`` [B] valid lengths.
    Returns (hs [T, B, H] (batch-major if input was), h_last [B, H], c_last [B, H])
    (+ cs, the cell states laid out like hs, with ``return_cells``); past a
    sequence's end its (h, c) stay frozen, so h_last is its final state.
    """
    if not time_major:
        x = x.transpose(0, 1)
    T, B, _ = x.shape
    H = w_hh.shape[0]
    if not persistent_ok(x, H, B):
        hs, h, c, cs = _lstm_ref(x, w_ih, w_hh, b, h0, c0, lens, cells=True)
    else:
        hs, h, c, cs = _tape.apply(_LstmFn, x.contiguous(), _lens_dev(lens, T, B, x.device), w_ih, w_hh, b, h0, c0)
    if not time_major:
        hs, cs = hs.transpose(0, 1), cs.transpose(0, 1)
    return (hs, h, c, cs) if return_cells else (hs, h, c)


def _lstm_ref(x, w_ih, w_hh, b=None, h0=None, c0=None, lens=None, cells=False):
    """Plain PyTorch recurrence with the same length-freezing semantics (CPU path
    and numerics reference)."""
    T, B, _ = x.shape
    H = w_hh.shape[0]
    dt = x.dtype
    h = h0.to(dt) if h0 is not None else x.new_zeros(B, H)
    c = c0.to(dt) if c0 is not None else x.new_zeros(B, H)
    xp = x.reshape(T * B, -1) if w_ih is None else x.reshape(T * B, -1) @ w_ih.to(dt)
    if b is not None:
        xp = xp + b.to(dt)
    xp = xp.view(T, B, 4 * H)
    L = lens.to(x.device) if lens is not None else None
    out, cout = [], []
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
        cout.append(c)
    if cells:
        return torch.stack(out), h, c, torch.stack(cout)
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


# ---------------------------------------------------------------- attention decoder
class _AttnDecoderFn(torch.autograd.Function):
    """Teacher-forced LSTM decoder with additive attention over an encoder output.

    Per step t (h_{-1} = h0, c_{-1} = c0):
        sp = h_{t-1} Wsp;  att = softmax_s(w . tanh(ep + sp)) over s < slen
        ctx = att . enc;   gates = [ctx, h_{t-1}] Wg + Y[t];  (h_t, c_t) = LSTM cell
    Forward = 4 launches per step (GEMM, fused attention, GEMM, fused cell); the
    backward walks the steps in reverse with 4 launches per step and forms every
    weight gradient (and enc's) after the loop as single large GEMMs.
    """

    @staticmethod
    def forward(ctx_, enc, ep, lens, Y, h0, c0, Wsp, w, Wg):
        B, Ts, E = enc.shape
        A = ep.shape[2]
        Tt, _, G = Y.shape
        H = G // 4
        dev, bf = enc.device, torch.bfloat16
        enc_b, ep_b = enc.to(bf).contiguous(), ep.to(bf).contiguous()
        Wsp_b, Wg_b = Wsp.detach().to(bf).contiguous(), Wg.detach().to(bf).contiguous()
        wf = w.detach().float().contiguous()
        Yf = Y.float().contiguous()
        XH = torch.empty(Tt, B, E + H, dtype=bf, device=dev)      # [ctx_t, h_{t-1}]
        XH[0, :, E:] = h0.to(bf)
        Hs = torch.empty(Tt, B, H, dtype=bf, device=dev)
        Cs = torch.empty(Tt, B, H, dtype=torch.float32, device=dev)
        gates = torch.empty(Tt, B, G, dtype=bf, device=dev)
        SP = torch.empty(Tt, B, A, dtype=bf, device=dev)
        att = torch.empty(Tt, B, Ts, dtype=torch.float32, device=dev)
        c0f = c0.float().contiguous()
        st = N.stream()
        for t in range(Tt):
            hprev = XH[t, :, E:]
            torch.mm(hprev, Wsp_b, out=SP[t])
            N.call("pa_add_attn_fwd", N.ptr(ep_b), N.ptr(SP[t]), N.ptr(wf), N.ptr(enc_b), N.ptr(lens),
                   N.ptr(XH[t]), E + H, N.ptr(att[t]), B, Ts, A, E, st)
            gp = torch.mm(XH[t], Wg_b)
            nxt = XH[t + 1, :, E:] if t + 1 < Tt else None
            N.call("pa_lstm_cell_fwd", N.ptr(gp), N.ptr(Yf[t]), N.ptr(Cs[t - 1] if t else c0f), N.ptr(Cs[t]),
                   N.ptr(gates[t]), N.ptr(Hs[t]), H, N.ptr(nxt), E + H, B, H, st)
        ctx_.save_for_backward(enc_b, ep_b, lens, Wsp_b, wf, Wg_b, XH, Cs, gates, SP, att, c0f)
        ctx_.dt = (enc.dtype, ep.dtype, Y.dtype, h0.dtype, c0.dtype, Wsp.dtype, w.dtype, Wg.dtype)
        return Hs.to(Y.dtype) if Y.dtype != torch.float32 else Hs.float()

    @staticmethod
    def backward(ctx_, dHs):
        enc_b, ep_b, lens, Wsp_b, wf, Wg_b, XH, Cs, gates, SP, att, c0f = ctx_.saved_tensors
        d_enc, d_ep, d_Y, d_h0, d_c0, d_Wsp, d_w, d_Wg = ctx_.dt
        Tt, B, EH = XH.shape
        Ts, E, A = enc_b.shape[1], enc_b.shape[2], ep_b.shape[2]
        H = EH - E
        G = 4 * H
        dev, bf = XH.device, torch.bfloat16
        dHs_b = dHs.to(bf).contiguous()
        dGP = torch.empty(Tt, B, G, dtype=bf, device=dev)
        dSP = torch.empty(Tt, B, A, dtype=bf, device=dev)
        dXH = torch.empty(Tt, B, E + H, dtype=bf, device=dev)          # [dctx_t, dh_{t-1} via Wg]
        dep = torch.zeros(B, Ts, A, dtype=torch.float32, device=dev)
        dw = torch.zeros(A, dtype=torch.float32, device=dev)
        dc = torch.zeros(B, H, dtype=torch.float32, device=dev)
        WgT, WspT = Wg_b.t(), Wsp_b.t()
        st = N.stream()
        dh_rec = None
        for t in range(Tt - 1, -1, -1):
            N.call("pa_lstm_cell_bwd", N.ptr(dHs_b[t]), N.ptr(dh_rec), H, N.ptr(dc), N.ptr(gates[t]),
                   N.ptr(Cs[t]), N.ptr(Cs[t - 1] if t else c0f), N.ptr(dGP[t]), B, H, st)
            torch.mm(dGP[t], WgT, out=dXH[t])
            N.call("pa_add_attn_bwd", N.ptr(dXH[t]), E + H, N.ptr(att[t]), N.ptr(ep_b), N.ptr(SP[t]), N.ptr(wf),
                   N.ptr(enc_b), N.ptr(lens), N.ptr(dep), N.ptr(dSP[t]), N.ptr(dw), B, Ts, A, E, st)
            dh_rec = torch.addmm(dXH[t, :, E:], dSP[t], WspT)            # dh_{t-1} from this step
        TB = Tt * B
        dWg = torch.mm(XH.view(TB, EH).t(), dGP.view(TB, G))
        hprev = XH[:, :, E:].reshape(TB, H)
        dWsp = torch.mm(hprev.t(), dSP.view(TB, A))
        # enc gradient: sum_t att_t^T dctx_t, batched over b
        denc = torch.bmm(att.permute(1, 2, 0).to(bf), dXH[:, :, :E].permute(1, 0, 2))   # [B, Ts, E]
        return (denc.to(d_enc), dep.to(d_ep), None, dGP.to(d_Y), dh_rec.to(d_h0), dc.to(d_c0), dWsp.to(d_Wsp),
                dw.to(d_w), dWg.to(d_Wg))


def attention_lstm_decoder(enc, ep, lens, Y, h0, c0, Wsp, w, Wg):
    """enc [B, Ts, E], ep [B, Ts, A] (= enc projected), lens [B] source lengths,
    Y [Tt, B, 4H] (target-word gate inputs incl. bias), h0/c0 [B, H],
    Wsp [H, A], w [A], Wg [E + H, 4H].  Returns the decoder states [Tt, B, H]."""
    B, Ts, E = enc.shape
    A = ep.shape[2]
    if enc.is_cuda and A % 512 == 0 and E % 1024 == 0 and (Ts + 32 * A) * 4 <= 160 * 1024 and \
            (Ts + 4 * E) * 4 <= 160 * 1024:
        return _tape.apply(_AttnDecoderFn, enc, ep, lens.to(device=enc.device, dtype=torch.int32), Y, h0, c0, Wsp, w, Wg)
    return _attn_decoder_ref(enc, ep, lens, Y, h0, c0, Wsp, w, Wg)


def _attn_decoder_ref(enc, ep, lens, Y, h0, c0, Wsp, w, Wg):
    B, Ts, E = enc.shape
    Tt = Y.shape[0]
    smask = torch.arange(Ts, device=enc.device)[None] < lens.to(enc.device)[:, None]
    h, c = h0, c0
    out = []
    for t in range(Tt):
        e = torch.tanh(ep + (h @ Wsp)[:, None]) @ w
        att = torch.softmax(e.masked_fill(~smask, float("-inf")), 1)
        ctx = torch.bmm(att[:, None].to(enc.dtype), enc).squeeze(1)
        g = torch.cat([ctx, h], 1) @ Wg + Y[t]
        i, f, gg, o = g.chunk(4, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        out.append(h)
    return torch.stack(out)
