"""Recurrent operators over LoD sequences: lstm, lstmp, gru, gru_unit, lstm_unit,
fusion_lstm, fusion_gru.

Parity: paddle/fluid/operators/{lstm,lstmp,gru,gru_unit,lstm_unit,fusion_lstm,
fusion_gru}_op.* with math/detail/{lstm,gru}_kernel.h semantics:
  * LSTM gate layout in the 4D axis is {candidate, input, forget, output}; with
    ``use_peepholes`` the bias is [1, 7D] = {b_c, b_i, b_f, b_o, W_ic, W_fc, W_oc};
    i, f see c_{t-1} and o sees c_t (lstm_kernel.h:36-40);
  * GRU gate layout is {update, reset, candidate}; the hidden-hidden weight
    [D, 3D] holds W_{u,r} in its first 2D columns and W_c in the last D; the
    update is h = h_prev - u*h_prev + u*c (gru_kernel.h:62);
  * ``is_reverse`` processes every sequence from its end.

Execution: the LoD batch is gathered ONCE into a time-major padded block (one
index_select), each time step is a single batched GEMM for all live sequences
(masked for finished ones), and the outputs are scattered back in one op -- the
reference's ``LoDTensor2Batch`` reordering (math/sequence2batch.cc) done with two
device gathers.  Gradients come from the autograd VJP of the same kernels.
"""
from __future__ import annotations

import torch

from ..framework.registry import register_op
from ..ops import oplib as _oplib

_ACTS = {"sigmoid": torch.sigmoid, "tanh": torch.tanh, "relu": torch.relu, "identity": lambda x: x,
         "linear": lambda x: x}
_ACT_ENUM = {0: "identity", 1: "sigmoid", 2: "tanh", 3: "relu"}


def _act(name):
    if isinstance(name, int):
        name = _ACT_ENUM[name]
    return _ACTS[name]


def _pack_index(off, reverse, device):
    """[N, L] packed-row index (-1 = padding) and its validity mask."""
    lens = [off[i + 1] - off[i] for i in range(len(off) - 1)]
    L = max(lens) if lens else 0
    idx = torch.full((len(lens), L), -1, dtype=torch.int64)
    for i, n in enumerate(lens):
        r = torch.arange(off[i], off[i] + n)
        idx[i, :n] = r.flip(0) if reverse else r
    idx = idx.to(device)
    return idx, idx >= 0


def _gather(x, idx, mask):
    g = x.index_select(0, idx.clamp(min=0).reshape(-1)).reshape(idx.shape + x.shape[1:])
    return g * mask.reshape(mask.shape + (1,) * (x.dim() - 1)).to(x.dtype)


def _scatter(seq, idx, mask, T):
    """seq: [N, L, ...] -> packed [T, ...]."""
    flat = seq.reshape((-1,) + seq.shape[2:])
    sel = mask.reshape(-1)
    out = torch.zeros((T,) + seq.shape[2:], dtype=seq.dtype, device=seq.device)
    return out.index_copy(0, idx.reshape(-1)[sel], flat[sel])


def _offsets(ctx, slot):
    lod = ctx.input_lod(slot)
    x = ctx.input(slot)
    return (lod[-1] if lod else [0, x.shape[0]]), lod


def _lstm_core(gx, W, bias, h0, c0, D, peep, acts, idx, mask, T, proj=None, proj_act=None):
    act_gate, act_cell, act_cand = acts
    N, L = idx.shape
    P = proj.shape[1] if proj is not None else D
    h = h0 if h0 is not None else gx.new_zeros(N, P)
    c = c0 if c0 is not None else gx.new_zeros(N, D)
    if proj is not None and h0 is not None:
        h = proj_act(h0 @ proj)
    if peep:
        wic, wfc, woc = bias[0, 4 * D:5 * D], bias[0, 5 * D:6 * D], bias[0, 6 * D:7 * D]
    hs, cs, gates, pre = [], [], [], []
    for t in range(L):
        m = mask[:, t:t + 1]
        g = gx[:, t] + h @ W
        gc, gi, gf, go = g.split(D, dim=1)
        if peep:
            gi = gi + c * wic
            gf = gf + c * wfc
        cand, i, f = act_cand(gc), act_gate(gi), act_gate(gf)
        c_new = cand * i + c * f
        if peep:
            go = go + c_new * woc
        o = act_gate(go)
        h_new = o * act_cell(c_new)
        if proj is not None:
            h_new = proj_act(h_new @ proj)
        h = torch.where(m, h_new, h)
        c = torch.where(m, c_new, c)
        hs.append(h_new)
        cs.append(c_new)
        gates.append(torch.cat([cand, i, f, o], 1))
        pre.append(c_new)
    st = lambda xs: _scatter(torch.stack(xs, 1), idx, mask, T)  # noqa: E731
    return st(hs), st(cs), st(gates), st(pre)


def _persistent_lstm_ok(ctx, x, D, nseq):
    import os

    from ..ops import rnn as R

    return (not ctx.attr("use_peepholes") and os.environ.get("PADDLE_AMD_PERSISTENT_LSTM", "1") != "0"
            and _act(ctx.attr("gate_activation")) is torch.sigmoid and _act(ctx.attr("cell_activation")) is torch.tanh
            and _act(ctx.attr("candidate_activation")) is torch.tanh and R.persistent_ok(x, D, nseq))


def _lstm_persistent(gx, W, h0, c0, D, idx, mask, T):
    """The LoD LSTM on the persistent gfx950 kernel (ops/rnn.py).  Fluid's gate
    order {c~, i, f, o} is permuted to the kernel's {i, f, c~, o}."""
    from ..ops import rnn as R

    perm = torch.cat([torch.arange(D, 2 * D), torch.arange(2 * D, 3 * D), torch.arange(0, D),
                      torch.arange(3 * D, 4 * D)]).to(gx.device)
    lens = mask.sum(1).to(torch.int32)
    xt = gx.index_select(2, perm).transpose(0, 1)            # [L, N, 4D] time-major
    hs, _, _, cs = R.lstm(xt, None, W.index_select(1, perm), None, h0, c0, lens=lens, return_cells=True)
    return (_scatter(hs.transpose(0, 1), idx, mask, T),       # [N, L, D] -> LoD rows
            _scatter(cs.transpose(0, 1), idx, mask, T))


def _lstm_attrs(extra=None):
    a = {"use_peepholes": True, "is_reverse": False, "gate_activation": "sigmoid", "cell_activation": "tanh",
         "candidate_activation": "tanh"}
    a.update(extra or {})
    return a


@register_op("lstm", ["Input", "H0?", "C0?", "Weight", "Bias"],
             ["Hidden", "Cell", "BatchGate~", "BatchCellPreAct~"], _lstm_attrs())
def lstm(ctx):
    x, W, b = ctx.input("Input"), ctx.input("Weight"), ctx.input("Bias")
    D = W.shape[0]
    T = x.shape[0]
    if ctx.meta:
        for s, n in (("Hidden", D), ("Cell", D), ("BatchGate", 4 * D), ("BatchCellPreAct", D)):
            ctx.set_output(s, torch.empty(T, n, dtype=x.dtype, device="meta"))
        return
    off, lod = _offsets(ctx, "Input")
    idx, mask = _pack_index(off, ctx.attr("is_reverse"), x.device)
    gx = _gather(x + b[:, :4 * D], idx, mask)
    acts = (_act(ctx.attr("gate_activation")), _act(ctx.attr("cell_activation")),
            _act(ctx.attr("candidate_activation")))
    h0 = ctx.input("H0") if ctx.has_input("H0") else None
    c0 = ctx.input("C0") if ctx.has_input("C0") else None
    if _persistent_lstm_ok(ctx, x, D, idx.shape[0]):
        H, C = _lstm_persistent(gx, W, h0, c0, D, idx, mask, T)
        ctx.set_output("Hidden", H, lod)
        ctx.set_output("Cell", C, lod)
        ctx.set_output("BatchGate", _scatter(gx.detach(), idx, mask, T))
        ctx.set_output("BatchCellPreAct", C.detach())
        return
    H, C, G, P = _lstm_core(gx, W, b, h0, c0, D, ctx.attr("use_peepholes"), acts, idx, mask, T)
    ctx.set_output("Hidden", H, lod)
    ctx.set_output("Cell", C, lod)
    ctx.set_output("BatchGate", G.detach())
    ctx.set_output("BatchCellPreAct", P.detach())


@register_op("lstmp", ["Input", "H0?", "C0?", "Weight", "ProjWeight", "Bias"],
             ["Projection", "Cell", "BatchGate~", "BatchCellPreAct~", "BatchHidden~", "OrderedP0~"],
             _lstm_attrs({"proj_activation": "tanh"}))
def lstmp(ctx):
    x, W, PW, b = ctx.input("Input"), ctx.input("Weight"), ctx.input("ProjWeight"), ctx.input("Bias")
    D, P = PW.shape
    T = x.shape[0]
    if ctx.meta:
        for s, n in (("Projection", P), ("Cell", D), ("BatchGate", 4 * D), ("BatchCellPreAct", D),
                     ("BatchHidden", P)):
            ctx.set_output(s, torch.empty(T, n, dtype=x.dtype, device="meta"))
        return
    off, lod = _offsets(ctx, "Input")
    idx, mask = _pack_index(off, ctx.attr("is_reverse"), x.device)
    gx = _gather(x + b[:, :4 * D], idx, mask)
    acts = (_act(ctx.attr("gate_activation")), _act(ctx.attr("cell_activation")),
            _act(ctx.attr("candidate_activation")))
    pact = _act(ctx.attr("proj_activation"))
    h0 = ctx.input("H0") if ctx.has_input("H0") else None
    c0 = ctx.input("C0") if ctx.has_input("C0") else None
    R, C, G, Pre = _lstm_core(gx, W, b, h0, c0, D, ctx.attr("use_peepholes"), acts, idx, mask, T, PW, pact)
    ctx.set_output("Projection", R, lod)
    ctx.set_output("Cell", C, lod)
    ctx.set_output("BatchGate", G.detach())
    ctx.set_output("BatchCellPreAct", Pre.detach())
    ctx.set_output("BatchHidden", R.detach())
    if h0 is not None:
        ctx.set_output("OrderedP0", pact(h0 @ PW).detach())


def _gru_step(g, h, W, D, act, act_gate):
    if g.is_cuda and act is torch.tanh and act_gate is torch.sigmoid:
        # fused gate / output kernels (math/detail/gru_gpu_kernel.h)
        r = _oplib.gru_step(g, h, W, D)
        if r is not None:
            return r
    ur = g[:, :2 * D] + h @ W[:, :2 * D]
    u, r = act_gate(ur[:, :D]), act_gate(ur[:, D:])
    rh = r * h
    c = act(g[:, 2 * D:] + rh @ W[:, 2 * D:])
    return h - u * h + u * c, u, r, c, rh


@register_op("gru", ["Input", "H0?", "Weight", "Bias?"],
             ["BatchGate~", "BatchResetHiddenPrev~", "BatchHidden~", "Hidden"],
             {"activation": "tanh", "gate_activation": "sigmoid", "is_reverse": False})
def gru(ctx):
    x, W = ctx.input("Input"), ctx.input("Weight")
    D = W.shape[0]
    T = x.shape[0]
    if ctx.meta:
        for s, n in (("Hidden", D), ("BatchGate", 3 * D), ("BatchResetHiddenPrev", D), ("BatchHidden", D)):
            ctx.set_output(s, torch.empty(T, n, dtype=x.dtype, device="meta"))
        return
    off, lod = _offsets(ctx, "Input")
    if ctx.has_input("Bias"):
        x = x + ctx.input("Bias")
    idx, mask = _pack_index(off, ctx.attr("is_reverse"), x.device)
    gx = _gather(x, idx, mask)
    act, act_gate = _act(ctx.attr("activation")), _act(ctx.attr("gate_activation"))
    h = ctx.input("H0") if ctx.has_input("H0") else x.new_zeros(idx.shape[0], D)
    hs, gates, rhs = [], [], []
    for t in range(idx.shape[1]):
        h_new, u, r, c, rh = _gru_step(gx[:, t], h, W, D, act, act_gate)
        h = torch.where(mask[:, t:t + 1], h_new, h)
        hs.append(h_new)
        gates.append(torch.cat([u, r, c], 1))
        rhs.append(rh)
    st = lambda xs: _scatter(torch.stack(xs, 1), idx, mask, T)  # noqa: E731
    Hd = st(hs)
    ctx.set_output("Hidden", Hd, lod)
    ctx.set_output("BatchGate", st(gates).detach())
    ctx.set_output("BatchResetHiddenPrev", st(rhs).detach())
    ctx.set_output("BatchHidden", Hd.detach())


@register_op("gru_unit", ["Input", "HiddenPrev", "Weight", "Bias?"], ["Gate~", "ResetHiddenPrev~", "Hidden"],
             {"activation": 2, "gate_activation": 1}, share_lod=False)
def gru_unit(ctx):
    x, h, W = ctx.input("Input"), ctx.input("HiddenPrev"), ctx.input("Weight")
    D = W.shape[0]
    if ctx.has_input("Bias"):
        x = x + ctx.input("Bias")
    h_new, u, r, c, rh = _gru_step(x, h, W, D, _act(ctx.attr("activation")), _act(ctx.attr("gate_activation")))
    ctx.set_output("Gate", torch.cat([u, r, c], 1))
    ctx.set_output("ResetHiddenPrev", rh)
    ctx.set_output("Hidden", h_new)


@register_op("lstm_unit", ["X", "C_prev"], ["C", "H"], {"forget_bias": 0.0}, share_lod=False)
def lstm_unit(ctx):
    """Gate order {i, f, o, g} (lstm_unit_op.h:63-71); forget_bias added before the sigmoid."""
    x, cp = ctx.input("X"), ctx.input("C_prev")
    from ..ops import nnmisc as _nm
    r = _nm.lstm_unit(x, cp, ctx.attr("forget_bias"))
    if r is not None:  # lstm_unit kernels (nnmisc.hip)
        ctx.set_output("C", r[0])
        ctx.set_output("H", r[1])
        return
    D = cp.shape[1]
    i, f, o, g = x.split(D, dim=1)
    c = torch.sigmoid(f + ctx.attr("forget_bias")) * cp + torch.sigmoid(i) * torch.tanh(g)
    ctx.set_output("C", c)
    ctx.set_output("H", torch.sigmoid(o) * torch.tanh(c))


@register_op("fusion_lstm", ["X", "WeightX", "WeightH", "Bias", "H0?", "C0?"],
             ["Hidden", "Cell", "XX~", "BatchedInput~", "BatchedHidden~", "BatchedCell~", "ReorderedH0~",
              "ReorderedC0~"], _lstm_attrs({"use_seq": True}))
def fusion_lstm(ctx):
    """x @ WeightX folded into the recurrence (one GEMM for all time steps first)."""
    x, WX, WH, b = ctx.input("X"), ctx.input("WeightX"), ctx.input("WeightH"), ctx.input("Bias")
    D = WH.shape[0]
    T = x.shape[0]
    if ctx.meta:
        for s, n in (("Hidden", D), ("Cell", D), ("XX", 4 * D)):
            ctx.set_output(s, torch.empty(T, n, dtype=x.dtype, device="meta"))
        return
    off, lod = _offsets(ctx, "X")
    xx = x @ WX
    idx, mask = _pack_index(off, ctx.attr("is_reverse"), x.device)
    gx = _gather(xx + b[:, :4 * D], idx, mask)
    acts = (_act(ctx.attr("gate_activation")), _act(ctx.attr("cell_activation")),
            _act(ctx.attr("candidate_activation")))
    h0 = ctx.input("H0") if ctx.has_input("H0") else None
    c0 = ctx.input("C0") if ctx.has_input("C0") else None
    if _persistent_lstm_ok(ctx, x, D, idx.shape[0]):
        # all time steps of the recurrence in one persistent kernel launch (rnn.hip)
        H, C = _lstm_persistent(gx, WH, h0, c0, D, idx, mask, T)
    else:
        H, C, _, _ = _lstm_core(gx, WH, b, h0, c0, D, ctx.attr("use_peepholes"), acts, idx, mask, T)
    ctx.set_output("Hidden", H, lod)
    ctx.set_output("Cell", C, lod)
    ctx.set_output("XX", xx.detach())


@register_op("fusion_gru", ["X", "H0?", "WeightX", "WeightH", "Bias?"],
             ["ReorderedH0~", "XX~", "BatchedInput~", "BatchedOut~", "Hidden"],
             {"activation": "tanh", "gate_activation": "sigmoid", "is_reverse": False, "use_seq": True})
def fusion_gru(ctx):
    x, WX, WH = ctx.input("X"), ctx.input("WeightX"), ctx.input("WeightH")
    D = WH.shape[0]
    T = x.shape[0]
    if ctx.meta:
        ctx.set_output("Hidden", torch.empty(T, D, dtype=x.dtype, device="meta"))
        ctx.set_output("XX", torch.empty(T, 3 * D, dtype=x.dtype, device="meta"))
        return
    off, lod = _offsets(ctx, "X")
    xx = x @ WX
    if ctx.has_input("Bias"):
        xx = xx + ctx.input("Bias")
    idx, mask = _pack_index(off, ctx.attr("is_reverse"), x.device)
    gx = _gather(xx, idx, mask)
    act, act_gate = _act(ctx.attr("activation")), _act(ctx.attr("gate_activation"))
    h = ctx.input("H0") if ctx.has_input("H0") else x.new_zeros(idx.shape[0], D)
    hs = []
    for t in range(idx.shape[1]):
        h_new = _gru_step(gx[:, t], h, WH, D, act, act_gate)[0]
        h = torch.where(mask[:, t:t + 1], h_new, h)
        hs.append(h_new)
    ctx.set_output("Hidden", _scatter(torch.stack(hs, 1), idx, mask, T), lod)
    ctx.set_output("XX", xx.detach())
