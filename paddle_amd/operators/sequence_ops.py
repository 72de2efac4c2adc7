"""LoD (variable-length sequence) operators.

Parity: paddle/fluid/operators/{sequence_pool,sequence_softmax,sequence_expand,
sequence_expand_as,sequence_concat,sequence_conv,sequence_erase,sequence_reshape,
sequence_slice,sequence_pad,sequence_unpad,sequence_mask,sequence_enumerate,
lod_reset}_op.* and math/sequence_pooling.cu (SURVEY §2.7 "Sequence / LoD ops").

LoD offsets are host lists; per-sequence work is expressed with segment ops over
the packed rows (index_add / segment reductions) so the device does one launch
per op instead of one per sequence wherever the math allows.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ..framework import core
from ..framework.registry import register_op
from ..ops import blas as _blas
from ..ops import fluidk as _fk
from ..ops import oplib as _oplib


def _last_level(ctx, slot="X"):
    lod = ctx.input_lod(slot)
    x = ctx.input(slot)
    if not lod:
        return [0, x.shape[0]], lod
    return lod[-1], lod


def _seg_ids(off, device):
    lens = torch.tensor([off[i + 1] - off[i] for i in range(len(off) - 1)], device=device)
    return torch.repeat_interleave(torch.arange(len(off) - 1, device=device), lens), lens


@register_op("sequence_pool", ["X"], ["Out", "MaxIndex~"], {"pooltype": "AVERAGE", "is_test": False},
             share_lod=False)
def sequence_pool(ctx):
    x = ctx.input("X")
    off, lod = _last_level(ctx)
    n = len(off) - 1
    pt = ctx.attr("pooltype").upper()
    D = x.shape[1:]
    if ctx.meta:
        ctx.set_output("Out", torch.empty((n,) + tuple(D), dtype=x.dtype, device="meta"))
        return
    out_lod = lod[:-1] if len(lod) > 1 else None
    r = _oplib.seq_pool_op(x, off, pt) if x.is_cuda else None
    if r is not None:  # math/sequence_pooling.cu on the native kernel (MaxIndex int32)
        ctx.set_output("Out", r[0], out_lod)
        ctx.set_output("MaxIndex", r[1])
        return
    seg, lens = _seg_ids(off, x.device)
    lensf = lens.to(x.dtype).reshape((-1,) + (1,) * len(D)).clamp_min(1)
    idx = torch.zeros((n,) + tuple(D), dtype=torch.int64, device=x.device)
    if pt in ("AVERAGE", "SUM", "SQRT"):
        out = torch.zeros((n,) + tuple(D), dtype=x.dtype, device=x.device).index_add_(0, seg, x)
        if pt == "AVERAGE":
            out = out / lensf
        elif pt == "SQRT":
            out = out / torch.sqrt(lensf)
    elif pt == "MAX":
        out = torch.full((n,) + tuple(D), float("-inf"), dtype=x.dtype, device=x.device)
        out = out.scatter_reduce(0, seg.reshape((-1,) + (1,) * len(D)).expand_as(x), x, "amax")
        out = torch.where(torch.isinf(out), torch.zeros_like(out), out)
    elif pt == "LAST":
        out = x[torch.tensor([max(off[i + 1] - 1, off[i]) for i in range(n)], device=x.device)]
    elif pt == "FIRST":
        out = x[torch.tensor(off[:-1], device=x.device)]
    else:
        raise ValueError(pt)
    out_lod = lod[:-1] if len(lod) > 1 else None
    ctx.set_output("Out", out, out_lod)
    ctx.set_output("MaxIndex", idx)


@register_op("sequence_softmax", ["X"], ["Out"], {"use_cudnn": False})
def sequence_softmax(ctx):
    x = ctx.input("X")
    off, lod = _last_level(ctx)
    flat = x.reshape(-1)
    if ctx.meta:
        ctx.set_output("Out", torch.empty_like(x))
        return
    if x.is_cuda and _fk.ok(x):
        # one wave per sequence: max / sum / normalise over the LoD segment in one pass
        ctx.set_output("Out", _fk.seq_softmax(flat, off).reshape(x.shape), lod)
        return
    seg, _ = _seg_ids(off, x.device)
    n = len(off) - 1
    mx = torch.full((n,), float("-inf"), dtype=x.dtype, device=x.device).scatter_reduce(0, seg, flat, "amax")
    e = torch.exp(flat - mx[seg])
    s = torch.zeros(n, dtype=x.dtype, device=x.device).index_add_(0, seg, e)
    ctx.set_output("Out", (e / s[seg]).reshape(x.shape), lod)


@register_op("sequence_softmax_grad", ["X?", "Out", "Out@GRAD"], ["X@GRAD"], {"use_cudnn": False}, grad=None,
             no_infer=True)
def sequence_softmax_grad(ctx):
    y, g = ctx.input("Out"), ctx.input("Out@GRAD")
    lod = ctx.input_lod("Out") or ctx.input_lod("X")
    off = lod[-1] if lod else [0, y.shape[0]]
    if y.is_cuda and _fk.ok(y, g):
        ctx.set_output("X@GRAD", _fk.seq_softmax_grad(y.reshape(-1), g.reshape(-1), off).reshape(y.shape))
        return
    seg, _ = _seg_ids(off, y.device)
    yf, gf = y.reshape(-1), g.reshape(-1)
    dot = torch.zeros(len(off) - 1, dtype=y.dtype, device=y.device).index_add_(0, seg, yf * gf)
    ctx.set_output("X@GRAD", (yf * (gf - dot[seg])).reshape(y.shape))


@register_op("sequence_expand", ["X", "Y"], ["Out"], {"ref_level": -1}, share_lod=False)
def sequence_expand(ctx):
    x = ctx.input("X")
    ylod = ctx.input_lod("Y")
    ref = ctx.attr("ref_level")
    ref = len(ylod) - 1 if ref == -1 else ref
    yoff = ylod[ref]
    if len(yoff) <= 1:
        ctx.set_output("Out", x, ctx.input_lod("X"))
        return
    xlod = ctx.input_lod("X")
    # (sequence_expand_op.h) only a 1-level X LoD defines X's sequences; otherwise
    # every row is one sequence and the output carries no LoD
    xlod = xlod if len(xlod) == 1 else []
    xoff = xlod[0] if xlod else list(range(x.shape[0] + 1))
    xo = np.asarray(xoff, dtype=np.int64)
    reps = np.diff(np.asarray(yoff, dtype=np.int64))
    # block b = one copy of X's sequence i; rows = concatenated ranges (no per-row loop)
    starts, lens = np.repeat(xo[:-1], reps), np.repeat(np.diff(xo), reps)
    out_off = np.concatenate([[0], np.cumsum(lens)])
    rows = np.repeat(starts - out_off[:-1], lens) + np.arange(int(out_off[-1]))
    out = _oplib.gather_rows_op(x, rows) if x.is_cuda and rows.size else None
    if out is None:
        out = x[torch.as_tensor(rows, dtype=torch.long, device=x.device)]
    ctx.set_output("Out", out, [out_off.tolist()] if xlod else None)


@register_op("sequence_expand_as", ["X", "Y"], ["Out"], {}, share_lod=False)
def sequence_expand_as(ctx):
    """Row i of X repeated len(Y's sequence i) times (sequence_expand_as_op.h), as
    one HIP row gather with a scatter-add backward."""
    x = ctx.input("X")
    yoff = ctx.input_lod("Y")[0]
    reps = np.diff(np.asarray(yoff, dtype=np.int64))
    rows = np.repeat(np.arange(len(reps)), reps)
    out = _oplib.gather_rows_op(x, rows) if x.is_cuda and rows.size else None
    if out is None:
        out = x[torch.as_tensor(rows, dtype=torch.long, device=x.device)]
    ctx.set_output("Out", out, [list(yoff)])


def _abs_lod(lod):
    """Every LoD level as absolute row offsets (framework ToAbsOffset)."""
    out = [list(lv) for lv in lod]
    for i in range(len(out) - 2, -1, -1):
        out[i] = [out[i + 1][o] for o in lod[i]]
    return out


def _concat_lod(lods, level):
    """LoD of the axis-0 concatenation at ``level`` (0 = finest): that level's
    offsets add up over the inputs, the levels below are re-laid out sequence by
    sequence (reference sequence_concat_op.h ConcatLoD)."""
    n, nlev = len(lods), len(lods[0])
    li = nlev - 1 - level
    out = [list(lv) for lv in lods[0]]
    out[li] = [sum(l[li][j] for l in lods) for j in range(len(lods[0][li]))]
    for i in range(li, nlev - 1):
        new = [0]
        for j in range(len(lods[0][i]) - 1):
            for k in range(n):
                for m in range(lods[k][i][j], lods[k][i][j + 1]):
                    new.append(new[-1] + lods[k][i + 1][m + 1] - lods[k][i + 1][m])
        out[i + 1] = new
    return out


@register_op("sequence_concat", ["X*"], ["Out"], {"axis": 0, "level": 0}, share_lod=False)
def sequence_concat(ctx):
    """Per sequence of LoD level ``level`` (0 = the finest), the inputs' slices
    joined along ``axis``: axis 0 stacks their rows (LoD from ConcatLoD), another
    axis joins columns of equally long slices (LoD of X[0])."""
    xs = ctx.input_values("X")
    axis, level = int(ctx.attr("axis")), int(ctx.attr("level"))
    lods = [[list(lv) for lv in v.lod()] for v in xs]
    if not lods[0] or any(len(l) != len(lods[0]) for l in lods) or level >= len(lods[0]):
        raise ValueError("sequence_concat: inputs need the same number of LoD levels, more than `level`")
    li = len(lods[0]) - 1 - level
    out_lod = _concat_lod(lods, level) if axis == 0 else lods[0]
    abs_in = [_abs_lod(l)[li] for l in lods]
    parts = []
    for i in range(len(abs_in[0]) - 1):
        sl = [v.tensor[a[i]:a[i + 1]] for v, a in zip(xs, abs_in)]
        parts.append(torch.cat(sl, axis))
    ctx.set_output("Out", torch.cat(parts, 0), out_lod)


def _context_index(off, T, cl, cs, up_pad, has_pad):
    """Row map of the context projection (math/context_project.h): column block k
    of output row r reads row r + cs + k of the same sequence; outside it, the
    trainable padding row up_pad + (src - start) above / up_pad + (src - end) below
    (stored after the T input rows), else -1 (zero)."""
    o = np.asarray(off, dtype=np.int64)
    seg = np.repeat(np.arange(len(o) - 1), np.diff(o))
    s, e = o[seg][:, None], o[seg + 1][:, None]
    src = np.arange(T)[:, None] + cs + np.arange(cl)[None, :]
    idx = np.where((src >= s) & (src < e), src, -1)
    if has_pad:
        idx = np.where(src < s, T + up_pad + (src - s), idx)
        idx = np.where(src >= e, T + up_pad + (src - e), idx)
    return idx.reshape(-1)


@register_op("sequence_conv", ["X", "Filter", "PaddingData?"], ["Out"],
             {"contextLength": 3, "contextStart": 0, "contextStride": 1, "paddingTrainable": False})
def sequence_conv(ctx):
    """Context projection + GEMM with the filter (sequence_conv_op.h).  The
    projection is one HIP row gather over [X; PaddingData] (scatter-add backward
    into both), the product the native GEMM; gradients by the eager engine."""
    x, w = ctx.input("X"), ctx.input("Filter")
    off, lod = _last_level(ctx)
    cl, cs = ctx.attr("contextLength"), ctx.attr("contextStart")
    if ctx.attr("contextStride") != 1:
        raise ValueError("sequence_conv: contextStride must be 1 (sequence_conv_op.cc)")
    T, D = x.shape[0], x.shape[1]
    if ctx.meta:
        ctx.set_output("Out", torch.empty(T, w.shape[1], dtype=x.dtype, device="meta"))
        return
    up_pad = max(0, -cs)
    pad = ctx.input("PaddingData") if ctx.attr("paddingTrainable") and ctx.has_input("PaddingData") else None
    idx = _context_index(off, T, cl, cs, up_pad, pad is not None)
    table = torch.cat([x, pad.to(x.dtype)], 0) if pad is not None else x
    cols = _oplib.gather_rows_op(table, idx) if x.is_cuda and T else None
    if cols is None:
        table = torch.cat([table, table.new_zeros(1, D)], 0)
        it = torch.as_tensor(np.where(idx < 0, table.shape[0] - 1, idx), dtype=torch.long, device=x.device)
        cols = table[it]
    cols = cols.reshape(T, cl * D)
    w = w.to(cols.dtype)
    out = _blas.matmul(cols, w) if _blas.supported(cols, w) else cols @ w
    ctx.set_output("Out", out, lod)


@register_op("sequence_erase", ["X"], ["Out"], {"tokens": []}, share_lod=False)
def sequence_erase(ctx):
    x = ctx.input("X")
    off, lod = _last_level(ctx)
    toks = set(ctx.attr("tokens"))
    flat = x.reshape(-1).tolist()
    keep, new_off = [], [0]
    for s, e in zip(off[:-1], off[1:]):
        k = [i for i in range(s, e) if flat[i] not in toks]
        keep += k
        new_off.append(new_off[-1] + len(k))
    ctx.set_output("Out", x[torch.tensor(keep, dtype=torch.long, device=x.device)], [new_off])


@register_op("sequence_reshape", ["X"], ["Out"], {"new_dim": 1}, share_lod=False)
def sequence_reshape(ctx):
    x = ctx.input("X")
    off, _ = _last_level(ctx)
    nd = ctx.attr("new_dim")
    D = x.shape[1]
    new_off = [o * D // nd for o in off]
    ctx.set_output("Out", x.reshape(-1, nd), [new_off])


@register_op("sequence_slice", ["X", "Offset", "Length"], ["Out"], {}, share_lod=False)
def sequence_slice(ctx):
    x = ctx.input("X")
    off, _ = _last_level(ctx)
    so = ctx.input("Offset").reshape(-1).tolist()
    sl = ctx.input("Length").reshape(-1).tolist()
    rows, new_off = [], [0]
    for i in range(len(off) - 1):
        st = off[i] + int(so[i])
        rows += list(range(st, st + int(sl[i])))
        new_off.append(new_off[-1] + int(sl[i]))
    ctx.set_output("Out", x[torch.tensor(rows, dtype=torch.long, device=x.device)], [new_off])


@register_op("sequence_pad", ["X", "PadValue"], ["Out", "Length"], {"padded_length": -1}, share_lod=False)
def sequence_pad(ctx):
    x, pv = ctx.input("X"), ctx.input("PadValue")
    off, _ = _last_level(ctx)
    n = len(off) - 1
    lens = [off[i + 1] - off[i] for i in range(n)]
    L = ctx.attr("padded_length")
    L = max(lens) if L == -1 else L
    if x.is_cuda and pv.numel() == 1 and x.dim() >= 1:
        # one row gather: padded slot (i, t) <- row off[i] + t, or the pad value
        src = [off[i] + t if t < lens[i] else -1 for i in range(n) for t in range(L)]
        out = _oplib.gather_rows_op(x, src, float(pv.reshape(-1)[0].item())) if src else None
        if out is not None:
            ctx.set_output("Out", out.reshape((n, L) + tuple(x.shape[1:])))
            ctx.set_output("Length", torch.tensor(lens, dtype=torch.int64, device=x.device))
            return
    out = pv.reshape((1, 1) + tuple(x.shape[1:]) if pv.numel() > 1 else (1,)).expand(
        (n, L) + tuple(x.shape[1:])).clone()
    for i in range(n):
        out[i, :lens[i]] = x[off[i]:off[i + 1]]
    ctx.set_output("Out", out)
    ctx.set_output("Length", torch.tensor(lens, dtype=torch.int64, device=x.device))


@register_op("sequence_unpad", ["X", "Length"], ["Out"], {}, share_lod=False)
def sequence_unpad(ctx):
    x = ctx.input("X")
    lens = [int(v) for v in ctx.input("Length").reshape(-1).tolist()]
    if x.is_cuda and x.dim() >= 2 and sum(lens):
        L = x.shape[1]
        out = _oplib.gather_rows_op(x.reshape((-1,) + tuple(x.shape[2:])),
                                    [i * L + t for i, l in enumerate(lens) for t in range(l)])
        if out is not None:
            off = [0]
            for l in lens:
                off.append(off[-1] + l)
            ctx.set_output("Out", out, [off])
            return
    parts = [x[i, :l] for i, l in enumerate(lens)]
    off = [0]
    for l in lens:
        off.append(off[-1] + l)
    ctx.set_output("Out", torch.cat(parts, 0), [off])


@register_op("sequence_mask", ["X"], ["Y"], {"maxlen": -1, "out_dtype": 3}, grad=None)
def sequence_mask(ctx):
    x = ctx.input("X")
    ml = ctx.attr("maxlen")
    if ml < 0:
        ml = int(x.max().item()) if not ctx.meta else 8191
    r = torch.arange(ml, device=x.device)
    ctx.set_output("Y", (r < x.unsqueeze(-1)).to(core.to_torch_dtype(ctx.attr("out_dtype"))))


@register_op("sequence_enumerate", ["X"], ["Out"], {"win_size": 2, "pad_value": 0}, grad=None)
def sequence_enumerate(ctx):
    x = ctx.input("X")
    off, lod = _last_level(ctx)
    w, pv = ctx.attr("win_size"), ctx.attr("pad_value")
    flat = x.reshape(-1)
    out = torch.full((flat.shape[0], w), pv, dtype=x.dtype, device=x.device)
    for s, e in zip(off[:-1], off[1:]):
        for k in range(w):
            if e - s - k > 0:
                out[s:e - k, k] = flat[s + k:e]
    ctx.set_output("Out", out, lod)


@register_op("lod_reset", ["X", "Y?"], ["Out"], {"target_lod": []}, share_lod=False)
def lod_reset(ctx):
    x = ctx.input("X")
    if ctx.has_input("Y"):
        yv = ctx.input_value("Y")
        lod = yv.lod() if yv.lod() else [[int(v) for v in yv.tensor.reshape(-1).tolist()]]
    else:
        lod = [list(ctx.attr("target_lod"))]
    ctx.set_output("Out", x, lod)


@register_op("sequence_scatter", ["X", "Ids", "Updates"], ["Out"], {}, share_lod=False)
def sequence_scatter(ctx):
    x, ids, up = ctx.input("X"), ctx.input("Ids"), ctx.input("Updates")
    off = ctx.input_lod("Ids")[0]
    # one out-of-place accumulating index_put: differentiable in X and Updates
    # (sequence_scatter_op.h: Updates@GRAD[k] = Out@GRAD[seq(k), Ids[k]])
    rows = torch.repeat_interleave(torch.arange(len(off) - 1, device=x.device),
                                   torch.tensor([off[i + 1] - off[i] for i in range(len(off) - 1)], device=x.device))
    cols = ids.reshape(-1).long()
    ctx.set_output("Out", x.index_put((rows, cols), up.reshape(-1).to(x.dtype), accumulate=True))


@register_op("sequence_reverse", ["X"], ["Y"], {})
def sequence_reverse(ctx):
    """Reverse the rows of every sequence (later Paddle's sequence_reverse_op; the v1
    recurrent layers' ``reverse=True``).  A gather: its VJP is the inverse gather."""
    x = ctx.input("X")
    off, lod = _last_level(ctx)
    if ctx.meta:
        ctx.set_output("Y", torch.empty_like(x, device="meta"), lod or None)
        return
    idx = [j for i in range(len(off) - 1) for j in range(off[i + 1] - 1, off[i] - 1, -1)]
    ctx.set_output("Y", x[torch.tensor(idx, dtype=torch.long, device=x.device)], lod or None)


@register_op("scale_sub_region", ["X", "Indices"], ["Out"], {"value": 1.0})
def scale_sub_region(ctx):
    """v1 ScaleSubRegionLayer: multiply the box [c0, c1] x [h0, h1] x [w0, w1]
    (1-based, inclusive; one row of Indices per sample) of each [C, H, W] sample."""
    x = ctx.input("X")
    if ctx.meta:
        ctx.set_output("Out", torch.empty_like(x, device="meta"))
        return
    ind = ctx.input("Indices").to(torch.long).reshape(x.shape[0], 6).cpu().tolist()
    m = torch.ones_like(x)
    v = float(ctx.attr("value"))
    for n, (c0, c1, h0, h1, w0, w1) in enumerate(ind):
        m[n, c0 - 1:c1, h0 - 1:h1, w0 - 1:w1] = v
    ctx.set_output("Out", x * m)
