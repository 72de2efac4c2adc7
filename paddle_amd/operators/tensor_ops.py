"""Tensor manipulation, creation, random, comparison and logical operators.

Parity: paddle/fluid/operators/{reshape,squeeze,unsqueeze,flatten,transpose,concat,
split,stack,unstack,expand,gather,scatter,slice,reverse,cast,shape,assign,
assign_value,fill_constant,fill,fill_zeros_like,fill_constant_batch_size_like,
uniform_random(_batch_size_like),gaussian_random(_batch_size_like),sampling_id,
random_crop,multiplex,compare,logical,increment,is_empty,arg_max,arg_min,argsort,
print,delete_var,shuffle_channel}_op.* (SURVEY §2.7 "Tensor manipulation").
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import fluidk as _fk
from ..ops import oplib as _oplib

from ..framework import core
from ..framework.registry import register_op


def _infer_reshape(shape, src):
    shape = list(shape)
    out = []
    for i, s in enumerate(shape):
        out.append(src[i] if s == 0 else s)
    return out


@register_op("reshape", ["X", "Shape?"], ["Out"], {"shape": [], "inplace": False})
def reshape(ctx):
    x = ctx.input("X")
    if ctx.has_input("Shape") and not ctx.meta:
        shape = [int(v) for v in ctx.input("Shape").reshape(-1).tolist()]
    else:
        shape = _infer_reshape(ctx.attr("shape"), list(x.shape))
    ctx.set_output("Out", x.reshape(shape))


@register_op("reshape2", ["X", "Shape?"], ["Out", "XShape~"], {"shape": []})
def reshape2(ctx):
    reshape(ctx)
    x = ctx.input("X")
    ctx.set_output("XShape", torch.empty((0,) + tuple(x.shape), dtype=x.dtype, device=x.device))


@register_op("squeeze", ["X"], ["Out"], {"axes": []})
def squeeze(ctx):
    x = ctx.input("X")
    axes = ctx.attr("axes")
    if not axes:
        out = x.squeeze()
    else:
        out = x
        for a in sorted([a % x.dim() for a in axes], reverse=True):
            if out.shape[a] == 1:
                out = out.squeeze(a)
    ctx.set_output("Out", out)


@register_op("unsqueeze", ["X"], ["Out"], {"axes": []})
def unsqueeze(ctx):
    out = ctx.input("X")
    for a in sorted(ctx.attr("axes")):
        out = out.unsqueeze(a)
    ctx.set_output("Out", out)


@register_op("flatten", ["X"], ["Out"], {"axis": 1})
def flatten(ctx):
    x = ctx.input("X")
    a = ctx.attr("axis")
    ctx.set_output("Out", x.reshape(int(np.prod(x.shape[:a])) if a else 1, -1))


def _dev(ctx, *ts):
    """HIP path: a device place, real (not meta) run, every operand on the device."""
    return not ctx.meta and all(t is not None and t.is_cuda for t in ts)


def _permute(ctx, x, perm):
    if _dev(ctx, x) and x.dim() <= 8:
        return _fk.permute(x, perm)
    return x.permute(*perm).contiguous()


@register_op("transpose", ["X"], ["Out"], {"axis": [], "use_mkldnn": False, "data_format": "AnyLayout"})
def transpose(ctx):
    ctx.set_output("Out", _permute(ctx, ctx.input("X"), list(ctx.attr("axis"))))


_reg_t2 = register_op("transpose2", ["X"], ["Out", "XShape~"], {"axis": []})(
    lambda ctx: transpose(ctx))


def _transpose_grad(ctx):
    perm = list(ctx.attr("axis"))
    inv = [0] * len(perm)
    for i, p in enumerate(perm):
        inv[p] = i
    ctx.set_output("X@GRAD", _permute(ctx, ctx.input("Out@GRAD"), inv))


register_op("transpose_grad", ["X?", "Out?", "Out@GRAD"], ["X@GRAD"], {"axis": []}, grad=None,
            no_infer=True)(_transpose_grad)
register_op("transpose2_grad", ["X?", "Out?", "XShape?", "Out@GRAD"], ["X@GRAD"], {"axis": []}, grad=None,
            no_infer=True)(_transpose_grad)


@register_op("concat", ["X*"], ["Out"], {"axis": 0})
def concat(ctx):
    xs = [t for t in ctx.inputs("X") if t is not None]
    ax = ctx.attr("axis")
    out = _oplib.concat_op(xs, ax) if xs and xs[0].is_cuda else None
    if out is None:
        out = torch.cat(xs, ax)
    lod = None
    if ax == 0:
        lods = [v.lod() for v in ctx.input_values("X")]
        if all(lods) and len(lods[0]) == 1:
            off = [0]
            for l in lods:
                base = off[-1]
                off += [base + o for o in l[0][1:]]
            lod = [off]
    ctx.set_output("Out", out, lod)


@register_op("split", ["X"], ["Out*"], {"num": 0, "sections": [], "axis": 0})
def split(ctx):
    x = ctx.input("X")
    ax = ctx.attr("axis")
    secs = ctx.attr("sections")
    if secs:
        secs = list(secs)
        if -1 in secs:
            i = secs.index(-1)
            secs[i] = x.shape[ax] - (sum(secs) + 1)
    else:
        n = ctx.attr("num") or len(ctx.output_names("Out"))
        secs = [c.shape[0] for c in torch.chunk(torch.empty(x.shape[ax], device="meta"), n, 0)] \
            if x.shape[ax] else [0] * n
    parts = _oplib.split_op(x, secs, ax) if x.is_cuda else None
    if parts is None:
        parts = torch.split(x, secs, ax)
    ctx.set_outputs("Out", list(parts))


@register_op("split_byref", ["X"], ["Out*"], {"sections": [], "num": 0})
def split_byref(ctx):
    x = ctx.input("X")
    secs = ctx.attr("sections") or [x.shape[0] // len(ctx.output_names("Out"))] * len(ctx.output_names("Out"))
    ctx.set_outputs("Out", list(torch.split(x, secs, 0)))


@register_op("stack", ["X*"], ["Y"], {"axis": 0})
def stack(ctx):
    ctx.set_output("Y", torch.stack(ctx.inputs("X"), ctx.attr("axis")))


@register_op("unstack", ["X"], ["Y*"], {"axis": 0, "num": 0})
def unstack(ctx):
    ctx.set_outputs("Y", list(torch.unbind(ctx.input("X"), ctx.attr("axis"))))


@register_op("expand", ["X"], ["Out"], {"expand_times": []})
def expand(ctx):
    x, reps = ctx.input("X"), list(ctx.attr("expand_times"))
    if _dev(ctx, x) and len(reps) == x.dim() and 2 * x.dim() <= 8:
        ctx.set_output("Out", _fk.tile(x, reps))
        return
    ctx.set_output("Out", x.repeat(*reps))


@register_op("expand_grad", ["X", "Out?", "Out@GRAD"], ["X@GRAD"], {"expand_times": []}, grad=None, no_infer=True)
def expand_grad(ctx):
    x, g = ctx.input("X"), ctx.input("Out@GRAD")
    reps = list(ctx.attr("expand_times"))
    shp = []
    for n, r in zip(x.shape, reps):
        shp += [r, n]
    red = tuple(range(0, 2 * x.dim(), 2))
    ctx.set_output("X@GRAD", g.reshape(shp).sum(red) if red else g.clone())


@register_op("gather", ["X", "Index"], ["Out"], {})
def gather(ctx):
    x, idx = ctx.input("X"), ctx.input("Index")
    ctx.set_output("Out", x.index_select(0, idx.reshape(-1).long()))


@register_op("scatter", ["X", "Ids", "Updates"], ["Out"], {"overwrite": True})
def scatter(ctx):
    x, ids, up = ctx.input("X"), ctx.input("Ids").reshape(-1).long(), ctx.input("Updates")
    out = x.clone()
    if ctx.attr("overwrite"):
        out[ids] = up
    else:
        out.index_add_(0, ids, up)
    ctx.set_output("Out", out)


@register_op("slice", ["Input"], ["Out"], {"axes": [], "starts": [], "ends": []})
def slice_op(ctx):
    x = ctx.input("Input")
    sl = [slice(None)] * x.dim()
    for a, s, e in zip(ctx.attr("axes"), ctx.attr("starts"), ctx.attr("ends")):
        n = x.shape[a]
        s = max(0, s + n if s < 0 else min(s, n))
        e = max(0, e + n if e < 0 else min(e, n))
        sl[a] = slice(s, e)
    if _dev(ctx, x) and 0 < x.dim() <= 8:
        ctx.set_output("Out", _fk.slice_(x, list(ctx.attr("axes")), list(ctx.attr("starts")),
                                         list(ctx.attr("ends"))))
        return
    ctx.set_output("Out", x[tuple(sl)])


@register_op("slice_grad", ["Input", "Out?", "Out@GRAD"], ["Input@GRAD"], {"axes": [], "starts": [], "ends": []},
             grad=None, no_infer=True)
def slice_grad(ctx):
    x, g = ctx.input("Input"), ctx.input("Out@GRAD")
    sl = [slice(None)] * x.dim()
    for a, s, e in zip(ctx.attr("axes"), ctx.attr("starts"), ctx.attr("ends")):
        n = x.shape[a]
        s = max(0, s + n if s < 0 else min(s, n))
        e = max(0, e + n if e < 0 else min(e, n))
        sl[a] = slice(s, e)
    gx = torch.zeros_like(x, dtype=g.dtype)
    gx[tuple(sl)] = g
    ctx.set_output("Input@GRAD", gx)


@register_op("reverse", ["X"], ["Out"], {"axis": []})
def reverse(ctx):
    x = ctx.input("X")
    if _dev(ctx, x) and 0 < x.dim() <= 8:
        ctx.set_output("Out", _fk.flip(x, list(ctx.attr("axis"))))
        return
    ctx.set_output("Out", torch.flip(x, list(ctx.attr("axis"))))


@register_op("reverse_grad", ["X?", "Out?", "Out@GRAD"], ["X@GRAD"], {"axis": []}, grad=None, no_infer=True)
def reverse_grad(ctx):
    g = ctx.input("Out@GRAD")
    if _dev(ctx, g) and 0 < g.dim() <= 8:
        ctx.set_output("X@GRAD", _fk.flip(g, list(ctx.attr("axis"))))
        return
    ctx.set_output("X@GRAD", torch.flip(g, list(ctx.attr("axis"))))


def _cast(ctx, x, dt):
    if _dev(ctx, x):
        return _fk.cast(x, dt)
    return x.to(dt)


@register_op("cast", ["X"], ["Out"], {"in_dtype": 5, "out_dtype": 5})
def cast(ctx):
    ctx.set_output("Out", _cast(ctx, ctx.input("X"), core.to_torch_dtype(ctx.attr("out_dtype"))),
                   ctx.input_lod("X"))


@register_op("cast_grad", ["X", "Out?", "Out@GRAD"], ["X@GRAD"], {"in_dtype": 5, "out_dtype": 5}, grad=None,
             no_infer=True)
def cast_grad(ctx):
    x, g = ctx.input("X"), ctx.input("Out@GRAD")
    ctx.set_output("X@GRAD", _cast(ctx, g, x.dtype))


@register_op("shape", ["Input"], ["Out"], {}, grad=None)
def shape_op(ctx):
    x = ctx.input("Input")
    ctx.set_output("Out", torch.tensor(list(x.shape), dtype=torch.int32, device="cpu" if ctx.meta else x.device)
                   if not ctx.meta else torch.empty(x.dim(), dtype=torch.int32, device="meta"))


@register_op("assign", ["X"], ["Out"], {})
def assign(ctx):
    v = ctx.input_value("X")
    if isinstance(v, core.LoDTensor):
        ctx.set_output("Out", v.tensor.clone(), v.lod())
    else:
        ctx.set_output("Out", v)


@register_op("assign_value", [], ["Out"], {"shape": [], "dtype": 5, "fp32_values": [], "int32_values": []},
             grad=None)
def assign_value(ctx):
    dt = core.to_torch_dtype(ctx.attr("dtype"))
    vals = ctx.attr("fp32_values") or ctx.attr("int32_values")
    ctx.set_output("Out", torch.tensor(vals, dtype=dt, device=ctx.device).reshape(ctx.attr("shape"))
                   if not ctx.meta else torch.empty(ctx.attr("shape"), dtype=dt, device="meta"))


def _full(ctx, shape, value, dtype):
    dev = ctx.device
    if ctx.attr("force_cpu", False) and not ctx.meta:
        dev = torch.device("cpu")
    return torch.full([int(s) for s in shape], value, dtype=core.to_torch_dtype(dtype), device=dev)


@register_op("fill_constant", [], ["Out"], {"shape": [], "dtype": 5, "value": 0.0, "force_cpu": False}, grad=None)
def fill_constant(ctx):
    ctx.set_output("Out", _full(ctx, ctx.attr("shape"), ctx.attr("value"), ctx.attr("dtype")))


@register_op("fill", [], ["Out"], {"shape": [], "dtype": 5, "value": [], "force_cpu": False}, grad=None)
def fill(ctx):
    dt = core.to_torch_dtype(ctx.attr("dtype"))
    ctx.set_output("Out", torch.tensor(ctx.attr("value"), dtype=dt, device=ctx.device).reshape(ctx.attr("shape")))


@register_op("fill_zeros_like", ["X"], ["Out"], {}, grad=None)
def fill_zeros_like(ctx):
    ctx.set_output("Out", torch.zeros_like(ctx.input("X")))


def _batch_like_shape(ctx):
    shape = list(ctx.attr("shape"))
    x = ctx.input("Input")
    shape[ctx.attr("output_dim_idx")] = x.shape[ctx.attr("input_dim_idx")]
    return shape


@register_op("fill_constant_batch_size_like", ["Input"], ["Out"],
             {"shape": [], "dtype": 5, "value": 0.0, "input_dim_idx": 0, "output_dim_idx": 0}, grad=None)
def fill_constant_batch_size_like(ctx):
    ctx.set_output("Out", _full(ctx, _batch_like_shape(ctx), ctx.attr("value"), ctx.attr("dtype")))


def _gen(ctx):
    seed = ctx.attr("seed", 0)
    if ctx.meta or not seed:
        return None
    g = torch.Generator(device=ctx.device)
    g.manual_seed(int(seed))
    return g


def _philox(ctx, shape, kind, a, b):
    """Counter-based Philox4x32-10 fill on the device (csrc/kernels/fluid_ops.hip):
    op seed when set, else a draw from the host generator (paddle.seed / torch.manual_seed)."""
    dt = core.to_torch_dtype(ctx.attr("dtype"))
    if ctx.meta or ctx.device.type != "cuda" or dt not in (torch.float32, torch.bfloat16):
        return None
    seed = int(ctx.attr("seed", 0)) or int(torch.randint(1, 2 ** 62, (1,)).item())
    return _fk.random(shape, kind, a, b, seed, dtype=dt, device=ctx.device)


@register_op("uniform_random", [], ["Out"], {"shape": [], "min": -1.0, "max": 1.0, "seed": 0, "dtype": 5},
             grad=None)
def uniform_random(ctx):
    dt = core.to_torch_dtype(ctx.attr("dtype"))
    shape = [int(s) for s in ctx.attr("shape")]
    t = _philox(ctx, shape, "uniform", ctx.attr("min"), ctx.attr("max"))
    if t is not None:
        ctx.set_output("Out", t)
        return
    t = torch.empty(shape, dtype=torch.float32, device=ctx.device)
    if not ctx.meta:
        t.uniform_(ctx.attr("min"), ctx.attr("max"), generator=_gen(ctx))
    ctx.set_output("Out", t.to(dt))


@register_op("uniform_random_batch_size_like", ["Input"], ["Out"],
             {"shape": [], "min": -1.0, "max": 1.0, "seed": 0, "dtype": 5, "input_dim_idx": 0,
              "output_dim_idx": 0}, grad=None)
def uniform_random_bsl(ctx):
    t = torch.empty(_batch_like_shape(ctx), dtype=torch.float32, device=ctx.device)
    if not ctx.meta:
        t.uniform_(ctx.attr("min"), ctx.attr("max"), generator=_gen(ctx))
    ctx.set_output("Out", t.to(core.to_torch_dtype(ctx.attr("dtype"))))


@register_op("gaussian_random", [], ["Out"], {"shape": [], "mean": 0.0, "std": 1.0, "seed": 0, "dtype": 5,
                                              "use_mkldnn": False}, grad=None)
def gaussian_random(ctx):
    shape = [int(s) for s in ctx.attr("shape")]
    t = _philox(ctx, shape, "gaussian", ctx.attr("mean"), ctx.attr("std"))
    if t is not None:
        ctx.set_output("Out", t)
        return
    t = torch.empty(shape, dtype=torch.float32, device=ctx.device)
    if not ctx.meta:
        t.normal_(ctx.attr("mean"), ctx.attr("std"), generator=_gen(ctx))
    ctx.set_output("Out", t.to(core.to_torch_dtype(ctx.attr("dtype"))))


@register_op("gaussian_random_batch_size_like", ["Input"], ["Out"],
             {"shape": [], "mean": 0.0, "std": 1.0, "seed": 0, "dtype": 5, "input_dim_idx": 0,
              "output_dim_idx": 0}, grad=None)
def gaussian_random_bsl(ctx):
    t = torch.empty(_batch_like_shape(ctx), dtype=torch.float32, device=ctx.device)
    if not ctx.meta:
        t.normal_(ctx.attr("mean"), ctx.attr("std"), generator=_gen(ctx))
    ctx.set_output("Out", t.to(core.to_torch_dtype(ctx.attr("dtype"))))


@register_op("truncated_gaussian_random", [], ["Out"], {"shape": [], "mean": 0.0, "std": 1.0, "seed": 0,
                                                        "dtype": 5}, grad=None)
def truncated_gaussian_random(ctx):
    t = torch.empty([int(s) for s in ctx.attr("shape")], dtype=torch.float32, device=ctx.device)
    if not ctx.meta:
        m, s = ctx.attr("mean"), ctx.attr("std")
        torch.nn.init.trunc_normal_(t, m, s, m - 2 * s, m + 2 * s)
    ctx.set_output("Out", t.to(core.to_torch_dtype(ctx.attr("dtype"))))


@register_op("sampling_id", ["X"], ["Out"], {"min": 0.0, "max": 1.0, "seed": 0}, grad=None)
def sampling_id(ctx):
    x = ctx.input("X")
    ctx.set_output("Out", torch.multinomial(x.float(), 1, generator=_gen(ctx)).reshape(-1) if not ctx.meta
                   else torch.empty(x.shape[0], dtype=torch.int64, device="meta"))


@register_op("random_crop", ["X", "Seed"], ["Out", "SeedOut~"], {"shape": [], "startup_seed": 0}, grad=None)
def random_crop(ctx):
    x = ctx.input("X")
    shape = ctx.attr("shape")
    k = len(shape)
    lead = x.dim() - k
    sl = [slice(None)] * lead
    for i, s in enumerate(shape):
        n = x.shape[lead + i]
        st = int(torch.randint(0, n - s + 1, (1,)).item()) if not ctx.meta else 0
        sl.append(slice(st, st + s))
    ctx.set_output("Out", x[tuple(sl)])
    ctx.set_output("SeedOut", ctx.input("Seed"))


@register_op("multiplex", ["Ids", "X*"], ["Out"], {})
def multiplex(ctx):
    ids = ctx.input("Ids").reshape(-1).long()
    xs = torch.stack(ctx.inputs("X"))  # K, N, ...
    K, Nr = xs.shape[0], xs.shape[1]
    # row i of candidate ids[i]: one row gather of the stacked [K*N, ...] rows
    rows = ids * Nr + torch.arange(Nr, device=xs.device)
    ctx.set_output("Out", xs.reshape(K * Nr, -1).index_select(0, rows).reshape(xs.shape[1:]))


def _cmp(name, fn):
    @register_op(name, ["X", "Y"], ["Out"], {"axis": -1, "force_cpu": False}, grad=None)
    def k(ctx):
        x, y = ctx.input("X"), ctx.input("Y")
        if x.device != y.device:
            # loop counters / array lengths live on the host: compare scalars there (the
            # While condition is read on the host anyway), else follow the larger operand
            if x.numel() == 1 and y.numel() == 1:
                x, y = x.cpu(), y.cpu()
            elif x.numel() >= y.numel():
                y = y.to(x.device)
            else:
                x = x.to(y.device)
        ctx.set_output("Out", fn(x, y.to(x.dtype) if y.dtype != x.dtype else y))


for _n, _f in {"less_than": torch.lt, "less_equal": torch.le, "greater_than": torch.gt,
               "greater_equal": torch.ge, "equal": torch.eq, "not_equal": torch.ne}.items():
    _cmp(_n, _f)


def _logic(name, fn, unary=False):
    @register_op(name, ["X"] if unary else ["X", "Y"], ["Out"], {}, grad=None)
    def k(ctx):
        x = ctx.input("X").bool()
        ctx.set_output("Out", fn(x) if unary else fn(x, ctx.input("Y").bool()))


_logic("logical_and", torch.logical_and)
_logic("logical_or", torch.logical_or)
_logic("logical_xor", torch.logical_xor)
_logic("logical_not", torch.logical_not, unary=True)


@register_op("increment", ["X"], ["Out"], {"step": 1.0}, grad=None)
def increment(ctx):
    x = ctx.input("X")
    ctx.set_output("Out", x + torch.tensor(ctx.attr("step"), dtype=x.dtype, device=x.device))


@register_op("is_empty", ["X"], ["Out"], {}, grad=None)
def is_empty(ctx):
    x = ctx.input("X")
    ctx.set_output("Out", torch.tensor([x.numel() == 0], device="cpu" if not ctx.meta else "meta"))


@register_op("arg_max", ["X"], ["Out"], {"axis": 0}, grad=None)
def arg_max(ctx):
    ctx.set_output("Out", torch.argmax(ctx.input("X"), ctx.attr("axis")))


@register_op("arg_min", ["X"], ["Out"], {"axis": 0}, grad=None)
def arg_min(ctx):
    ctx.set_output("Out", torch.argmin(ctx.input("X"), ctx.attr("axis")))


@register_op("argsort", ["X"], ["Out", "Indices"], {"axis": -1}, grad=None)
def argsort(ctx):
    x = ctx.input("X")
    r = _oplib.argsort_op(x, ctx.attr("axis")) if x.is_cuda else None
    v, i = r if r is not None else torch.sort(x, ctx.attr("axis"))
    ctx.set_output("Out", v)
    ctx.set_output("Indices", i)


@register_op("print", ["In"], ["Out?"], {"first_n": -1, "message": "", "summarize": -1, "print_tensor_name": True,
                                         "print_tensor_type": True, "print_tensor_shape": True,
                                         "print_tensor_lod": True, "print_phase": "BOTH"}, no_infer=True)
def print_op(ctx):
    v = ctx.input_value("In")
    t = v.tensor if isinstance(v, core.LoDTensor) else v
    msg = ctx.attr("message")
    n = ctx.attr("summarize")
    flat = t.reshape(-1)
    data = flat[:n] if n > 0 else flat
    print(f"{msg} {ctx.op.input('In')[0] if ctx.op else ''} shape={list(t.shape)} "
          f"lod={v.lod() if isinstance(v, core.LoDTensor) else []} data={data.tolist()}")
    if ctx.has_output("Out"):
        ctx.set_output("Out", t, v.lod() if isinstance(v, core.LoDTensor) else None)


@register_op("delete_var", ["X*"], [], {}, grad=None, no_infer=True)
def delete_var(ctx):
    if ctx.scope is not None and ctx.op is not None:
        ctx.scope.erase(ctx.op.input("X"))


@register_op("shuffle_channel", ["X"], ["Out"], {"group": 1})
def shuffle_channel(ctx):
    x = ctx.input("X")
    g = ctx.attr("group")
    N, C, H, W = x.shape
    ctx.set_output("Out", x.reshape(N, g, C // g, H, W).transpose(1, 2).reshape(N, C, H, W))


@register_op("where_index", ["Condition"], ["Out"], {}, grad=None, no_infer=True)
def where_index(ctx):
    ctx.set_output("Out", torch.nonzero(ctx.input("Condition")))


@register_op("size", ["Input"], ["Out"], {}, grad=None)
def size_op(ctx):
    x = ctx.input("Input")
    ctx.set_output("Out", torch.tensor([x.numel()], dtype=torch.int64, device=x.device) if not ctx.meta else
                   torch.empty(1, dtype=torch.int64, device="meta"))
