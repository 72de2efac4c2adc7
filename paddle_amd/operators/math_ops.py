"""Dense math operators: mul/matmul, elementwise (+broadcast), activations, reductions.

Parity: paddle/fluid/operators/{mul,matmul,elementwise_*,activation,scale,sum,mean,
reduce_*,clip,clip_by_norm,cumsum,minus,sign,l1_norm,squared_l2_norm,
squared_l2_distance,cos_sim,norm}_op.* (SURVEY §2.7 "Dense NN / math").
On the HIP device mul / matmul / fc run on the framework's exact-fp32 MFMA GEMM
(``ops/blas.py`` -> ``csrc/kernels/convnd.hip``; bf16 on ``gemm.hip``), and the
elementwise / activation / reduction expressions of the other kernels run on the
generic strided kernels of ``csrc/kernels/tensor_ops.hip`` (native dispatch inside
the executor's op region, ``ops/aten_native.py``).  Shapes the native GEMM does not
cover fall back to ATen and are counted by ``utils/strict.py``.  Gradients of ops without an
explicit ``*_grad`` kernel come from the registry's automatic VJP.
"""
from __future__ import annotations

import math

import torch

import torch.nn.functional as F

from ..framework import core
from ..framework.registry import register_op
from ..ops import blas as _blas
from ..ops import fluidk as _fk
from ..ops import oplib as _oplib

# ------------------------------------------------------------------ mul / matmul


def _flat2(t, k):
    return t.reshape(int(math.prod(t.shape[:k])), int(math.prod(t.shape[k:])))


@register_op("mul", ["X", "Y"], ["Out"], {"x_num_col_dims": 1, "y_num_col_dims": 1})
def mul(ctx):
    """Out = flatten(X, x_num_col_dims) @ flatten(Y, y_num_col_dims)."""
    x, y = ctx.input("X"), ctx.input("Y")
    xn, yn = ctx.attr("x_num_col_dims"), ctx.attr("y_num_col_dims")
    x2, y2 = _flat2(x, xn), _flat2(y, yn).to(x.dtype)
    out = _blas.matmul(x2, y2) if _blas.supported(x2, y2) else x2 @ y2
    ctx.set_output("Out", out.reshape(tuple(x.shape[:xn]) + tuple(y.shape[yn:])))


@register_op("fc", ["Input", "W", "Bias?"], ["Out"], {"in_num_col_dims": 1, "activation_type": ""})
def fc(ctx):
    """Fused fully-connected op produced by ``fc_fuse_pass`` (reference fc_op.cc:154):
    Out = act(flatten(Input, in_num_col_dims) @ W + Bias).  On the HIP device the
    bias rides the epilogue of the native MFMA GEMM (``ops/blas.py`` fc); the
    activation is one pass of the native elementwise kernels."""
    x, w = ctx.input("Input"), ctx.input("W")
    n = ctx.attr("in_num_col_dims")
    x2 = _flat2(x, n)
    w = w.to(x2.dtype)
    act = ctx.attr("activation_type") or ""
    if ctx.has_input("Bias") and _blas.supported(x2, w):
        out = _blas.fc(x2, w, ctx.input("Bias").reshape(-1).to(x2.dtype))
    elif not ctx.has_input("Bias") and _blas.supported(x2, w):
        out = _blas.matmul(x2, w)
    elif ctx.has_input("Bias"):
        b = ctx.input("Bias").reshape(-1).to(x2.dtype)
        if act in ("relu", "gelu") and x2.is_cuda:
            out = torch._addmm_activation(b, x2, w, use_gelu=(act == "gelu"))
            act = ""
        else:
            out = torch.addmm(b, x2, w)
    else:
        out = x2 @ w
    if act:
        out = {"relu": torch.relu, "gelu": torch.nn.functional.gelu, "tanh": torch.tanh,
               "sigmoid": torch.sigmoid}[act](out)
    ctx.set_output("Out", out.reshape(tuple(x.shape[:n]) + (w.shape[1],)), ctx.input_lod("Input"))


@register_op("mul_grad", ["X", "Y", "Out?", "Out@GRAD"], ["X@GRAD?", "Y@GRAD?"],
             {"x_num_col_dims": 1, "y_num_col_dims": 1}, grad=None, no_infer=True)
def mul_grad(ctx):
    x, y, dout = ctx.input("X"), ctx.input("Y"), ctx.input("Out@GRAD")
    xn, yn = ctx.attr("x_num_col_dims"), ctx.attr("y_num_col_dims")
    x2, y2 = _flat2(x, xn), _flat2(y, yn)
    d2 = dout.reshape(x2.shape[0], y2.shape[1])
    mm = (lambda a, b: _blas.matmul(a, b)) if _blas.supported(x2, y2) and d2.dtype == x2.dtype else \
        (lambda a, b: a @ b)
    if ctx.has_output("X@GRAD"):
        ctx.set_output("X@GRAD", mm(d2, y2.t()).reshape(x.shape), ctx.input_lod("X"))
    if ctx.has_output("Y@GRAD"):
        ctx.set_output("Y@GRAD", mm(x2.t(), d2).reshape(y.shape))


@register_op("matmul", ["X", "Y"], ["Out"], {"transpose_X": False, "transpose_Y": False, "alpha": 1.0})
def matmul(ctx):
    x, y = ctx.input("X"), ctx.input("Y")
    tx, ty = ctx.attr("transpose_X"), ctx.attr("transpose_Y")
    x1, y1 = x.dim() == 1, y.dim() == 1
    if x1:
        x = x.unsqueeze(0) if not tx else x.unsqueeze(1)
    if y1:
        y = y.unsqueeze(1) if not ty else y.unsqueeze(0)
    if tx:
        x = x.transpose(-1, -2)
    if ty:
        y = y.transpose(-1, -2)
    a = ctx.attr("alpha")
    if _blas.supported(x, y):  # strided views: the transposes cost nothing
        out = _blas.matmul(x, y, a)
    else:
        out = torch.matmul(x, y)
        if a != 1.0:
            out = out * a
    if x1:
        out = out.squeeze(-2)
    if y1:
        out = out.squeeze(-1)
    if out.dim() == 0:
        out = out.reshape(1)
    ctx.set_output("Out", out)


# ------------------------------------------------------------------ elementwise


def bcast_y(x, y, axis):
    """Reference broadcast (elementwise_op_function.h): Y's dims align with X starting
    at ``axis`` (-1: trailing alignment); trailing singular dims of Y are trimmed."""
    if x.shape == y.shape or y.dim() == 0:
        return y
    ys = list(y.shape)
    if axis is None or axis < 0:
        axis = x.dim() - len(ys)
    while ys and ys[-1] == 1:
        ys.pop()
    shape = [1] * axis + ys + [1] * (x.dim() - axis - len(ys))
    return y.reshape(shape)


def _reduce_to(g, shape):
    """Sum a broadcast gradient back to ``shape`` (reference ElemwiseGradBroadcast kernels)."""
    if tuple(g.shape) == tuple(shape):
        return g
    n = int(math.prod(shape)) if shape else 1
    # find the matching alignment: try every axis offset
    gs = list(g.shape)
    for axis in range(0, len(gs) - len(shape) + 1):
        if all(gs[axis + i] == shape[i] or shape[i] == 1 for i in range(len(shape))):
            dims = list(range(axis)) + list(range(axis + len(shape), len(gs)))
            r = g.sum(dim=dims) if dims else g
            keep = [i for i in range(len(shape)) if shape[i] == 1 and r.shape[i] != 1]
            if keep:
                r = r.sum(dim=keep, keepdim=True)
            return r.reshape(shape)
    return g.sum().reshape(shape) if n == 1 else g.reshape(shape)


_EW = {
    "elementwise_add": lambda a, b: a + b,
    "elementwise_sub": lambda a, b: a - b,
    "elementwise_mul": lambda a, b: a * b,
    "elementwise_div": lambda a, b: a / b,
    "elementwise_max": torch.maximum,
    "elementwise_min": torch.minimum,
    "elementwise_pow": torch.pow,
    "elementwise_mod": torch.remainder,
    "elementwise_floordiv": lambda a, b: torch.div(a, b, rounding_mode="floor"),
}


_EW_NATIVE = {"elementwise_add": "add", "elementwise_sub": "sub", "elementwise_mul": "mul",
              "elementwise_div": "div", "elementwise_max": "max", "elementwise_min": "min",
              "elementwise_pow": "pow"}


def _make_ew(name, fn):
    @register_op(name, ["X", "Y"], ["Out"], {"axis": -1, "use_mkldnn": False})
    def k(ctx):
        x, y = ctx.input("X"), ctx.input("Y")
        if x.device != y.device:  # data transform: a host scalar (force_cpu counter) joins the other place
            if y.numel() <= x.numel():
                y = y.to(x.device)
            else:
                x = x.to(y.device)
        yb = bcast_y(x, y, ctx.attr("axis")).to(x.dtype)
        out = _oplib.ew(_EW_NATIVE[name], x, yb) if (x.is_cuda and name in _EW_NATIVE) else None
        ctx.set_output("Out", out if out is not None else fn(x, yb))

    k.__name__ = name
    return k


for _n, _f in _EW.items():
    _make_ew(_n, _f)


def _ew_grad(name, dx_fn, dy_fn):
    @register_op(name + "_grad", ["X", "Y", "Out?", "Out@GRAD"], ["X@GRAD?", "Y@GRAD?"], {"axis": -1},
                 grad=None, no_infer=True)
    def k(ctx):
        x, y, d = ctx.input("X"), ctx.input("Y"), ctx.input("Out@GRAD")
        yb = bcast_y(x, y, ctx.attr("axis")).to(x.dtype)
        if x.is_cuda and yb.dim() == x.dim() and not (x.requires_grad or yb.requires_grad):
            # native: the same broadcast kernels forward and backward, broadcast
            # gradients summed by the reduce kernel (ElemwiseGradBroadcast)
            with torch.no_grad():
                res = _oplib._BinaryFn.backward(_NativeGradCtx(name, x, yb), d.to(x.dtype).contiguous()) \
                    if _oplib._ok(x, yb, d) and x.dtype == yb.dtype else None
            if res is not None and res[1] is not None:
                if ctx.has_output("X@GRAD"):
                    ctx.set_output("X@GRAD", res[1], ctx.input_lod("X"))
                if ctx.has_output("Y@GRAD"):
                    ctx.set_output("Y@GRAD", res[2].reshape(y.shape).to(y.dtype))
                return
        if ctx.has_output("X@GRAD"):
            ctx.set_output("X@GRAD", _reduce_to(dx_fn(x, yb, d), x.shape), ctx.input_lod("X"))
        if ctx.has_output("Y@GRAD"):
            # sum over the dims Y was broadcast along, in Y's aligned (op-axis) layout;
            # matching Y's raw shape against the gradient instead is ambiguous when two
            # dims have Y's size (bias [16] of a [16, 16] activation)
            g = dy_fn(x, yb, d)
            if g.dim() == yb.dim():
                dims = [i for i in range(g.dim()) if yb.shape[i] == 1 and g.shape[i] != 1]
                g = g.sum(dim=dims, keepdim=True) if dims else g
                ctx.set_output("Y@GRAD", g.reshape(y.shape).to(y.dtype))
            else:
                ctx.set_output("Y@GRAD", _reduce_to(g, y.shape).to(y.dtype))


class _NativeGradCtx:
    """Stands in for an autograd ctx so the grad op reuses ``_BinaryFn.backward``."""

    def __init__(self, name, x, y):
        self.op = name[len("elementwise_"):]
        self.saved_tensors = (x, y)
        self.needs_input_grad = (False, True, True)


_ew_grad("elementwise_add", lambda x, y, d: d, lambda x, y, d: d)
_ew_grad("elementwise_sub", lambda x, y, d: d, lambda x, y, d: -d)
_ew_grad("elementwise_mul", lambda x, y, d: d * y, lambda x, y, d: d * x)
_ew_grad("elementwise_div", lambda x, y, d: d / y, lambda x, y, d: -d * x / (y * y))


# ------------------------------------------------------------------ activations
# name -> (attrs, (a, b) from attrs, forward f(x, a, b), derivative df(x, y, a, b))
# GPU: one templated HIP kernel pair (csrc/kernels/fluid_ops.hip, ops/fluidk.py);
# CPU: the same formulas in torch.  Every activation has an explicit grad op
# ``<name>_grad`` (X, Out, Out@GRAD -> X@GRAD), reference activation_op.h:877-906.
def _sg(x):
    return torch.sigmoid(x)


_ACT = {
    "relu": ({}, None, lambda x, a, b: F.relu(x), lambda x, y, a, b: (y > 0).to(x.dtype)),
    "sigmoid": ({}, None, lambda x, a, b: torch.sigmoid(x), lambda x, y, a, b: y * (1 - y)),
    "logsigmoid": ({}, None, lambda x, a, b: F.logsigmoid(x), lambda x, y, a, b: _sg(-x)),
    "exp": ({}, None, lambda x, a, b: torch.exp(x), lambda x, y, a, b: y),
    "tanh": ({}, None, lambda x, a, b: torch.tanh(x), lambda x, y, a, b: 1 - y * y),
    "tanh_shrink": ({}, None, lambda x, a, b: x - torch.tanh(x), lambda x, y, a, b: torch.tanh(x) ** 2),
    "softshrink": ({"lambda": 0.5}, ("lambda", None), lambda x, a, b: F.softshrink(x, a),
                   lambda x, y, a, b: (x.abs() > a).to(x.dtype)),
    "sqrt": ({}, None, lambda x, a, b: torch.sqrt(x), lambda x, y, a, b: 0.5 / y),
    "rsqrt": ({}, None, lambda x, a, b: torch.rsqrt(x), lambda x, y, a, b: -0.5 * y * y * y),
    "abs": ({}, None, lambda x, a, b: torch.abs(x), lambda x, y, a, b: torch.sign(x)),
    "ceil": ({}, None, lambda x, a, b: torch.ceil(x), lambda x, y, a, b: torch.zeros_like(x)),
    "floor": ({}, None, lambda x, a, b: torch.floor(x), lambda x, y, a, b: torch.zeros_like(x)),
    "cos": ({}, None, lambda x, a, b: torch.cos(x), lambda x, y, a, b: -torch.sin(x)),
    "sin": ({}, None, lambda x, a, b: torch.sin(x), lambda x, y, a, b: torch.cos(x)),
    "round": ({}, None, lambda x, a, b: torch.round(x), lambda x, y, a, b: torch.zeros_like(x)),
    "reciprocal": ({}, None, lambda x, a, b: torch.reciprocal(x), lambda x, y, a, b: -y * y),
    "log": ({}, None, lambda x, a, b: torch.log(x), lambda x, y, a, b: 1 / x),
    "square": ({}, None, lambda x, a, b: x * x, lambda x, y, a, b: 2 * x),
    "softplus": ({}, None, lambda x, a, b: F.softplus(x), lambda x, y, a, b: _sg(x)),
    "softsign": ({}, None, lambda x, a, b: F.softsign(x), lambda x, y, a, b: 1 / (1 + x.abs()) ** 2),
    "brelu": ({"t_min": 0.0, "t_max": 24.0}, ("t_min", "t_max"), lambda x, a, b: torch.clamp(x, a, b),
              lambda x, y, a, b: ((x > a) & (x < b)).to(x.dtype)),
    "leaky_relu": ({"alpha": 0.02}, ("alpha", None), lambda x, a, b: F.leaky_relu(x, a),
                   lambda x, y, a, b: torch.where(x > 0, torch.ones_like(x), torch.full_like(x, a))),
    "soft_relu": ({"threshold": 40.0}, ("threshold", None),
                  lambda x, a, b: torch.log1p(torch.exp(torch.clamp(x, -a, a))),
                  lambda x, y, a, b: ((x > -a) & (x < a)).to(x.dtype) * (1 - torch.exp(-y))),
    "elu": ({"alpha": 1.0}, ("alpha", None), lambda x, a, b: F.elu(x, a),
            lambda x, y, a, b: torch.where(x > 0, torch.ones_like(x), y + a)),
    "relu6": ({"threshold": 6.0}, ("threshold", None), lambda x, a, b: torch.clamp(x, 0.0, a),
              lambda x, y, a, b: ((x > 0) & (x < a)).to(x.dtype)),
    "pow": ({"factor": 1.0}, ("factor", None), lambda x, a, b: torch.pow(x, a),
            lambda x, y, a, b: a * torch.pow(x, a - 1)),
    "stanh": ({"scale_a": 2.0 / 3.0, "scale_b": 1.7159}, ("scale_a", "scale_b"),
              lambda x, a, b: b * torch.tanh(a * x), lambda x, y, a, b: a * b * (1 - torch.tanh(a * x) ** 2)),
    "hard_shrink": ({"threshold": 0.5}, ("threshold", None), lambda x, a, b: F.hardshrink(x, a),
                    lambda x, y, a, b: (x.abs() > a).to(x.dtype)),
    "thresholded_relu": ({"threshold": 1.0}, ("threshold", None),
                         lambda x, a, b: torch.where(x > a, x, torch.zeros_like(x)),
                         lambda x, y, a, b: (x > a).to(x.dtype)),
    "hard_sigmoid": ({"slope": 0.2, "offset": 0.5}, ("slope", "offset"),
                     lambda x, a, b: torch.clamp(x * a + b, 0.0, 1.0),
                     lambda x, y, a, b: (((x * a + b) > 0) & ((x * a + b) < 1)).to(x.dtype) * a),
    "swish": ({"beta": 1.0}, ("beta", None), lambda x, a, b: x * torch.sigmoid(a * x),
              lambda x, y, a, b: _sg(a * x) + a * x * _sg(a * x) * (1 - _sg(a * x))),
    "gelu": ({}, None, lambda x, a, b: F.gelu(x),
             lambda x, y, a, b: 0.5 * (1 + torch.erf(x / math.sqrt(2.0))) + x * torch.exp(-0.5 * x * x) /
             math.sqrt(2 * math.pi)),
    "silu": ({}, None, lambda x, a, b: F.silu(x), lambda x, y, a, b: _sg(x) * (1 + x * (1 - _sg(x)))),
}


def _act_ab(ctx, keys):
    if keys is None:
        return 0.0, 0.0
    ka, kb = keys
    return float(ctx.attr(ka)) if ka else 0.0, float(ctx.attr(kb)) if kb else 0.0


def _make_act(name, attrs, keys, fwd, dfn):
    @register_op(name, ["X"], ["Out"], dict(attrs, use_mkldnn=False, use_cudnn=False, is_test=False))
    def k(ctx):
        x = ctx.input("X")
        a, b = _act_ab(ctx, keys)
        if _fk.ok(x) and not ctx.meta:
            ctx.set_output("Out", _fk.act_fwd(name, x, a, b))
        else:
            ctx.set_output("Out", fwd(x, a, b))

    @register_op(name + "_grad", ["X?", "Out?", "Out@GRAD"], ["X@GRAD"], dict(attrs), grad=None, no_infer=True)
    def kg(ctx):
        d = ctx.input("Out@GRAD")
        x = ctx.input("X") if ctx.has_input("X") else None
        y = ctx.input("Out") if ctx.has_input("Out") else None
        a, b = _act_ab(ctx, keys)
        if _fk.ok(d) and not ctx.meta:
            ctx.set_output("X@GRAD", _fk.act_bwd(name, d, x, y, a, b))
            return
        if y is None:
            y = fwd(x, a, b)
        if x is None:
            x = torch.zeros_like(y)
        ctx.set_output("X@GRAD", d * dfn(x, y, a, b).to(d.dtype))

    k.__name__ = name
    kg.__name__ = name + "_grad"


for _n, (_a, _k, _f, _d) in _ACT.items():
    _make_act(_n, _a, _k, _f, _d)


@register_op("prelu", ["X", "Alpha"], ["Out"], {"mode": "all"})
def prelu(ctx):
    x, a = ctx.input("X"), ctx.input("Alpha")
    mode = ctx.attr("mode")
    if mode == "channel":
        a = a.reshape([1, -1] + [1] * (x.dim() - 2))
    elif mode == "element":
        a = a.reshape((1,) + tuple(x.shape[1:]))
    ctx.set_output("Out", torch.where(x > 0, x, a * x))


@register_op("maxout", ["X"], ["Out"], {"groups": 1})
def maxout(ctx):
    x = ctx.input("X")
    g = ctx.attr("groups")
    from ..ops import convnd as _cnd
    if _cnd.supported_pool(x):
        ctx.set_output("Out", _cnd.maxout(x, g))
        return
    N, C, H, W = x.shape
    ctx.set_output("Out", x.reshape(N, C // g, g, H, W).max(2).values)


# ------------------------------------------------------------------ scale / sum / mean


@register_op("scale", ["X"], ["Out"], {"scale": 1.0, "bias": 0.0, "bias_after_scale": True})
def scale(ctx):
    v = ctx.input_value("X")
    s, b = ctx.attr("scale"), ctx.attr("bias")
    if isinstance(v, core.SelectedRows):
        t = v.get_tensor().tensor
        out = core.SelectedRows(v.rows(), v.height(), t * s + b if ctx.attr("bias_after_scale") else (t + b) * s)
        ctx.set_output("Out", out)
        return
    x = v.tensor
    out = x * s + b if ctx.attr("bias_after_scale") else (x + b) * s
    ctx.set_output("Out", out.to(x.dtype))


@register_op("sum", ["X*"], ["Out"], {"use_mkldnn": False})
def sum_op(ctx):
    """Sums dense tensors and SelectedRows (sum_op.cc); SelectedRows-only -> SelectedRows."""
    vals = [v for v in ctx.input_values("X") if v is not None]
    if vals and all(isinstance(v, core.SelectedRows) for v in vals):
        rows, ts = [], []
        for v in vals:
            rows += v.rows()
            ts.append(v.get_tensor().tensor)
        ctx.set_output("Out", core.SelectedRows(rows, vals[0].height(), torch.cat(ts, 0)))
        return
    out = None
    for v in vals:
        t = v.to_dense() if isinstance(v, core.SelectedRows) else v.tensor
        if t is None:
            continue
        out = t.clone() if out is None else out + t
    lod = vals[0].lod() if vals and isinstance(vals[0], core.LoDTensor) else None
    ctx.set_output("Out", out, lod)


@register_op("mean", ["X"], ["Out"], {})
def mean(ctx):
    x = ctx.input("X")
    ctx.set_output("Out", x.float().mean().reshape(1).to(x.dtype))


@register_op("minus", ["X", "Y"], ["Out"], {})
def minus(ctx):
    ctx.set_output("Out", ctx.input("X") - ctx.input("Y"))


@register_op("sign", ["X"], ["Out"], {})
def sign(ctx):
    ctx.set_output("Out", torch.sign(ctx.input("X")))


@register_op("clip", ["X"], ["Out"], {"min": -1e30, "max": 1e30})
def clip(ctx):
    ctx.set_output("Out", torch.clamp(ctx.input("X"), ctx.attr("min"), ctx.attr("max")))


@register_op("clip_by_norm", ["X"], ["Out"], {"max_norm": 1.0})
def clip_by_norm(ctx):
    x = ctx.input("X")
    n = torch.sqrt((x.float() ** 2).sum())
    mx = ctx.attr("max_norm")
    ctx.set_output("Out", (x * torch.where(n > mx, mx / n, torch.ones_like(n))).to(x.dtype))


@register_op("cumsum", ["X"], ["Out"], {"axis": -1, "exclusive": False, "reverse": False})
def cumsum(ctx):
    x = ctx.input("X")
    ax = ctx.attr("axis")
    if ctx.attr("reverse"):
        x = x.flip(ax)
    out = torch.cumsum(x, ax)
    if ctx.attr("exclusive"):
        out = out - x
    if ctx.attr("reverse"):
        out = out.flip(ax)
    ctx.set_output("Out", out)


def _reduce(name, fn):
    @register_op(name, ["X"], ["Out"], {"dim": [0], "keep_dim": False, "reduce_all": False})
    def k(ctx):
        x = ctx.input("X")
        dims = ctx.attr("dim")
        dims = [dims] if isinstance(dims, int) else list(dims)
        if x.is_cuda and x.dim() > 0:
            rdims = list(range(x.dim())) if (ctx.attr("reduce_all") or not dims) else dims
            out = _oplib.reduce_op(name[len("reduce_"):], x, rdims, ctx.attr("keep_dim"))
            if out is not None:
                if out.dim() == 0 or (not ctx.attr("keep_dim") and len(set(d % x.dim() for d in rdims)) == x.dim()):
                    out = out.reshape([1] * x.dim()) if ctx.attr("keep_dim") else out.reshape(1)
                ctx.set_output("Out", out)
                return
        if ctx.attr("reduce_all") or not dims:
            out = fn(x.reshape(-1), 0, False)
            out = out.reshape([1] * x.dim()) if ctx.attr("keep_dim") else out.reshape(1)
        else:
            dims = [d % x.dim() for d in dims]
            out = x
            for d in sorted(dims, reverse=True):
                out = fn(out, d, True)
            if not ctx.attr("keep_dim"):
                out = out.squeeze(dims) if len(dims) < x.dim() else out.reshape(1)
        ctx.set_output("Out", out)

    k.__name__ = name


_reduce("reduce_sum", lambda t, d, k: t.sum(d, keepdim=k))
_reduce("reduce_mean", lambda t, d, k: t.mean(d, keepdim=k))
_reduce("reduce_max", lambda t, d, k: t.amax(d, keepdim=k))
_reduce("reduce_min", lambda t, d, k: t.amin(d, keepdim=k))
_reduce("reduce_prod", lambda t, d, k: t.prod(d, keepdim=k))


@register_op("l1_norm", ["X"], ["Out"], {})
def l1_norm(ctx):
    ctx.set_output("Out", ctx.input("X").abs().sum().reshape(1))


@register_op("squared_l2_norm", ["X"], ["Out"], {})
def squared_l2_norm(ctx):
    x = ctx.input("X")
    ctx.set_output("Out", (x.float() ** 2).sum().reshape(1).to(x.dtype))


@register_op("squared_l2_distance", ["X", "Y"], ["sub_result~", "Out"], {})
def squared_l2_distance(ctx):
    x, y = ctx.input("X"), ctx.input("Y")
    sub = x - y
    ctx.set_output("sub_result", sub)
    ctx.set_output("Out", (sub.reshape(sub.shape[0], -1) ** 2).sum(1, keepdim=True))


@register_op("cos_sim", ["X", "Y"], ["Out", "XNorm~", "YNorm~"], {})
def cos_sim(ctx):
    x, y = ctx.input("X"), ctx.input("Y")
    from ..ops import nnmisc as _nm
    r = _nm.cos_sim(x, y)
    if r is not None:  # cos_sim kernels (nnmisc.hip)
        ctx.set_output("Out", r[0])
        ctx.set_output("XNorm", r[1])
        ctx.set_output("YNorm", r[2])
        return
    x2, y2 = x.reshape(x.shape[0], -1), y.reshape(y.shape[0], -1)
    xn = x2.norm(dim=1, keepdim=True)
    yn = y2.norm(dim=1, keepdim=True)
    out = (x2 * y2).sum(1, keepdim=True) / (xn * yn)
    ctx.set_output("Out", out)
    ctx.set_output("XNorm", xn)
    ctx.set_output("YNorm", yn)


@register_op("norm", ["X"], ["Out", "Norm~"], {"axis": 1, "epsilon": 1e-10})
def norm(ctx):
    x = ctx.input("X")
    ax = ctx.attr("axis")
    n = torch.sqrt((x * x).sum(ax, keepdim=True) + ctx.attr("epsilon"))
    ctx.set_output("Out", x / n)
    ctx.set_output("Norm", n)


@register_op("bilinear_tensor_product", ["X", "Y", "Weight", "Bias?"], ["Out"], {})
def bilinear_tensor_product(ctx):
    x, y, w = ctx.input("X"), ctx.input("Y"), ctx.input("Weight")
    out = torch.einsum("bi,kij,bj->bk", x, w, y)
    if ctx.has_input("Bias"):
        out = out + ctx.input("Bias")
    ctx.set_output("Out", out)


@register_op("fused_elemwise_activation", ["X", "Y"], ["Out", "IntermediateOut?~"],
             {"functor_list": ["elementwise_add", "relu"], "axis": -1, "scale": 0.0, "recomputation": True,
              "save_intermediate_out": False})
def fused_elemwise_activation(ctx):
    """{scale, relu} o {elementwise_add, elementwise_mul} in either order (fused_elemwise_activation_op.cc)."""
    x, y = ctx.input("X"), ctx.input("Y")
    f0, f1 = ctx.attr("functor_list")
    if x.is_cuda:
        r = _oplib.fused_ew_act(x, y, (f0, f1), ctx.attr("axis"), ctx.attr("scale"),
                                ctx.has_output("IntermediateOut"))
        if r is not None:
            ctx.set_output("Out", r[0])
            if ctx.has_output("IntermediateOut"):
                ctx.set_output("IntermediateOut", r[1])
            return

    def unary(name, t):
        if name == "relu":
            return F.relu(t)
        if name == "scale":
            return t * ctx.attr("scale")
        raise ValueError(name)

    def binary(name, a, b):
        b = bcast_y(a, b, ctx.attr("axis"))
        return a + b if name == "elementwise_add" else a * b

    if f0.startswith("elementwise"):
        inter = unary(f1, y)
        out = binary(f0, x, inter)
    else:
        inter = binary(f1, x, y)
        out = unary(f0, inter)
    ctx.set_output("Out", out)
    if ctx.has_output("IntermediateOut"):
        ctx.set_output("IntermediateOut", inter)
