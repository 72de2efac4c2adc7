"""Native execution of tensor ops issued on GPU tensors by framework code.

The framework's DyGraph tensors, the eager engine's backward rules, the
``paddle.*`` tensor API and the Fluid op library express much of their pointwise,
cast, fill and reduction work as ordinary tensor expressions.  Inside a framework
region (:func:`paddle_amd.utils.strict.region`) those expressions arrive here as
ATen op overloads (``aten::add.Tensor``, ``aten::_to_copy``, ``aten::sum.dim_IntList``
...) and run on the framework's own HIP kernels (``csrc/kernels/tensor_ops.hip``:
one strided elementwise kernel family with per-operand dtype and strides, one
reduction family) instead of ATen's.

Reference parity: the reference's elementwise / activation / reduce operators are
one CUDA functor per (op, dtype) (paddle/fluid/operators/elementwise_op_function.h:
391-468, activation_op.h, reduce_op.h); here a handler maps each ATen overload onto
the generic kernels: broadcasting becomes stride 0, views and type promotion are
folded into the operand descriptors, so no op materialises a broadcast or a cast.

A handler returns ``NotImplemented`` for a case it does not cover (too many dims
after coalescing, a complex dtype, a CPU operand ...); the caller then counts the
ATen kernel (and raises under ``FLAGS_strict_native=1``).
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _native as N

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3, torch.int64: 4, torch.int32: 5,
       torch.int16: 6, torch.int8: 7, torch.uint8: 8, torch.bool: 9}
_FLOATS = (torch.float32, torch.bfloat16, torch.float16, torch.float64)
_ND = 6

# op codes of tensor_ops.hip
U = dict(copy=0, fill=1, neg=2, abs=3, exp=4, log=5, sqrt=6, rsqrt=7, sin=8, cos=9, tanh=10, sigmoid=11, relu=12,
         reciprocal=13, floor=14, ceil=15, round=16, trunc=17, sign=18, affine=19, pows=20, clamp=21,
         logical_not=22, erf=23, log1p=24, expm1=25, gelu=26, gelu_tanh=27, silu=28, leaky_relu=29, elu=30,
         softplus=31, log2=32, isnan=33, isinf=34, isfinite=35, bitwise_not=36, rpow=37, hardsigmoid=38,
         hardswish=39, square=40, clamp_min=41, clamp_max=42, atan=43, log10=44, exp2=45, frac=46, mish=47,
         iota=48)
B = dict(add=50, sub=51, mul=52, div=53, maximum=54, minimum=55, pow=56, eq=57, ne=58, lt=59, le=60, gt=61, ge=62,
         logical_and=63, logical_or=64, logical_xor=65, floor_divide=66, remainder=67, atan2=68, fmod=69,
         threshold_backward=70, sigmoid_backward=71, tanh_backward=72, bitwise_and=73, bitwise_or=74,
         bitwise_xor=75, div_trunc=76, div_floor=77, gelu_backward=78, gelu_tanh_backward=79, silu_backward=80,
         leaky_relu_backward=81, hardtanh_backward=82, lerps=83, elu_backward=84, softplus_backward=85, fmax=86,
         fmin=87, hardsigmoid_backward=88, hardswish_backward=89,
         where=90, addcmul=91, addcdiv=92, lerp=93, clamp_t=94, mish_backward=95)
RED = dict(sum=0, mean=1, max=2, min=3, prod=4, any=5, all=6, norm2=7, sumsq=8, argmax=9, argmin=10, norm1=11,
           amax=12, amin=13)

_LA = ctypes.c_long * _ND
_lib_ready = [False]


def _lib():
    L = N.lib()
    if not _lib_ready[0]:
        P, I, Lg, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_double
        LP = ctypes.POINTER(ctypes.c_long)
        L.pa_ew.argtypes = [I, I, I, I, LP, P, I, LP, P, I, LP, P, I, LP, P, I, LP, D, D, P]
        L.pa_ew.restype = I
        L.pa_ew_flat.argtypes = [I, I, I, Lg, P, I, P, I, P, I, P, I, D, D, P]
        L.pa_ew_flat.restype = I
        L.pa_reduce_any.argtypes = [I, I, P, I, P, I, Lg, Lg, Lg, D, P, Lg, P]
        L.pa_reduce_any.restype = Lg
        L.pa_index_select.argtypes = [P, I, Lg, Lg, Lg, P, I, Lg, P, P]
        L.pa_index_select.restype = I
        L.pa_cumsum.argtypes = [I, P, I, P, I, Lg, Lg, Lg, P]
        L.pa_cumsum.restype = I
        _lib_ready[0] = True
    return L


# ---------------------------------------------------------------------------- helpers
def _is_scalar(v):
    return isinstance(v, (bool, int, float)) or (isinstance(v, torch.Tensor) and v.dim() == 0
                                                and v.device.type == "cpu")


def _sval(v):
    if isinstance(v, torch.Tensor):
        return v.item()  # a host 0-d tensor: no device sync
    return v


def _cdt(dtype):
    if dtype == torch.float64:
        return 1
    if dtype in _FLOATS:
        return 0
    return 2


def _ok(t):
    return isinstance(t, torch.Tensor) and t.device.type == "cuda" and t.dtype in _DT


def _coalesce(shape, strides_list):
    """Drop size-1 dims and merge adjacent dims that are contiguous for every operand."""
    dims = [(s, [st[i] for st in strides_list]) for i, s in enumerate(shape) if s != 1]
    if not dims:
        return [1], [[0] * 0 + [0] for _ in strides_list]
    out = [dims[0]]
    for s, sts in dims[1:]:
        ps, psts = out[-1]
        if all(psts[k] == sts[k] * s for k in range(len(sts))):
            out[-1] = (ps * s, sts)
        else:
            out.append((s, sts))
    shp = [s for s, _ in out]
    return shp, [[sts[k] for _, sts in out] for k in range(len(strides_list))]


_FASTFN = []


def _fast_fns():
    F = N.fastops()
    _FASTFN.append((F.ew0, F.ew1, F.ew2, F.ew3) if F is not None else None)
    return _FASTFN[0]


def _launch(op, out, ins, a=0.0, b=0.0, cdt=None):
    """out[...] = op(ins...) over out's shape; inputs broadcast by stride 0.
    Returns False when the launch does not fit the kernel (caller falls back)."""
    fns = _FASTFN[0] if _FASTFN else _fast_fns()
    if fns is not None and len(ins) <= 3 and fns[len(ins)](op, -1 if cdt is None else cdt, out, *ins, float(a),
                                                              float(b), N.stream()):
        return True  # contiguous same-shape operands: the C++ entry (csrc/fastops)
    if cdt is None:
        cdt = _cdt(out.dtype if not ins else ins[0].dtype)
    if out.is_contiguous() and all(t.is_contiguous() and t.shape == out.shape for t in ins):
        # hot path: one flat launch, scalar arguments only
        x = ins[0] if len(ins) > 0 else None
        y = ins[1] if len(ins) > 1 else None
        z = ins[2] if len(ins) > 2 else None
        rc = _lib().pa_ew_flat(op, cdt, len(ins), out.numel(), out.data_ptr(), _DT[out.dtype],
                               x.data_ptr() if x is not None else None, _DT[x.dtype] if x is not None else 0,
                               y.data_ptr() if y is not None else None, _DT[y.dtype] if y is not None else 0,
                               z.data_ptr() if z is not None else None, _DT[z.dtype] if z is not None else 0,
                               float(a), float(b), N.stream())
        N.check(rc, "pa_ew_flat")
        return True
    shape = list(out.shape)
    strs = [list(out.stride())]
    for t in ins:
        if t.dim() > len(shape):
            return False
        e = t.expand(shape) if list(t.shape) != shape else t
        strs.append(list(e.stride()))
    shp, sts = _coalesce(shape, strs)
    if len(shp) > _ND:
        return False
    nd = len(shp)
    sz = _LA(*shp)
    arr = [_LA(*s) for s in sts]
    if cdt is None:
        cdt = _cdt(out.dtype if not ins else ins[0].dtype)
    x = ins[0] if len(ins) > 0 else None
    y = ins[1] if len(ins) > 1 else None
    z = ins[2] if len(ins) > 2 else None
    zero = _LA(*([0] * _ND))
    rc = _lib().pa_ew(op, cdt, len(ins), nd, sz, out.data_ptr(), _DT[out.dtype], arr[0],
                      x.data_ptr() if x is not None else None, _DT[x.dtype] if x is not None else 0,
                      arr[1] if x is not None else zero,
                      y.data_ptr() if y is not None else None, _DT[y.dtype] if y is not None else 0,
                      arr[2] if y is not None else zero,
                      z.data_ptr() if z is not None else None, _DT[z.dtype] if z is not None else 0,
                      arr[3] if z is not None else zero, float(a), float(b), N.stream())
    N.check(rc, "pa_ew")
    return True


def _new_out(shape, dtype, like=None):
    """Output allocation: keep the first same-shape input's dense layout (channels-last
    activations stay channels-last), else contiguous."""
    if like is not None and list(like.shape) == list(shape) and like.dtype in _DT and _dense(like):
        return torch.empty_like(like, dtype=dtype)
    dev = like.device if like is not None else torch.device("cuda", torch.cuda.current_device())
    return torch.empty(shape, dtype=dtype, device=dev)


def _dense(t):
    """Non-overlapping and dense (a permutation of a contiguous layout)."""
    if t.is_contiguous():
        return True
    dims = sorted((st, s) for s, st in zip(t.shape, t.stride()) if s != 1)
    expect = 1
    for st, s in dims:
        if st != expect:
            return False
        expect *= s
    return True


def _bshape(*ts):
    return list(torch.broadcast_shapes(*[t.shape for t in ts]))


# ---------------------------------------------------------------------------- registry
HANDLERS: dict = {}


def _h(*names):
    def deco(fn):
        for n in names:
            HANDLERS[n] = fn
        return fn
    return deco


_FUNC = {}  # OpOverload -> (name, handler): resolved once per overload


def try_native(func, args, kwargs):
    """Run ``func`` (an ATen OpOverload) on the HIP kernels; NotImplemented if no handler
    covers this call."""
    ent = _FUNC.get(func)
    if ent is None:
        name = f"{func.overloadpacket.__name__}.{func._overloadname}"
        ent = _FUNC[func] = (name, HANDLERS.get(name))
    name, h = ent
    if h is None:
        return NotImplemented
    try:
        return h(name, *args, **kwargs)
    except _Skip:
        return NotImplemented


class _Skip(Exception):
    pass


def _need(cond):
    if not cond:
        raise _Skip()


# ---------------------------------------------------------------------------- binary
_BIN = {"add": "add", "sub": "sub", "mul": "mul", "div": "div", "maximum": "maximum", "minimum": "minimum",
        "fmax": "fmax", "fmin": "fmin", "pow": "pow", "eq": "eq", "ne": "ne", "lt": "lt", "le": "le", "gt": "gt",
        "ge": "ge", "logical_and": "logical_and", "logical_or": "logical_or", "logical_xor": "logical_xor",
        "remainder": "remainder", "fmod": "fmod", "atan2": "atan2", "floor_divide": "floor_divide",
        "bitwise_and": "bitwise_and", "bitwise_or": "bitwise_or", "bitwise_xor": "bitwise_xor",
        "rsub": "sub", "greater": "gt", "less": "lt", "greater_equal": "ge", "less_equal": "le",
        "not_equal": "ne", "true_divide": "div", "multiply": "mul", "subtract": "sub"}
_CMP = {"eq", "ne", "lt", "le", "gt", "ge", "logical_and", "logical_or", "logical_xor"}


_FAST_BIN = {"add.Tensor": (0, False), "sub.Tensor": (1, False), "mul.Tensor": (2, False),
             "add_.Tensor": (0, True), "sub_.Tensor": (1, True), "mul_.Tensor": (2, True)}
_FAST_DT = None


def _binary(name, self, other, alpha=1, rounding_mode=None, out=None):
    # hot path: same-shape, same-dtype, contiguous fp32 / bf16 device tensors (the
    # residual adds, gradient sums and scalings of a training step) -- metadata
    # checks only, one flat launch
    fb = _FAST_BIN.get(name)
    if fb is not None and out is None and isinstance(other, torch.Tensor):
        fns = _FASTFN[0] if _FASTFN else _fast_fns()
        if fns is not None and isinstance(alpha, (int, float)):
            r = N.fastops().bin(_FAST_OPS[fb[0]], self, other, float(alpha), fb[1])  # all in C++
            if r is not None:
                return r
        global _FAST_DT
        if _FAST_DT is None:
            _FAST_DT = {torch.float32: _DT[torch.float32], torch.bfloat16: _DT[torch.bfloat16]}
        dt = self.dtype
        code = _FAST_DT.get(dt)
        if (code is not None and other.dtype is dt and self.is_cuda and other.is_cuda and self.dim() > 0
                and self.shape == other.shape and self.is_contiguous() and other.is_contiguous()
                and isinstance(alpha, (int, float))):
            dst = self if fb[1] else torch.empty_like(self)
            op = _FAST_OPS[fb[0]]
            rc = _lib().pa_ew_flat(op, 0, 2, dst.numel(), dst.data_ptr(), code, self.data_ptr(), code,
                                   other.data_ptr(), code, None, 0, float(alpha), 0.0, N.stream())
            N.check(rc, "pa_ew_flat")
            return dst
    base, ovl = name.split(".")
    inplace = base.endswith("_")
    base = base.rstrip("_")
    kind = _BIN[base]
    rsub = base == "rsub"
    _need(_ok(self) or _ok(other))
    # operand dtype promotion (torch semantics), computed on metadata only
    rdt = torch.result_type(self, other)
    if kind == "div" and rdt not in _FLOATS and rounding_mode is None:
        rdt = torch.get_default_dtype()
    _need(rdt in _DT)
    odt = torch.bool if kind in _CMP else rdt
    op = B[kind]
    if kind == "div" and rounding_mode == "trunc":
        op = B["div_trunc"]
    elif kind == "div" and rounding_mode == "floor":
        op = B["div_floor"]
    cdt = _cdt(rdt)
    if cdt == 2 and kind in ("atan2",):
        raise _Skip()
    if cdt != 2 and kind.startswith("bitwise"):
        raise _Skip()
    tensors = [t for t in (self, other) if isinstance(t, torch.Tensor) and not _is_scalar(t)]
    _need(all(_ok(t) for t in tensors))
    a = _sval(alpha) if alpha is not None else 1
    # a scalar operand becomes a 0-stride fill of the compute type: use the affine
    # / scalar kernels where they exist, else a 1-element device constant
    if _is_scalar(other) and not _is_scalar(self):
        s = _sval(other)
        x = self
        res_shape = list(x.shape)
        if kind in ("add", "sub") and not rsub and cdt != 2:
            sign = 1 if kind == "add" else -1
            return _unary_out(x, U["affine"], res_shape, odt, inplace, out, a=1.0, b=sign * a * s, cdt=cdt)
        if kind == "mul" and cdt != 2:
            return _unary_out(x, U["affine"], res_shape, odt, inplace, out, a=s, b=0.0, cdt=cdt)
        if kind == "sub" and rsub and cdt != 2:
            return _unary_out(x, U["affine"], res_shape, odt, inplace, out, a=-a, b=s, cdt=cdt)
        if kind == "div" and op == B["div"] and cdt != 2:
            return _unary_out(x, U["affine"], res_shape, odt, inplace, out, a=1.0 / s if s != 0 else math.inf,
                              b=0.0, cdt=cdt) if s != 0 else _const_bin(op, x, s, odt, inplace, out, cdt, a)
        if kind == "pow" and cdt != 2:
            if s == 2:
                return _unary_out(x, U["square"], res_shape, odt, inplace, out, cdt=cdt)
            return _unary_out(x, U["pows"], res_shape, odt, inplace, out, a=s, cdt=cdt)
        if rsub:
            return _const_bin(op, x, s, odt, inplace, out, cdt, a, swap=True)
        return _const_bin(op, x, s, odt, inplace, out, cdt, a)
    if _is_scalar(self) and not _is_scalar(other):
        s = _sval(self)
        if kind == "pow" and cdt != 2:
            return _unary_out(other, U["rpow"], list(other.shape), odt, inplace, out, a=s, cdt=cdt)
        return _const_bin(op, other, s, odt, inplace, out, cdt, a, swap=not rsub)
    _need(isinstance(self, torch.Tensor) and isinstance(other, torch.Tensor))
    x, y = (other, self) if rsub else (self, other)
    shape = _bshape(self, other)
    if inplace:
        _need(list(self.shape) == shape)
        dst = self
    elif out is not None:
        _need(list(out.shape) == shape and out.dtype in _DT)
        dst = out
    else:
        dst = _new_out(shape, odt, like=self if list(self.shape) == shape else other)
    _need(_launch(op, dst, [x, y], a=a, cdt=cdt))
    return dst


def _const_bin(op, x, s, odt, inplace, out, cdt, a=1, swap=False):
    """x (op) scalar via a one-element device constant broadcast by stride 0."""
    c = torch.empty((), dtype=torch.float64 if cdt == 1 else (torch.float32 if cdt == 0 else torch.int64),
                    device=x.device)
    _launch(U["fill"], c, [], a=s, cdt=cdt)
    dst = x if inplace else (out if out is not None else _new_out(list(x.shape), odt, like=x))
    _need(list(dst.shape) == list(x.shape))
    _need(_launch(op, dst, [c, x] if swap else [x, c], a=a, cdt=cdt))
    return dst


def _unary_out(x, op, shape, odt, inplace, out, a=0.0, b=0.0, cdt=None):
    dst = x if inplace else (out if out is not None else _new_out(shape, odt, like=x))
    _need(list(dst.shape) == list(shape))
    _need(_launch(op, dst, [x], a=a, b=b, cdt=cdt))
    return dst


_FAST_OPS = (B["add"], B["sub"], B["mul"])
_FAST_CODE = {torch.float32: _DT[torch.float32], torch.bfloat16: _DT[torch.bfloat16]}

for _n in _BIN:
    for _s in ("Tensor", "Scalar", "out", "Tensor_Tensor", "Tensor_Scalar", "Tensor_mode", "Scalar_mode",
               "Self", "Scalar_Tensor", "default"):
        HANDLERS[f"{_n}.{_s}"] = _binary
        HANDLERS[f"{_n}_.{_s}"] = _binary


@_h("pow.Scalar")
def _pow_scalar(name, self, exponent):
    return _binary("pow.Scalar", self, exponent)


# ---------------------------------------------------------------------------- unary
_UN = {"neg": "neg", "abs": "abs", "exp": "exp", "log": "log", "sqrt": "sqrt", "rsqrt": "rsqrt", "sin": "sin",
       "cos": "cos", "tanh": "tanh", "sigmoid": "sigmoid", "relu": "relu", "reciprocal": "reciprocal",
       "floor": "floor", "ceil": "ceil", "round": "round", "trunc": "trunc", "sign": "sign", "erf": "erf",
       "log1p": "log1p", "expm1": "expm1", "silu": "silu", "log2": "log2", "log10": "log10", "exp2": "exp2",
       "atan": "atan", "frac": "frac", "mish": "mish", "hardsigmoid": "hardsigmoid", "hardswish": "hardswish",
       "square": "square", "logical_not": "logical_not", "bitwise_not": "bitwise_not", "isnan": "isnan",
       "isinf": "isinf", "negative": "neg", "absolute": "abs"}
_FLOAT_ONLY = {"exp", "log", "sqrt", "rsqrt", "sin", "cos", "tanh", "sigmoid", "reciprocal", "erf", "log1p", "expm1",
               "silu", "log2", "log10", "exp2", "atan", "mish", "hardsigmoid", "hardswish"}


def _unary(name, self, *rest, out=None, **kw):
    base = name.split(".")[0]
    inplace = base.endswith("_")
    base = base.rstrip("_")
    kind = _UN[base]
    _need(_ok(self))
    dt = self.dtype
    if kind in _FLOAT_ONLY and dt not in _FLOATS:
        _need(not inplace)
        odt = torch.get_default_dtype()
    elif kind in ("logical_not", "isnan", "isinf"):
        odt = torch.bool
    else:
        odt = dt
    if kind in ("floor", "ceil", "round", "trunc") and dt not in _FLOATS:
        return self if inplace else _unary_out(self, U["copy"], list(self.shape), dt, False, out, cdt=2)
    if kind == "round" and rest and rest[0]:
        raise _Skip()  # round(decimals=)
    if kind == "bitwise_not" and dt == torch.bool:
        kind = "logical_not"
        odt = torch.bool
    _need(not (kind == "bitwise_not" and dt in _FLOATS))
    cdt = _cdt(dt if dt in _FLOATS or kind in ("abs", "neg", "sign", "square", "logical_not", "bitwise_not")
               else torch.float32)
    if inplace:
        _need(odt == dt)
    return _unary_out(self, U[kind], list(self.shape), odt, inplace, out, cdt=cdt)


for _n in _UN:
    for _s in ("default", "out"):
        HANDLERS[f"{_n}.{_s}"] = _unary
        HANDLERS[f"{_n}_.{_s}"] = _unary


@_h("gelu.default", "gelu_.default", "gelu.out")
def _gelu(name, self, approximate="none", out=None):
    _need(_ok(self) and self.dtype in _FLOATS)
    return _unary_out(self, U["gelu_tanh" if approximate == "tanh" else "gelu"], list(self.shape), self.dtype,
                      name.startswith("gelu_"), out)


@_h("leaky_relu.default", "leaky_relu_.default")
def _leaky(name, self, negative_slope=0.01):
    _need(_ok(self) and self.dtype in _FLOATS)
    return _unary_out(self, U["leaky_relu"], list(self.shape), self.dtype, name.startswith("leaky_relu_"), None,
                      a=_sval(negative_slope))


@_h("elu.default", "elu_.default")
def _elu(name, self, alpha=1.0, scale=1.0, input_scale=1.0):
    _need(_ok(self) and self.dtype in _FLOATS and scale == 1 and input_scale == 1)
    return _unary_out(self, U["elu"], list(self.shape), self.dtype, name.startswith("elu_"), None, a=_sval(alpha))


@_h("softplus.default")
def _softplus(name, self, beta=1, threshold=20):
    _need(_ok(self) and self.dtype in _FLOATS)
    return _unary_out(self, U["softplus"], list(self.shape), self.dtype, False, None, a=_sval(beta),
                      b=_sval(threshold))


@_h("hardtanh.default", "hardtanh_.default")
def _hardtanh(name, self, min_val=-1, max_val=1):
    _need(_ok(self))
    return _unary_out(self, U["clamp"], list(self.shape), self.dtype, name.startswith("hardtanh_"), None,
                      a=_sval(min_val), b=_sval(max_val))


@_h("clamp.default", "clamp_.default", "clip.default", "clip_.default")
def _clamp(name, self, min=None, max=None):
    _need(_ok(self))
    inplace = name.split(".")[0].endswith("_")
    mn, mx = _sval(min), _sval(max)
    _need(not isinstance(mn, torch.Tensor) and not isinstance(mx, torch.Tensor))
    if mn is not None and mx is not None:
        return _unary_out(self, U["clamp"], list(self.shape), self.dtype, inplace, None, a=mn, b=mx)
    if mn is not None:
        return _unary_out(self, U["clamp_min"], list(self.shape), self.dtype, inplace, None, a=mn)
    if mx is not None:
        return _unary_out(self, U["clamp_max"], list(self.shape), self.dtype, inplace, None, a=mx)
    raise _Skip()


@_h("clamp_min.default", "clamp_min_.default")
def _clamp_min(name, self, min):
    _need(_ok(self) and _is_scalar(min))
    return _unary_out(self, U["clamp_min"], list(self.shape), self.dtype, name.startswith("clamp_min_"), None,
                      a=_sval(min))


@_h("clamp_max.default", "clamp_max_.default")
def _clamp_max(name, self, max):
    _need(_ok(self) and _is_scalar(max))
    return _unary_out(self, U["clamp_max"], list(self.shape), self.dtype, name.startswith("clamp_max_"), None,
                      a=_sval(max))


# ---------------------------------------------------------------------------- backward pointwise
def _bwd2(kind):
    def h(name, grad, x, *extra, **kw):
        if "approximate" in kw:
            extra = (kw["approximate"],)
        _need(_ok(grad) and _ok(x) and grad.dtype in _FLOATS)
        shape = _bshape(grad, x)
        dst = _new_out(shape, grad.dtype, like=grad)
        a = b = 0.0
        k = kind
        if kind == "threshold_backward":
            a = _sval(extra[0])
        elif kind == "gelu_backward":
            k = "gelu_tanh_backward" if (extra and extra[0] == "tanh") else "gelu_backward"
        elif kind == "leaky_relu_backward":
            a = _sval(extra[0])
        elif kind == "hardtanh_backward":
            a, b = _sval(extra[0]), _sval(extra[1])
        elif kind == "softplus_backward":
            a, b = _sval(extra[0]), _sval(extra[1])
        elif kind == "elu_backward":
            alpha, scale, input_scale, is_result = extra[0], extra[1], extra[2], extra[3]
            _need(_sval(scale) == 1 and _sval(input_scale) == 1 and not is_result)
            a = _sval(alpha)
        _need(_launch(B[k], dst, [grad, x], a=a, b=b))
        return dst
    return h


for _k in ("threshold_backward", "sigmoid_backward", "tanh_backward", "gelu_backward", "silu_backward",
           "leaky_relu_backward", "hardtanh_backward", "softplus_backward", "hardsigmoid_backward",
           "hardswish_backward", "mish_backward", "elu_backward"):
    HANDLERS[f"{_k}.default"] = _bwd2(_k)


# ---------------------------------------------------------------------------- ternary
@_h("where.self", "where.self_out", "where.ScalarOther", "where.ScalarSelf", "where.Scalar")
def _where(name, cond, self, other, out=None):
    _need(_ok(cond))
    ts = [t for t in (self, other) if isinstance(t, torch.Tensor) and not _is_scalar(t)]
    _need(all(_ok(t) for t in ts) and ts)
    rdt = torch.result_type(self, other)
    _need(rdt in _DT)
    shape = _bshape(cond, *ts)
    dst = out if out is not None else _new_out(shape, rdt, like=ts[0] if list(ts[0].shape) == shape else None)
    ops = []
    for v in (self, other):
        if isinstance(v, torch.Tensor) and not _is_scalar(v):
            ops.append(v)
        else:
            c = torch.empty((), dtype=rdt, device=cond.device)
            _launch(U["fill"], c, [], a=_sval(v), cdt=_cdt(rdt))
            ops.append(c)
    _need(_launch(B["where"], dst, [cond, ops[0], ops[1]], cdt=_cdt(rdt)))
    return dst


@_h("addcmul.default", "addcmul_.default", "addcdiv.default", "addcdiv_.default")
def _addc(name, self, t1, t2, value=1):
    _need(_ok(self) and _ok(t1) and _ok(t2) and self.dtype in _FLOATS)
    inplace = name.split(".")[0].endswith("_")
    k = "addcmul" if name.startswith("addcmul") else "addcdiv"
    shape = _bshape(self, t1, t2)
    dst = self if inplace else _new_out(shape, self.dtype, like=self)
    _need(list(dst.shape) == shape)
    _need(_launch(B[k], dst, [self, t1, t2], a=_sval(value)))
    return dst


@_h("lerp.Scalar", "lerp_.Scalar", "lerp.Tensor", "lerp_.Tensor")
def _lerp(name, self, end, weight):
    _need(_ok(self) and _ok(end) and self.dtype in _FLOATS)
    inplace = name.split(".")[0].endswith("_")
    shape = _bshape(self, end) if _is_scalar(weight) else _bshape(self, end, weight)
    dst = self if inplace else _new_out(shape, self.dtype, like=self)
    _need(list(dst.shape) == shape)
    if _is_scalar(weight):
        _need(_launch(B["lerps"], dst, [self, end], a=_sval(weight)))
    else:
        _need(_ok(weight) and _launch(B["lerp"], dst, [self, end, weight]))
    return dst


@_h("masked_fill.Scalar", "masked_fill_.Scalar", "masked_fill.Tensor", "masked_fill_.Tensor")
def _masked_fill(name, self, mask, value):
    _need(_ok(self) and _ok(mask) and _is_scalar(value))
    inplace = name.split(".")[0].endswith("_")
    shape = list(self.shape)
    _need(not inplace or _bshape(self, mask) == shape)
    dst = self if inplace else _new_out(_bshape(self, mask), self.dtype, like=self)
    c = torch.empty((), dtype=self.dtype, device=self.device)
    _launch(U["fill"], c, [], a=_sval(value), cdt=_cdt(self.dtype))
    _need(_launch(B["where"], dst, [mask, c, self], cdt=_cdt(self.dtype)))
    return dst


# ---------------------------------------------------------------------------- copies, casts, fills
@_h("copy_.default")
def _copy(name, self, src, non_blocking=False):
    # hot path: contiguous same-shape fp32 / bf16 device copy or cast
    if isinstance(src, torch.Tensor) and src.is_cuda and self.is_cuda and self.shape == src.shape:
        dc, sc = _FAST_CODE.get(self.dtype), _FAST_CODE.get(src.dtype)
        if dc is not None and sc is not None and self.is_contiguous() and src.is_contiguous() and self.dim() > 0:
            rc = _lib().pa_ew_flat(U["copy"], 0, 1, self.numel(), self.data_ptr(), dc, src.data_ptr(), sc, None, 0,
                                   None, 0, 0.0, 0.0, N.stream())
            N.check(rc, "pa_ew_flat")
            return self
    _need(_ok(self) and isinstance(src, torch.Tensor))
    if src.device.type != "cuda":
        raise _Skip()  # host -> device transfer: a DMA copy, not a kernel
    _need(src.dtype in _DT and _bshape(self, src) == list(self.shape))
    _need(_launch(U["copy"], self, [src], cdt=_cdt(src.dtype if src.dtype in _FLOATS or self.dtype not in _FLOATS
                                                    else self.dtype)))
    return self


@_h("_to_copy.default")
def _to_copy(name, self, dtype=None, layout=None, device=None, pin_memory=None, non_blocking=False,
             memory_format=None):
    if (device is None and memory_format in (None, torch.preserve_format) and self.is_cuda and self.dim() > 0
            and self.is_contiguous()):
        dt = dtype or self.dtype
        code = _DT.get(dt)
        F = N.fastops()
        if F is not None and code is not None:
            r = F.cast(self, code)  # checks, allocation and launch in C++
            if r is not None:
                return r
        dc, sc = _FAST_CODE.get(dt), _FAST_CODE.get(self.dtype)
        if dc is not None and sc is not None:  # hot path: contiguous fp32 <-> bf16 cast / copy
            dst = torch.empty(self.shape, dtype=dt, device=self.device)
            rc = _lib().pa_ew_flat(U["copy"], 0, 1, dst.numel(), dst.data_ptr(), dc, self.data_ptr(), sc, None, 0,
                                   None, 0, 0.0, 0.0, N.stream())
            N.check(rc, "pa_ew_flat")
            return dst
    _need(_ok(self))
    if device is not None and torch.device(device).type != "cuda":
        raise _Skip()
    dt = dtype or self.dtype
    _need(dt in _DT)
    if memory_format in (None, torch.preserve_format):
        dst = _new_out(list(self.shape), dt, like=self)
    else:
        dst = torch.empty(self.shape, dtype=dt, device=self.device, memory_format=memory_format)
    _need(_launch(U["copy"], dst, [self], cdt=_cdt(self.dtype if self.dtype in _FLOATS or dt not in _FLOATS
                                                    else dt)))
    return dst


@_h("clone.default")
def _clone(name, self, memory_format=None):
    return _to_copy(name, self, memory_format=memory_format)


@_h("fill_.Scalar", "fill_.Tensor")
def _fill(name, self, value):
    _need(_ok(self) and _is_scalar(value))
    _need(_launch(U["fill"], self, [], a=_sval(value), cdt=_cdt(self.dtype)))
    return self


@_h("zero_.default")
def _zero(name, self):
    _need(_ok(self))
    _need(_launch(U["fill"], self, [], a=0.0, cdt=_cdt(self.dtype)))
    return self


def _factory_dev(device):
    return device is not None and torch.device(device).type == "cuda"


@_h("zeros_like.default", "ones_like.default", "full_like.default")
def _full_like(name, self, *args, dtype=None, layout=None, device=None, pin_memory=None, memory_format=None):
    _need(_ok(self) and (device is None or _factory_dev(device)))
    v = 0.0 if name.startswith("zeros") else 1.0 if name.startswith("ones") else _sval(args[0])
    dt = dtype or self.dtype
    _need(dt in _DT and isinstance(v, (int, float, bool)))
    dst = _new_out(list(self.shape), dt, like=self) if memory_format in (None, torch.preserve_format) else \
        torch.empty(self.shape, dtype=dt, device=self.device, memory_format=memory_format)
    _need(_launch(U["fill"], dst, [], a=v, cdt=_cdt(dt)))
    return dst


@_h("zeros.default", "ones.default", "full.default")
def _full(name, size, *args, dtype=None, layout=None, device=None, pin_memory=None):
    _need(_factory_dev(device))
    v = 0.0 if name.startswith("zeros") else 1.0 if name.startswith("ones") else _sval(args[0])
    _need(isinstance(v, (int, float, bool)))
    if dtype is None:
        if name.startswith(("zeros", "ones")) or isinstance(v, float):
            dtype = torch.get_default_dtype()
        else:
            dtype = torch.bool if isinstance(v, bool) else torch.int64
    dt = dtype
    _need(dt in _DT)
    dst = torch.empty(size, dtype=dt, device=device)
    _need(_launch(U["fill"], dst, [], a=v, cdt=_cdt(dt)))
    return dst


@_h("new_zeros.default", "new_ones.default", "new_full.default")
def _new_full(name, self, size, *args, dtype=None, layout=None, device=None, pin_memory=None):
    _need(_ok(self) and (device is None or _factory_dev(device)))
    v = 0.0 if "zeros" in name else 1.0 if "ones" in name else _sval(args[0])
    dt = dtype or self.dtype
    _need(dt in _DT)
    dst = torch.empty(size, dtype=dt, device=self.device)
    _need(_launch(U["fill"], dst, [], a=v, cdt=_cdt(dt)))
    return dst


@_h("flip.default")
def _flip(name, self, dims):
    _need(_ok(self))
    nd = self.dim()
    dims = {d % nd for d in dims} if nd else set()
    st = list(self.stride())
    off = 0
    for d in dims:
        if self.shape[d] > 1:
            off += (self.shape[d] - 1) * st[d]
            st[d] = -st[d]
    dst = torch.empty(self.shape, dtype=self.dtype, device=self.device)
    if dst.numel() == 0:
        return dst
    # negative strides are not expressible as a torch view: launch on raw operands
    shp, sts = _coalesce(list(self.shape), [list(dst.stride()), st])
    _need(len(shp) <= _ND)
    base = self.data_ptr() + off * self.element_size()
    rc = _lib().pa_ew(U["copy"], _cdt(self.dtype), 1, len(shp), _LA(*shp), dst.data_ptr(), _DT[dst.dtype],
                      _LA(*sts[0]), base, _DT[self.dtype], _LA(*sts[1]), None, 0, _LA(*([0] * _ND)), None, 0,
                      _LA(*([0] * _ND)), 0.0, 0.0, N.stream())
    N.check(rc, "pa_ew(flip)")
    return dst


def strided_copy(dst, src_base, src_dtype, src_strides):
    """dst (contiguous) <- a raw source view at ``src_base`` with element strides
    ``src_strides`` over dst's shape (negative strides allowed: flips / reversed
    taps that a torch view cannot express).  One launch of the strided copy kernel."""
    shp, sts = _coalesce(list(dst.shape), [list(dst.stride()), list(src_strides)])
    if len(shp) > _ND:
        raise RuntimeError("strided_copy: too many dimensions")
    rc = _lib().pa_ew(U["copy"], _cdt(src_dtype), 1, len(shp), _LA(*shp), dst.data_ptr(), _DT[dst.dtype],
                      _LA(*sts[0]), src_base, _DT[src_dtype], _LA(*sts[1]), None, 0, _LA(*([0] * _ND)), None, 0,
                      _LA(*([0] * _ND)), 0.0, 0.0, N.stream())
    N.check(rc, "pa_ew(strided_copy)")
    return dst


@_h("cat.default", "cat.out")
def _cat(name, tensors, dim=0, out=None):
    ts = [t for t in tensors if not (t.dim() == 1 and t.numel() == 0)]
    _need(ts and all(_ok(t) for t in ts))
    nd = ts[0].dim()
    dim = dim % nd
    rdt = ts[0].dtype
    for t in ts[1:]:
        rdt = torch.promote_types(rdt, t.dtype)
    _need(rdt in _DT)
    shape = list(ts[0].shape)
    shape[dim] = sum(t.shape[dim] for t in ts)
    if out is not None:
        _need(list(out.shape) == shape)
        dst = out
    elif nd == 4 and all(not t.is_contiguous() and t.is_contiguous(memory_format=torch.channels_last) for t in ts):
        dst = torch.empty(shape, dtype=rdt, device=ts[0].device, memory_format=torch.channels_last)
    else:
        dst = torch.empty(shape, dtype=rdt, device=ts[0].device)
    o = 0
    for t in ts:
        n = t.shape[dim]
        if n:
            _need(_launch(U["copy"], dst.narrow(dim, o, n), [t], cdt=_cdt(t.dtype if t.dtype in _FLOATS else rdt)))
        o += n
    return dst


@_h("stack.default")
def _stack(name, tensors, dim=0, out=None):
    _need(out is None and tensors)
    nd = tensors[0].dim() + 1
    return _cat("cat.default", [t.unsqueeze(dim % nd) for t in tensors], dim % nd)


# ---------------------------------------------------------------------------- reductions
def _norm_dims(dims, nd):
    if dims is None or (isinstance(dims, (list, tuple)) and len(dims) == 0):
        return list(range(nd))
    if isinstance(dims, int):
        dims = [dims]
    return sorted({d % nd for d in dims}) if nd else []


def _reduce(op, x, dims, keepdim, odt, cdt=None, idx_out=False):
    """Reduce ``x`` over ``dims`` into a new tensor of dtype ``odt``."""
    nd = x.dim()
    dims = _norm_dims(dims, nd)
    keep = [d for d in range(nd) if d not in dims]
    oshape = [x.shape[d] for d in keep]
    kshape = [1 if d in dims else x.shape[d] for d in range(nd)]
    # contiguous [outer, R, inner]: reduced dims that form one block are reduced in
    # place (after a contiguous copy if needed); otherwise the kept dims are moved in
    # front by one strided copy and the reduction runs over the trailing block
    if not dims or dims == list(range(dims[0], dims[-1] + 1)):
        src = x if x.is_contiguous() else _to_copy("_to_copy.default", x, memory_format=torch.contiguous_format)
        lo, hi = (dims[0], dims[-1] + 1) if dims else (0, 0)
        outer = math.prod(x.shape[:lo])
        R = math.prod(x.shape[lo:hi])
        inner = math.prod(x.shape[hi:])
    else:
        perm = keep + dims
        pv = x.permute(perm)
        src = torch.empty(pv.shape, dtype=x.dtype, device=x.device)
        _need(_launch(U["copy"], src, [pv], cdt=_cdt(x.dtype)))
        outer, R, inner = math.prod(oshape), math.prod(x.shape[d] for d in dims), 1
    if cdt is None:
        cdt = _cdt(x.dtype)
    dst = torch.empty(oshape, dtype=odt, device=x.device)
    if dst.numel() == 0:
        return dst.reshape(kshape) if keepdim else dst
    if R == 0:
        raise _Skip()
    L = _lib()
    rc = L.pa_reduce_any(op, cdt, src.data_ptr(), _DT[src.dtype], dst.data_ptr(), _DT[odt], outer, R, inner,
                         1.0 / R, None, 0, N.stream())
    if rc > 0:
        ws = torch.empty(int(rc), dtype=torch.uint8, device=x.device)
        rc = L.pa_reduce_any(op, cdt, src.data_ptr(), _DT[src.dtype], dst.data_ptr(), _DT[odt], outer, R, inner,
                             1.0 / R, ws.data_ptr(), int(rc), N.stream())
    N.check(int(rc), "pa_reduce_any")
    return dst.reshape(kshape) if keepdim else dst


def _acc_dtype(x, dtype):
    if dtype is not None:
        return dtype
    if x.dtype in (torch.bool, torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64):
        return torch.int64
    return x.dtype


@_h("sum.dim_IntList", "sum.default")
def _sum(name, self, dim=None, keepdim=False, dtype=None):
    _need(_ok(self))
    if name == "sum.default":
        dtype = dim if isinstance(dim, torch.dtype) else dtype
        dim = None
    odt = _acc_dtype(self, dtype)
    _need(odt in _DT)
    return _reduce(RED["sum"], self, dim, keepdim, odt, cdt=_cdt(odt))


@_h("mean.dim", "mean.default")
def _mean(name, self, dim=None, keepdim=False, dtype=None):
    _need(_ok(self))
    if name == "mean.default":
        dtype = dim if isinstance(dim, torch.dtype) else dtype
        dim = None
    odt = dtype or self.dtype
    _need(odt in _FLOATS)
    return _reduce(RED["mean"], self, dim, keepdim, odt, cdt=_cdt(odt))


@_h("amax.default", "amin.default")
def _amax(name, self, dim=(), keepdim=False):
    _need(_ok(self))
    return _reduce(RED["amax" if name.startswith("amax") else "amin"], self, list(dim) or None, keepdim, self.dtype)


@_h("max.default", "min.default")
def _max_all(name, self):
    _need(_ok(self) and self.numel() > 0)
    return _reduce(RED["max" if name.startswith("max") else "min"], self, None, False, self.dtype)


@_h("max.dim", "min.dim")
def _max_dim(name, self, dim, keepdim=False):
    _need(_ok(self) and self.numel() > 0)
    is_max = name.startswith("max")
    vals = _reduce(RED["max" if is_max else "min"], self, [dim], keepdim, self.dtype)
    idx = _reduce(RED["argmax" if is_max else "argmin"], self, [dim], keepdim, torch.int64, cdt=_cdt(self.dtype))
    return vals, idx


@_h("argmax.default", "argmin.default")
def _argmax(name, self, dim=None, keepdim=False):
    _need(_ok(self) and self.numel() > 0)
    k = "argmax" if name.startswith("argmax") else "argmin"
    if dim is None:
        r = _reduce(RED[k], self.reshape(-1) if self.is_contiguous() else self.contiguous().reshape(-1), [0], False,
                    torch.int64, cdt=_cdt(self.dtype))
        return r.reshape([1] * self.dim()) if keepdim else r
    return _reduce(RED[k], self, [dim], keepdim, torch.int64, cdt=_cdt(self.dtype))


@_h("prod.default", "prod.dim_int")
def _prod(name, self, dim=None, keepdim=False, dtype=None):
    _need(_ok(self))
    if name == "prod.default":
        dtype = dim if isinstance(dim, torch.dtype) else dtype
        dim = None
    odt = _acc_dtype(self, dtype)
    return _reduce(RED["prod"], self, None if dim is None else [dim], keepdim, odt, cdt=_cdt(odt))


@_h("any.default", "any.dim", "any.dims", "all.default", "all.dim", "all.dims")
def _anyall(name, self, dim=None, keepdim=False):
    _need(_ok(self))
    k = "any" if name.startswith("any") else "all"
    d = None if dim is None else ([dim] if isinstance(dim, int) else list(dim))
    return _reduce(RED[k], self, d, keepdim, torch.bool, cdt=_cdt(self.dtype) if self.dtype in _FLOATS else 2)


@_h("linalg_vector_norm.default")
def _vnorm(name, self, ord=2, dim=None, keepdim=False, dtype=None):
    _need(_ok(self) and self.dtype in _FLOATS and ord in (1, 2, 1.0, 2.0))
    odt = dtype or self.dtype
    d = None if dim is None else ([dim] if isinstance(dim, int) else list(dim))
    return _reduce(RED["norm2" if ord in (2, 2.0) else "norm1"], self, d, keepdim, odt, cdt=_cdt(odt))


# ---------------------------------------------------------------------------- random
@_h("uniform_.default")
def _uniform(name, self, from_=0.0, to=1.0, generator=None):
    _need(_ok(self) and self.dtype in (torch.float32, torch.bfloat16) and self.is_contiguous() and generator is None)
    seed = int(torch.randint(0, 2**62, (1,)).item())
    N.call("pa_random", N.dt(self), N.ptr(self), self.numel(), 0, float(from_), float(to), seed, N.stream())
    return self


@_h("normal_.default")
def _normal(name, self, mean=0.0, std=1.0, generator=None):
    _need(_ok(self) and self.dtype in (torch.float32, torch.bfloat16) and self.is_contiguous() and generator is None)
    seed = int(torch.randint(0, 2**62, (1,)).item())
    N.call("pa_random", N.dt(self), N.ptr(self), self.numel(), 1, float(mean), float(std), seed, N.stream())
    return self


# ---------------------------------------------------------------------------- softmax
@_h("_softmax.default", "_log_softmax.default")
def _softmax(name, self, dim, half_to_float):
    _need(_ok(self) and self.dtype in (torch.float32, torch.bfloat16) and not half_to_float)
    _need(dim % self.dim() == self.dim() - 1 and self.is_contiguous() and self.shape[-1] > 0)
    y = torch.empty_like(self)
    N.call("pa_softmax_fwd", N.dt(self), N.ptr(self), N.ptr(y), self.numel() // self.shape[-1], self.shape[-1],
           int(name.startswith("_log")), N.stream())
    return y


@_h("_softmax_backward_data.default", "_log_softmax_backward_data.default")
def _softmax_bwd(name, grad, output, dim, input_dtype):
    _need(_ok(grad) and _ok(output) and grad.dtype == output.dtype == input_dtype
          and grad.dtype in (torch.float32, torch.bfloat16))
    _need(dim % grad.dim() == grad.dim() - 1 and grad.is_contiguous() and output.is_contiguous())
    dx = torch.empty_like(grad)
    N.call("pa_softmax_bwd", N.dt(grad), N.ptr(output), N.ptr(grad), N.ptr(dx), grad.numel() // grad.shape[-1],
           grad.shape[-1], int(name.startswith("_log")), N.stream())
    return dx


# ---------------------------------------------------------------------------- matmul
def _bf16_operands(a, b):
    """(A tensor, a_kmaj, B tensor, b_kmaj) in the layouts ops/gemm.py takes, or None."""
    if a.stride(1) == 1:
        A, ak = a, True
    elif a.stride(0) == 1:
        A, ak = a.t(), False
    else:
        return None
    if b.stride(0) == 1:
        Bm, bk = b.t(), True
    elif b.stride(1) == 1:
        Bm, bk = b, False
    else:
        return None
    return A, ak, Bm, bk


def _mm_bf16(a, b, bias=None):
    from . import gemm as G

    M, K = a.shape
    Nn = b.shape[1]
    ops = _bf16_operands(a, b)
    if ops is not None:
        A, ak, Bm, bk = ops
        if G.supported(M, Nn, K, A, Bm):
            return G.gemm(A, Bm, M, Nn, K, a_kmaj=ak, b_kmaj=bk, bias=bias)
    # shapes the bf16 MFMA kernel does not take (a dim not a multiple of 8, e.g. a
    # 10-class head): fp32 operands on the exact-fp32 MFMA GEMM, one rounding back
    from . import blas

    af = _to_copy("_to_copy.default", a, dtype=torch.float32)
    bf = _to_copy("_to_copy.default", b, dtype=torch.float32)
    c = blas._bmm(af, bf)
    if bias is not None:
        _need(_launch(B["add"], c, [c, bias], a=1.0))
    return _to_copy("_to_copy.default", c, dtype=a.dtype)


@_h("mm.default")
def _mm(name, self, mat2):
    _need(_ok(self) and _ok(mat2) and self.dtype == mat2.dtype and self.dim() == 2 and mat2.dim() == 2)
    _need(self.numel() > 0 and mat2.numel() > 0)
    if self.dtype == torch.float32:
        from . import blas

        return blas._bmm(self, mat2)
    _need(self.dtype == torch.bfloat16)
    return _mm_bf16(self, mat2)


@_h("bmm.default")
def _bmm_h(name, self, mat2):
    _need(_ok(self) and _ok(mat2) and self.dtype == mat2.dtype == torch.float32)
    _need(self.dim() == 3 and mat2.dim() == 3 and self.shape[0] <= 65535 and self.numel() > 0 and mat2.numel() > 0)
    from . import blas

    return blas._bmm(self, mat2)


@_h("addmm.default")
def _addmm(name, bias, mat1, mat2, beta=1, alpha=1):
    _need(_ok(bias) and _ok(mat1) and _ok(mat2) and mat1.dtype == mat2.dtype == bias.dtype)
    _need(_sval(beta) == 1 and _sval(alpha) == 1 and mat1.numel() > 0 and mat2.numel() > 0)
    M, K = mat1.shape
    Nn = mat2.shape[1]
    if mat1.dtype == torch.float32:
        from . import convnd as _C

        c = torch.empty(M, Nn, dtype=torch.float32, device=mat1.device)
        _need(_launch(U["copy"], c, [bias], cdt=0))  # bias broadcast into C, GEMM accumulates (beta = 1)
        _C.sgemm(mat1, mat1.stride(0), mat1.stride(1), mat2, mat2.stride(0), mat2.stride(1), c, Nn, M, Nn, K, beta=1.0)
        return c
    _need(mat1.dtype == torch.bfloat16 and (bias.dim() == 1 or (bias.dim() == 2 and bias.shape[0] == 1)))
    b1 = bias.reshape(-1)
    _need(b1.numel() == Nn and b1.is_contiguous())
    return _mm_bf16(mat1, mat2, bias=b1)


# ---------------------------------------------------------------------------- indexing / scans
def _index_select_impl(x, dim, index):
    _need(_ok(x) and _ok(index) and index.dtype in (torch.int64, torch.int32) and index.dim() <= 1)
    nd = x.dim()
    dim = dim % nd if nd else 0
    src = x if x.is_contiguous() else _to_copy("_to_copy.default", x, memory_format=torch.contiguous_format)
    idx = index.reshape(-1)
    if not idx.is_contiguous():
        idx = _to_copy("_to_copy.default", idx, memory_format=torch.contiguous_format)
    shape = list(x.shape)
    outer, nsrc, inner = math.prod(shape[:dim]), shape[dim] if nd else 1, math.prod(shape[dim + 1:])
    shape[dim:dim + 1] = [idx.numel()] if nd else []
    out = torch.empty(shape, dtype=x.dtype, device=x.device)
    rc = _lib().pa_index_select(src.data_ptr(), src.element_size(), outer, nsrc, inner, idx.data_ptr(),
                                int(idx.dtype == torch.int64), idx.numel(), out.data_ptr(), N.stream())
    N.check(rc, "pa_index_select")
    return out


@_h("index_select.default")
def _index_select(name, self, dim, index):
    return _index_select_impl(self, dim, index)


@_h("embedding.default")
def _embedding(name, weight, indices, padding_idx=-1, scale_grad_by_freq=False, sparse=False):
    _need(_ok(weight) and _ok(indices) and weight.dim() == 2)
    flat = indices.reshape(-1)
    out = _index_select_impl(weight, 0, flat)
    return out.reshape(list(indices.shape) + [weight.shape[1]])


@_h("index.Tensor")
def _index(name, self, indices):
    # the common case: one integer index tensor on the first dim (x[idx])
    _need(len(indices) == 1 and indices[0] is not None and _ok(indices[0])
          and indices[0].dtype in (torch.int64, torch.int32))
    ix = indices[0]
    out = _index_select_impl(self, 0, ix.reshape(-1))
    return out.reshape(list(ix.shape) + list(self.shape[1:]))


@_h("arange.start_step", "arange.default", "arange.start")
def _arange(name, *args, dtype=None, layout=None, device=None, pin_memory=None):
    _need(_factory_dev(device))
    vals = [_sval(a) for a in args]
    _need(all(isinstance(v, (int, float)) for v in vals))
    if len(vals) == 1:
        start, end, step = 0, vals[0], 1
    elif len(vals) == 2:
        (start, end), step = vals, 1
    else:
        start, end, step = vals
    if dtype is None:
        dtype = torch.int64 if all(isinstance(v, int) for v in (start, end, step)) else torch.get_default_dtype()
    _need(dtype in _DT and step != 0)
    n = max(0, math.ceil((end - start) / step))
    out = torch.empty(n, dtype=dtype, device=device)
    if n:
        _need(_launch(U["iota"], out, [], a=start, b=step, cdt=_cdt(dtype) if dtype in _FLOATS else 1))
    return out


@_h("constant_pad_nd.default")
def _pad(name, self, pad, value=0):
    _need(_ok(self) and len(pad) % 2 == 0 and len(pad) // 2 <= self.dim() and all(p >= 0 for p in pad))
    shape = list(self.shape)
    sl = []
    for k in range(len(pad) // 2):
        d = self.dim() - 1 - k
        lo, hi = pad[2 * k], pad[2 * k + 1]
        shape[d] += lo + hi
        sl.append((d, lo))
    out = torch.empty(shape, dtype=self.dtype, device=self.device)
    _need(_launch(U["fill"], out, [], a=_sval(value), cdt=_cdt(self.dtype)))
    view = out
    for d, lo in sl:
        view = view.narrow(d, lo, self.shape[d])
    _need(_launch(U["copy"], view, [self], cdt=_cdt(self.dtype)))
    return out


@_h("cumsum.default")
def _cumsum(name, self, dim, dtype=None):
    _need(_ok(self))
    odt = dtype or (torch.int64 if self.dtype in (torch.bool, torch.uint8, torch.int8, torch.int16, torch.int32,
                                                   torch.int64) else self.dtype)
    _need(odt in _DT)
    nd = self.dim()
    dim = dim % nd if nd else 0
    src = self if self.is_contiguous() else _to_copy("_to_copy.default", self, memory_format=torch.contiguous_format)
    shape = list(self.shape)
    out = torch.empty(shape, dtype=odt, device=self.device)
    outer, R, inner = math.prod(shape[:dim]), (shape[dim] if nd else 1), math.prod(shape[dim + 1:])
    rc = _lib().pa_cumsum(_cdt(odt), src.data_ptr(), _DT[src.dtype], out.data_ptr(), _DT[odt], outer, R, inner,
                          N.stream())
    N.check(rc, "pa_cumsum")
    return out


@_h("var.correction", "var_mean.correction", "std.correction")
def _var(name, self, dim=None, correction=None, keepdim=False):
    _need(_ok(self) and self.dtype in _FLOATS and self.numel() > 0)
    corr = 1 if correction is None else _sval(correction)
    dims = _norm_dims(dim, self.dim())
    n = math.prod(self.shape[d] for d in dims) if dims else self.numel()
    mean = _reduce(RED["mean"], self, dims, True, self.dtype)
    dev = torch.empty(self.shape, dtype=torch.float32 if self.dtype != torch.float64 else torch.float64,
                      device=self.device)
    _need(_launch(B["sub"], dev, [self, mean], a=1.0))
    _need(_launch(U["square"], dev, [dev]))
    ss = _reduce(RED["sum"], dev, dims, keepdim, self.dtype, cdt=_cdt(dev.dtype))
    var = torch.empty(ss.shape, dtype=self.dtype, device=self.device)
    _need(_launch(U["affine"], var, [ss], a=1.0 / max(n - corr, 0) if n - corr > 0 else math.nan, b=0.0))
    if name.startswith("std"):
        _need(_launch(U["sqrt"], var, [var]))
        return var
    if name.startswith("var_mean"):
        return var, (mean if keepdim else mean.reshape(ss.shape))
    return var


@_h("topk.default")
def _topk(name, self, k, dim=-1, largest=True, sorted=True):
    _need(_ok(self) and self.dtype in (torch.float32, torch.bfloat16) and largest and self.dim() >= 1)
    _need(dim % self.dim() == self.dim() - 1 and 0 < k <= min(64, self.shape[-1]))
    src = self if self.is_contiguous() else _to_copy("_to_copy.default", self, memory_format=torch.contiguous_format)
    n = self.shape[-1]
    rows = self.numel() // n
    vals = torch.empty(list(self.shape[:-1]) + [k], dtype=self.dtype, device=self.device)
    idx = torch.empty(list(self.shape[:-1]) + [k], dtype=torch.int64, device=self.device)
    N.call("pa_topk", N.dt(src), N.ptr(src), N.ptr(vals), N.ptr(idx), rows, n, k, N.stream())
    return vals, idx
