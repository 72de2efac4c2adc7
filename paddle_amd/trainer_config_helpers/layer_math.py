"""v1 layer arithmetic (reference trainer_config_helpers/layer_math.py): unary math
layers (``layer_math.exp(x)`` ...) and the operators of layer outputs in a v1 config
(``1 + x``, ``x - y``, ``2 * y``, ``y * z`` with a width-1 ``z`` ...), expressed with
the v1 layers the reference emits for them (mixed + identity projections,
slope_intercept, scaling, repeat).

LayerOutput is the Fluid Variable here, so the operators are routed to this module
only for layers a v1 config recorded (config_proto's recorder); arithmetic on any
other Variable keeps Fluid's elementwise semantics."""
from __future__ import annotations

from ..v2 import activation as _act

__all__ = ["exp", "sqrt", "reciprocal", "log", "abs", "sigmoid", "tanh", "square", "relu"]


def _t():
    from .. import trainer_config_helpers as t

    return t


def _unary(name, act):
    def f(input, name=None):
        t = _t()
        from . import config_proto as cp

        rec = cp.current()
        nm = name or (rec.name_for(name_of, None) if rec is not None else None)
        return t.mixed_layer(input=[t.identity_projection(input=input)], name=nm, act=act())

    name_of = name
    f.__name__ = name
    return f


exp = _unary("exp", _act.Exp)
sqrt = _unary("sqrt", _act.Sqrt)
reciprocal = _unary("reciprocal", _act.Reciprocal)
log = _unary("log", _act.Log)
abs = _unary("abs", _act.Abs)  # noqa: A001  (the reference's name)
sigmoid = _unary("sigmoid", _act.Sigmoid)
tanh = _unary("tanh", _act.Tanh)
square = _unary("square", _act.Square)
relu = _unary("relu", _act.Relu)


def _size(v):
    from .layers_v1 import _size as s

    return s(v)


def _is_num(x):
    return isinstance(x, (int, float)) and not isinstance(x, bool)


def add(a, b):
    t = _t()
    if _is_num(b):
        a, b = b, a
    if _is_num(a):
        return t.slope_intercept_layer(input=b, slope=1.0, intercept=a)
    sa, sb = _size(a), _size(b)
    if sa != sb and 1 in (sa, sb):  # broadcast the width-1 layer (the second term)
        if sa == 1:
            a, b = b, t.repeat_layer(input=a, num_repeats=sb)
        else:
            b = t.repeat_layer(input=b, num_repeats=sa)
    return t.mixed_layer(input=[t.identity_projection(input=a), t.identity_projection(input=b)])


def sub(a, b):
    t = _t()
    if _is_num(b):
        return t.slope_intercept_layer(input=a, slope=1.0, intercept=-b)
    if _is_num(a):
        neg = t.slope_intercept_layer(input=b, slope=-1.0, intercept=0.0)
        return t.slope_intercept_layer(input=neg, slope=1.0, intercept=a)
    return add(a, t.slope_intercept_layer(input=b, slope=-1.0, intercept=0.0))


def mul(a, b):
    t = _t()
    if _is_num(b):
        a, b = b, a
    if _is_num(a):
        return t.slope_intercept_layer(input=b, slope=a, intercept=0.0)
    if _size(a) == 1:
        return t.scaling_layer(weight=a, input=b)
    if _size(b) == 1:
        return t.scaling_layer(weight=b, input=a)
    raise ValueError("v1 layer product: one operand must be a width-1 layer or a number")


def install():
    """Route the arithmetic of recorded v1 layers through this module (idempotent)."""
    from ..fluid.framework import Variable

    if getattr(Variable, "_pa_v1_math", False):
        return

    def v1(x):
        from . import config_proto as cp

        rec = cp.current()
        return rec is not None and rec.layer_name(x) is not None

    def route(name, v1fn, swap=False):
        fluid_op = getattr(Variable, name)

        def op(self, other):
            if v1(self) and (_is_num(other) or v1(other)):
                return v1fn(other, self) if swap else v1fn(self, other)
            return fluid_op(self, other)
        op.__name__ = name
        setattr(Variable, name, op)

    route("__add__", add)
    route("__radd__", add, swap=True)
    route("__sub__", sub)
    route("__rsub__", sub, swap=True)
    route("__mul__", mul)
    route("__rmul__", mul, swap=True)
    Variable._pa_v1_math = True
