"""Operator overloading on fluid Variables (python/paddle/fluid/layers/math_op_patch.py)."""
from __future__ import annotations

from ..framework import Variable
from ..layer_helper import LayerHelper


def _scalar_op(var, scale, bias):
    helper = LayerHelper("scale")
    out = helper.create_variable_for_type_inference(var.dtype)
    helper.append_op(type="scale", inputs={"X": [var]}, outputs={"Out": [out]},
                     attrs={"scale": float(scale), "bias": float(bias)})
    return out


def _to_var(ref, value):
    from .tensor import fill_constant

    return fill_constant(shape=[1], dtype=ref.dtype, value=value)


def _binary(op_type, reverse=False, scalar_method=None):
    def impl(self, other):
        if scalar_method is not None and isinstance(other, (int, float)):
            return scalar_method(self, other)
        if not isinstance(other, Variable):
            other = _to_var(self, other)
        lhs, rhs = (other, self) if reverse else (self, other)
        helper = LayerHelper(op_type)
        out = helper.create_variable_for_type_inference(lhs.dtype)
        helper.append_op(type=op_type, inputs={"X": [lhs], "Y": [rhs]}, outputs={"Out": [out]},
                         attrs={"axis": -1})
        return out

    return impl


def monkey_patch_variable():
    Variable.__add__ = _binary("elementwise_add", scalar_method=lambda v, s: _scalar_op(v, 1.0, s))
    Variable.__radd__ = _binary("elementwise_add", scalar_method=lambda v, s: _scalar_op(v, 1.0, s))
    Variable.__sub__ = _binary("elementwise_sub", scalar_method=lambda v, s: _scalar_op(v, 1.0, -s))
    Variable.__rsub__ = _binary("elementwise_sub", True, scalar_method=lambda v, s: _scalar_op(v, -1.0, s))
    Variable.__mul__ = _binary("elementwise_mul", scalar_method=lambda v, s: _scalar_op(v, s, 0.0))
    Variable.__rmul__ = _binary("elementwise_mul", scalar_method=lambda v, s: _scalar_op(v, s, 0.0))
    Variable.__div__ = _binary("elementwise_div", scalar_method=lambda v, s: _scalar_op(v, 1.0 / s, 0.0))
    Variable.__truediv__ = Variable.__div__
    Variable.__rdiv__ = _binary("elementwise_div", True)
    Variable.__rtruediv__ = Variable.__rdiv__
    Variable.__pow__ = _binary("elementwise_pow")
    Variable.__rpow__ = _binary("elementwise_pow", True)
    Variable.__floordiv__ = _binary("elementwise_floordiv")
    Variable.__mod__ = _binary("elementwise_mod")
    Variable.__eq__ = _binary("equal")
    Variable.__ne__ = _binary("not_equal")
    Variable.__lt__ = _binary("less_than")
    Variable.__le__ = _binary("less_equal")
    Variable.__gt__ = _binary("greater_than")
    Variable.__ge__ = _binary("greater_equal")
    Variable.__hash__ = object.__hash__
    Variable.__neg__ = lambda self: _scalar_op(self, -1.0, 0.0)

    def astype(self, dtype):
        from .tensor import cast

        return cast(self, dtype)

    Variable.astype = astype
