"""Layers auto-generated from registered op protos (layers/ops.py +
layer_function_generator.py:112 in the reference): one function per unary op."""
from __future__ import annotations

from .layer_utils import simple_op

_UNARY = ["sigmoid", "logsigmoid", "exp", "tanh", "tanh_shrink", "softshrink", "abs", "ceil", "floor", "cos",
          "sin", "round", "reciprocal", "square", "softplus", "softsign", "rsqrt", "sign", "silu"]

__all__ = list(_UNARY) + ["hard_shrink", "thresholded_relu", "cumsum", "uniform_random",
                          "gaussian_random", "logical_and", "logical_or", "logical_xor", "logical_not"]


def _gen(op):
    def f(x, name=None):
        return simple_op(op, {"X": x}, name=name)

    f.__name__ = op
    f.__doc__ = f"{op} activation (auto-generated from the '{op}' op proto)."
    return f


for _op in _UNARY:
    globals()[_op] = _gen(_op)


def hard_shrink(x, threshold=None):
    return simple_op("hard_shrink", {"X": x}, {"threshold": 0.5 if threshold is None else threshold})


def thresholded_relu(x, threshold=None):
    return simple_op("thresholded_relu", {"X": x}, {"threshold": 1.0 if threshold is None else threshold})


def cumsum(x, axis=None, exclusive=None, reverse=None):
    return simple_op("cumsum", {"X": x}, {"axis": -1 if axis is None else axis, "exclusive": bool(exclusive),
                                          "reverse": bool(reverse)})


def uniform_random(shape, dtype="float32", min=-1.0, max=1.0, seed=0):
    from ...framework import core

    return simple_op("uniform_random", {}, {"shape": list(shape), "dtype": core.convert_dtype(dtype),
                                            "min": float(min), "max": float(max), "seed": seed}, dtype=dtype)


def gaussian_random(shape, mean=0.0, std=1.0, seed=0, dtype="float32"):
    from ...framework import core

    return simple_op("gaussian_random", {}, {"shape": list(shape), "dtype": core.convert_dtype(dtype),
                                             "mean": float(mean), "std": float(std), "seed": seed}, dtype=dtype)


def _logic(op, unary=False):
    def f(x, y=None, out=None, name=None):
        ins = {"X": x} if unary else {"X": x, "Y": y}
        if out is None:
            return simple_op(op, ins, dtype="bool", name=name)
        # write into the given variable (e.g. a While condition updated in the loop body)
        from ..layer_helper import LayerHelper

        LayerHelper(op, name=name).append_op(type=op, inputs=ins, outputs={"Out": [out]})
        return out

    f.__name__ = op
    return f


logical_and = _logic("logical_and")
logical_or = _logic("logical_or")
logical_xor = _logic("logical_xor")
logical_not = _logic("logical_not", unary=True)
