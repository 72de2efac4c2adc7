"""Tensor creation / manipulation layers (python/paddle/fluid/layers/tensor.py)."""
from __future__ import annotations

import numpy as np

from ...framework import core
from ..framework import Variable, default_main_program
from ..initializer import ConstantInitializer, NumpyArrayInitializer
from ..layer_helper import LayerHelper
from .layer_utils import simple_op

__all__ = ["create_tensor", "create_parameter", "create_global_var", "cast", "concat", "sums", "assign",
           "fill_constant_batch_size_like", "fill_constant", "argmin", "argmax", "argsort", "ones", "zeros",
           "reverse", "has_inf", "has_nan", "isfinite", "zeros_like"]


def create_tensor(dtype, name=None, persistable=False):
    helper = LayerHelper("create_tensor", **locals())
    return helper.create_variable(name=helper.name, dtype=dtype, persistable=persistable)


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from ..param_attr import ParamAttr

    helper = LayerHelper("create_parameter", **locals())
    if attr is None:
        attr = ParamAttr(name=name)
    return helper.create_parameter(attr, shape, dtype, is_bias, default_initializer)


def create_global_var(shape, value, dtype, persistable=False, force_cpu=False, name=None):
    helper = LayerHelper("global_var", **locals())
    var = helper.create_global_variable(dtype=dtype, shape=shape, persistable=persistable, name=name,
                                        stop_gradient=True)
    helper.set_variable_initializer(var, initializer=ConstantInitializer(value=float(value), force_cpu=force_cpu))
    return var


def cast(x, dtype):
    helper = LayerHelper("cast", **locals())
    out = helper.create_variable_for_type_inference(dtype=dtype)
    helper.append_op(type="cast", inputs={"X": [x]}, outputs={"Out": [out]},
                     attrs={"in_dtype": x.dtype, "out_dtype": core.convert_dtype(dtype)})
    return out


def concat(input, axis=0, name=None):
    helper = LayerHelper("concat", **locals())
    out = helper.create_variable_for_type_inference(dtype=helper.input_dtype())
    helper.append_op(type="concat", inputs={"X": input}, outputs={"Out": [out]}, attrs={"axis": axis})
    return out


def sums(input, out=None):
    helper = LayerHelper("sum", **locals())
    if out is None:
        out = helper.create_variable_for_type_inference(dtype=helper.input_dtype())
    helper.append_op(type="sum", inputs={"X": input}, outputs={"Out": out})
    return out


def assign(input, output=None):
    helper = LayerHelper("assign", **locals())
    if isinstance(input, Variable):
        if output is None:
            output = helper.create_variable_for_type_inference(dtype=input.dtype)
        helper.append_op(type="assign", inputs={"X": [input]}, outputs={"Out": [output]})
    else:
        arr = np.asarray(input)
        dtype = core.convert_dtype(arr.dtype)
        if output is None:
            output = helper.create_variable_for_type_inference(dtype=dtype)
        if arr.dtype in (np.float32, np.float64):
            vals = {"fp32_values": [float(v) for v in arr.flat]}
            dtype = core.VT.FP32
        else:
            vals = {"int32_values": [int(v) for v in arr.flat]}
            dtype = core.VT.INT32
        helper.append_op(type="assign_value", outputs={"Out": [output]},
                         attrs=dict(dtype=dtype, shape=list(arr.shape), **vals))
    return output


def fill_constant(shape, dtype, value, force_cpu=False, out=None):
    helper = LayerHelper("fill_constant", **locals())
    if out is None:
        out = helper.create_variable_for_type_inference(dtype=dtype)
    helper.append_op(type="fill_constant", inputs={}, outputs={"Out": [out]},
                     attrs={"shape": list(shape), "dtype": core.convert_dtype(dtype), "value": float(value),
                            "force_cpu": force_cpu})
    out.stop_gradient = True
    return out


def fill_constant_batch_size_like(input, shape, dtype, value, input_dim_idx=0, output_dim_idx=0):
    helper = LayerHelper("fill_constant_batch_size_like", **locals())
    out = helper.create_variable_for_type_inference(dtype=dtype)
    helper.append_op(type="fill_constant_batch_size_like", inputs={"Input": input}, outputs={"Out": [out]},
                     attrs={"shape": list(shape), "dtype": core.convert_dtype(dtype), "value": float(value),
                            "input_dim_idx": input_dim_idx, "output_dim_idx": output_dim_idx})
    out.stop_gradient = True
    return out


def argmin(x, axis=0):
    return simple_op("arg_min", {"X": x}, {"axis": axis}, dtype="int64", stop_gradient=True)


def argmax(x, axis=0):
    return simple_op("arg_max", {"X": x}, {"axis": axis}, dtype="int64", stop_gradient=True)


def argsort(input, axis=-1, name=None):
    helper = LayerHelper("argsort", **locals())
    out = helper.create_variable_for_type_inference(dtype=input.dtype, stop_gradient=True)
    ids = helper.create_variable_for_type_inference("int64", stop_gradient=True)
    helper.append_op(type="argsort", inputs={"X": input}, outputs={"Out": out, "Indices": ids},
                     attrs={"axis": axis})
    return out, ids


def ones(shape, dtype, force_cpu=False):
    return fill_constant(value=1.0, **locals())


def zeros(shape, dtype, force_cpu=False):
    return fill_constant(value=0.0, **locals())


def zeros_like(x, out=None):
    return simple_op("fill_zeros_like", {"X": x}, stop_gradient=True)


def reverse(x, axis):
    if isinstance(axis, int):
        axis = [axis]
    return simple_op("reverse", {"X": x}, {"axis": axis})


def isfinite(x):
    from . import nn

    s = nn.reduce_sum(nn.elementwise_sub(x, x))
    return simple_op("equal", {"X": s, "Y": fill_constant([1], x.dtype, 0.0)}, dtype="bool", stop_gradient=True)


def has_inf(x):
    from . import nn

    a = nn.reduce_max(simple_op("abs", {"X": x}))
    return simple_op("equal", {"X": a, "Y": fill_constant([1], x.dtype, float("inf"))}, dtype="bool")


def has_nan(x):
    return simple_op("not_equal", {"X": x, "Y": x}, dtype="bool")


def _global_step_counter(counter_name=None, begin=1, step=1):
    helper = LayerHelper("global_step_counter")
    if counter_name is None:
        counter_name = "@STEP_COUNTER@"
    gb = default_main_program().global_block()
    if counter_name in gb.vars:
        return gb.vars[counter_name]
    counter = helper.create_global_variable(name=counter_name, dtype="int64", shape=[1], persistable=True)
    helper.set_variable_initializer(counter, ConstantInitializer(value=begin - 1, force_cpu=True))
    gb.prepend_op(type="increment", inputs={"X": [counter]}, outputs={"Out": [counter]},
                  attrs={"step": float(step)})
    counter.stop_gradient = True
    return counter
