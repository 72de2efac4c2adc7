"""LayerHelper (python/paddle/fluid/layer_helper.py:30-436): parameter creation with
startup-program initialisation, temp vars, bias / activation appending."""
from __future__ import annotations

import copy

from ..framework import core
from . import unique_name
from .framework import Parameter, Variable, default_main_program, default_startup_program
from .initializer import ConstantInitializer, XavierInitializer
from .param_attr import ParamAttr, WeightNormParamAttr


class LayerHelper:
    def __init__(self, layer_type, **kwargs):
        self.kwargs = kwargs
        self.layer_type = layer_type
        name = self.kwargs.get("name", None)
        if name is None:
            self.kwargs["name"] = unique_name.generate(self.layer_type)

    @property
    def name(self):
        return self.kwargs["name"]

    @property
    def main_program(self):
        return default_main_program()

    @property
    def startup_program(self):
        return default_startup_program()

    def append_op(self, *args, **kwargs):
        return self.main_program.current_block().append_op(*args, **kwargs)

    def multiple_input(self, input_param_name="input"):
        """The layer argument ``input_param_name`` as a list of Variables."""
        got = self.kwargs.get(input_param_name, [])
        if isinstance(got, Variable):
            return [got]
        if not isinstance(got, (list, tuple)):
            raise TypeError(f"{self.layer_type}: argument {input_param_name!r} must be a Variable or a list "
                            f"of Variables, got {type(got).__name__}")
        return list(got)

    def input(self, input_param_name="input"):
        got = self.multiple_input(input_param_name)
        if len(got) != 1:
            raise ValueError(f"{self.layer_type} expects exactly one {input_param_name!r}, got {len(got)}")
        return got[0]

    @property
    def param_attr(self):
        return ParamAttr._to_attr(self.kwargs.get("param_attr", None))

    @property
    def bias_attr(self):
        return ParamAttr._to_attr(self.kwargs.get("bias_attr", None))

    def multiple_param_attr(self, length):
        """One ParamAttr per input: a single attribute is replicated (each copy
        independent, so generated names differ); otherwise the counts must match."""
        attrs = self.param_attr
        attrs = [attrs] if isinstance(attrs, ParamAttr) else list(attrs)
        if len(attrs) == length:
            return attrs
        if len(attrs) == 1:
            return [copy.deepcopy(attrs[0]) for _ in range(length)]
        raise ValueError(f"{self.layer_type}: {len(attrs)} param_attr entries for {length} inputs")

    def iter_inputs_and_params(self, input_param_name="input"):
        ins = self.multiple_input(input_param_name)
        return zip(ins, self.multiple_param_attr(len(ins)))

    def input_dtype(self, input_param_name="input"):
        """The common dtype of the inputs (None when there are none)."""
        dtypes = {v.dtype for v in self.multiple_input(input_param_name)}
        if len(dtypes) > 1:
            raise ValueError(f"{self.layer_type}: inputs mix dtypes {sorted(map(str, dtypes))}")
        return next(iter(dtypes), None)

    def create_parameter(self, attr, shape, dtype, is_bias=False, default_initializer=None):
        if attr is False:
            return None
        attr = copy.deepcopy(attr) if attr is not None else ParamAttr()
        assert isinstance(attr, ParamAttr)
        suffix = "b" if is_bias else "w"
        if attr.name is None:
            attr.name = unique_name.generate(".".join([self.name, suffix]))
        if default_initializer is None and attr.initializer is None:
            if is_bias:
                attr._set_default_bias_initializer()
            else:
                attr._set_default_param_initializer()
        elif default_initializer is not None:
            attr._set_default_initializer(default_initializer)
        shape = [int(s) for s in shape]
        # startup program: var + init op
        sb = self.startup_program.global_block()
        if attr.name not in sb.vars:
            sv = sb.create_var(name=attr.name, shape=shape, dtype=dtype, persistable=True)
            attr.initializer(sv, sb)
        return self.main_program.global_block().create_parameter(shape=shape, dtype=dtype,
                                                                 **attr._to_kwargs(with_initializer=False))

    def get_parameter(self, name):
        p = self.main_program.global_block().var(name)
        if not isinstance(p, Parameter):
            raise ValueError(f"no Parameter name {name} found")
        return p

    def create_variable_for_type_inference(self, dtype, stop_gradient=False):
        return self.main_program.current_block().create_var(
            name=unique_name.generate(".".join([self.name, "tmp"])), dtype=dtype, persistable=False,
            stop_gradient=stop_gradient)

    create_tmp_variable = create_variable_for_type_inference

    def create_variable(self, *args, **kwargs):
        return self.main_program.current_block().create_var(*args, **kwargs)

    def create_global_variable(self, persistable=False, *args, **kwargs):
        return self.main_program.global_block().create_var(*args, persistable=persistable, **kwargs)

    def set_variable_initializer(self, var, initializer):
        sb = self.startup_program.global_block()
        sv = sb.create_var(name=var.name, type=var.type, dtype=var.dtype, shape=var.shape,
                           persistable=True)
        initializer(sv, sb)

    def append_bias_op(self, input_var, dim_start=1, dim_end=None):
        size = list(input_var.shape[dim_start:dim_end])
        bias_attr = self.bias_attr
        if not bias_attr:
            return input_var
        b = self.create_parameter(attr=bias_attr, shape=size, dtype=input_var.dtype, is_bias=True)
        tmp = self.create_variable_for_type_inference(dtype=input_var.dtype)
        self.append_op(type="elementwise_add", inputs={"X": [input_var], "Y": [b]}, outputs={"Out": [tmp]},
                       attrs={"axis": dim_start})
        return tmp

    def append_activation(self, input_var):
        act = self.kwargs.get("act", None)
        if act is None:
            return input_var
        if isinstance(act, str):
            act = {"type": act}
        act = dict(act)
        act_type = act.pop("type")
        tmp = self.create_variable_for_type_inference(dtype=input_var.dtype)
        self.append_op(type=act_type, inputs={"X": [input_var]}, outputs={"Out": [tmp]}, attrs=act)
        return tmp

    def _get_default_initializer(self, dtype):
        if dtype is None or core.convert_dtype(dtype) in (core.VT.FP16, core.VT.FP32, core.VT.FP64,
                                                          core.VT.BF16):
            return XavierInitializer()
        return ConstantInitializer()

    def is_instance(self, param_name, cls):
        param = self.kwargs.get(param_name, None)
        if not isinstance(param, cls):
            raise TypeError(f"The input {param_name} parameter of method {self.layer_type} must be {cls}")
