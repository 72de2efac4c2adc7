"""Sequence (LoD) layers from python/paddle/fluid/layers/nn.py (sequence_* family)."""
from __future__ import annotations

from ..layer_helper import LayerHelper
from .layer_utils import simple_op

__all__ = ["sequence_pool", "sequence_softmax", "sequence_expand", "sequence_expand_as", "sequence_concat",
           "sequence_conv", "sequence_erase", "sequence_reshape", "sequence_slice", "sequence_pad",
           "sequence_unpad", "sequence_mask", "sequence_enumerate", "sequence_first_step",
           "sequence_last_step", "lod_reset", "sequence_scatter"]


def sequence_pool(input, pool_type, is_test=False):
    return simple_op("sequence_pool", {"X": input}, {"pooltype": pool_type.upper(), "is_test": is_test},
                     extra_outputs=("MaxIndex",))[0]


def sequence_first_step(input):
    return sequence_pool(input, "first")


def sequence_last_step(input):
    return sequence_pool(input, "last")


def sequence_softmax(input, use_cudnn=False, name=None):
    return simple_op("sequence_softmax", {"X": input}, {"use_cudnn": use_cudnn}, name=name)


def sequence_expand(x, y, ref_level=-1, name=None):
    return simple_op("sequence_expand", {"X": x, "Y": y}, {"ref_level": ref_level}, name=name)


def sequence_expand_as(x, y, name=None):
    return simple_op("sequence_expand_as", {"X": x, "Y": y}, name=name)


def sequence_concat(input, name=None):
    out = simple_op("sequence_concat", {"X": input}, name=name)
    out.lod_level = max(int(getattr(v, "lod_level", 0) or 0) for v in input)  # a sequence batch like its inputs
    return out


def sequence_conv(input, num_filters, filter_size=3, filter_stride=1, padding=None, bias_attr=None,
                  param_attr=None, act=None, name=None):
    helper = LayerHelper("sequence_conv", **locals())
    dtype = helper.input_dtype()
    w = helper.create_parameter(attr=helper.param_attr, shape=[filter_size * input.shape[1], num_filters],
                                dtype=dtype)
    pre_bias = helper.create_variable_for_type_inference(dtype)
    helper.append_op(type="sequence_conv", inputs={"X": [input], "Filter": [w]}, outputs={"Out": pre_bias},
                     attrs={"contextStride": filter_stride, "contextStart": -int(filter_size // 2),
                            "contextLength": filter_size})
    pre_act = helper.append_bias_op(pre_bias)
    return helper.append_activation(pre_act)


def sequence_erase(input, tokens, name=None):
    return simple_op("sequence_erase", {"X": input}, {"tokens": list(tokens)}, name=name)


def sequence_reshape(input, new_dim):
    out = simple_op("sequence_reshape", {"X": input}, {"new_dim": new_dim})
    out.lod_level = max(int(getattr(input, "lod_level", 0) or 0), 1)
    return out


def sequence_slice(input, offset, length, name=None):
    return simple_op("sequence_slice", {"X": input, "Offset": offset, "Length": length}, name=name)


def sequence_pad(x, pad_value, maxlen=None, name=None):
    return simple_op("sequence_pad", {"X": x, "PadValue": pad_value},
                     {"padded_length": -1 if maxlen is None else maxlen}, extra_outputs=("Length",), name=name)


def sequence_unpad(x, length, name=None):
    return simple_op("sequence_unpad", {"X": x, "Length": length}, name=name)


def sequence_mask(x, maxlen=None, dtype="int64", name=None):
    from ...framework import core

    return simple_op("sequence_mask", {"X": x}, {"maxlen": -1 if maxlen is None else maxlen,
                                                 "out_dtype": core.convert_dtype(dtype)}, out_slot="Y",
                     dtype=dtype, name=name)


def sequence_enumerate(input, win_size, pad_value=0, name=None):
    return simple_op("sequence_enumerate", {"X": input}, {"win_size": win_size, "pad_value": pad_value},
                     name=name)


def lod_reset(x, y=None, target_lod=None):
    inputs = {"X": x}
    if y is not None:
        inputs["Y"] = y
    return simple_op("lod_reset", inputs, {"target_lod": list(target_lod or [])})


def sequence_scatter(input, index, updates, name=None):
    return simple_op("sequence_scatter", {"X": input, "Ids": index, "Updates": updates}, name=name)
