"""Neural-network layers (python/paddle/fluid/layers/nn.py).

Signatures follow paddle/fluid/API.spec; each layer appends the same op types,
slot names and attributes as the reference (fc :117, embedding :229, dropout :917,
cross_entropy :970, softmax :1318, conv2d :1372, pool2d :1845, batch_norm :2007,
layer_norm :2158, matmul :3386, transpose :3997, softmax_with_cross_entropy :4247,
reshape :4434, ...).
"""
from __future__ import annotations

import numpy as np

from ...framework import core
from ..framework import Variable
from ..initializer import ConstantInitializer, NormalInitializer
from ..layer_helper import LayerHelper
from ..param_attr import ParamAttr
from .layer_utils import simple_op

__all__ = []


def _export(fn):
    __all__.append(fn.__name__)
    return fn


@_export
def fc(input, size, num_flatten_dims=1, param_attr=None, bias_attr=None, use_mkldnn=False, act=None,
       is_test=False, name=None):
    helper = LayerHelper("fc", **locals())
    dtype = helper.input_dtype()
    mul_results = []
    for input_var, pa in helper.iter_inputs_and_params():
        input_shape = input_var.shape
        param_shape = [int(np.prod(input_shape[num_flatten_dims:]))] + [size]
        w = helper.create_parameter(attr=pa, shape=param_shape, dtype=dtype, is_bias=False)
        tmp = helper.create_variable_for_type_inference(dtype)
        helper.append_op(type="mul", inputs={"X": input_var, "Y": w}, outputs={"Out": tmp},
                         attrs={"x_num_col_dims": num_flatten_dims, "y_num_col_dims": 1})
        mul_results.append(tmp)
    if len(mul_results) == 1:
        pre_bias = mul_results[0]
    else:
        pre_bias = helper.create_variable_for_type_inference(dtype)
        helper.append_op(type="sum", inputs={"X": mul_results}, outputs={"Out": pre_bias})
    pre_activation = helper.append_bias_op(pre_bias, dim_start=num_flatten_dims)
    return helper.append_activation(pre_activation)


@_export
def embedding(input, size, is_sparse=False, is_distributed=False, padding_idx=None, param_attr=None,
              dtype="float32"):
    helper = LayerHelper("embedding", **locals())
    w = helper.create_parameter(attr=helper.param_attr, shape=size, dtype=dtype, is_bias=False)
    tmp = helper.create_variable_for_type_inference(dtype)
    padding_idx = -1 if padding_idx is None else padding_idx if padding_idx >= 0 else (size[0] + padding_idx)
    helper.append_op(type="lookup_table", inputs={"Ids": input, "W": w}, outputs={"Out": tmp},
                     attrs={"is_sparse": is_sparse, "is_distributed": is_distributed, "padding_idx": padding_idx})
    return tmp


@_export
def dropout(x, dropout_prob, is_test=False, seed=None, name=None, dropout_implementation="downgrade_in_infer"):
    helper = LayerHelper("dropout", **locals())
    out = helper.create_variable_for_type_inference(dtype=x.dtype)
    mask = helper.create_variable_for_type_inference(dtype=x.dtype, stop_gradient=True)
    helper.append_op(type="dropout", inputs={"X": [x]}, outputs={"Out": [out], "Mask": [mask]},
                     attrs={"dropout_prob": dropout_prob, "is_test": is_test, "fix_seed": seed is not None,
                            "seed": seed if seed is not None else 0,
                            "dropout_implementation": dropout_implementation})
    return out


@_export
def cross_entropy(input, label, soft_label=False, ignore_index=-100):
    return simple_op("cross_entropy", {"X": [input], "Label": [label]},
                     {"soft_label": soft_label, "ignore_index": ignore_index}, out_slot="Y")


@_export
def square_error_cost(input, label):
    helper = LayerHelper("square_error_cost", **locals())
    minus_out = helper.create_variable_for_type_inference(dtype=input.dtype)
    helper.append_op(type="elementwise_sub", inputs={"X": [input], "Y": [label]}, outputs={"Out": [minus_out]})
    square_out = helper.create_variable_for_type_inference(dtype=input.dtype)
    helper.append_op(type="square", inputs={"X": [minus_out]}, outputs={"Out": [square_out]})
    return square_out


@_export
def softmax(input, use_cudnn=True, name=None, axis=-1):
    return simple_op("softmax", {"X": [input]}, {"use_cudnn": use_cudnn, "axis": axis}, name=name)


@_export
def log_softmax(input, axis=-1, name=None):
    return simple_op("log_softmax", {"X": [input]}, {"axis": axis}, name=name)


def _pair(v, n=2):
    return list(v) if isinstance(v, (list, tuple)) else [v] * n


@_export
def conv2d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None, param_attr=None,
           bias_attr=None, use_cudnn=True, use_mkldnn=False, act=None, name=None):
    helper = LayerHelper("conv2d", **locals())
    dtype = helper.input_dtype()
    num_channels = input.shape[1]
    groups = groups or 1
    l_type = "depthwise_conv2d" if (num_channels == groups and num_filters % num_channels == 0 and groups > 1) \
        else "conv2d"
    fs = _pair(filter_size)
    filter_shape = [num_filters, num_channels // groups] + fs
    std = (2.0 / (fs[0] * fs[1] * num_channels)) ** 0.5
    w = helper.create_parameter(attr=helper.param_attr, shape=filter_shape, dtype=dtype,
                                default_initializer=NormalInitializer(0.0, std, 0))
    pre_bias = helper.create_variable_for_type_inference(dtype)
    helper.append_op(type=l_type, inputs={"Input": input, "Filter": w}, outputs={"Output": pre_bias},
                     attrs={"strides": _pair(stride), "paddings": _pair(padding), "dilations": _pair(dilation),
                            "groups": groups, "use_cudnn": use_cudnn, "use_mkldnn": use_mkldnn})
    pre_act = helper.append_bias_op(pre_bias, dim_start=1, dim_end=2)
    return helper.append_activation(pre_act)


@_export
def conv3d(input, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None, param_attr=None,
           bias_attr=None, use_cudnn=True, use_mkldnn=False, act=None, name=None):
    helper = LayerHelper("conv3d", **locals())
    dtype = helper.input_dtype()
    groups = groups or 1
    fs = _pair(filter_size, 3)
    filter_shape = [num_filters, input.shape[1] // groups] + fs
    std = (2.0 / (int(np.prod(fs)) * input.shape[1])) ** 0.5
    w = helper.create_parameter(attr=helper.param_attr, shape=filter_shape, dtype=dtype,
                                default_initializer=NormalInitializer(0.0, std, 0))
    pre_bias = helper.create_variable_for_type_inference(dtype)
    helper.append_op(type="conv3d", inputs={"Input": input, "Filter": w}, outputs={"Output": pre_bias},
                     attrs={"strides": _pair(stride, 3), "paddings": _pair(padding, 3),
                            "dilations": _pair(dilation, 3), "groups": groups, "use_cudnn": use_cudnn})
    pre_act = helper.append_bias_op(pre_bias, dim_start=1, dim_end=2)
    return helper.append_activation(pre_act)


@_export
def conv2d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None):
    helper = LayerHelper("conv2d_transpose", **locals())
    dtype = helper.input_dtype()
    groups = groups or 1
    padding, stride, dilation = _pair(padding), _pair(stride), _pair(dilation)
    if filter_size is None:
        output_size = _pair(output_size)
        h_in, w_in = input.shape[2], input.shape[3]
        fh = (output_size[0] - (h_in - 1) * stride[0] + 2 * padding[0] - 1) // dilation[0] + 1
        fw = (output_size[1] - (w_in - 1) * stride[1] + 2 * padding[1] - 1) // dilation[1] + 1
        filter_size = [fh, fw]
    filter_shape = [input.shape[1], num_filters // groups] + _pair(filter_size)
    w = helper.create_parameter(dtype=dtype, shape=filter_shape, attr=helper.param_attr)
    pre_bias = helper.create_variable_for_type_inference(dtype)
    helper.append_op(type="conv2d_transpose", inputs={"Input": [input], "Filter": [w]},
                     outputs={"Output": pre_bias},
                     attrs={"output_size": _pair(output_size) if output_size else [], "strides": stride,
                            "paddings": padding, "dilations": dilation, "groups": groups, "use_cudnn": use_cudnn})
    out = helper.append_bias_op(pre_bias, dim_start=1, dim_end=2)
    return helper.append_activation(out)


@_export
def pool2d(input, pool_size=-1, pool_type="max", pool_stride=1, pool_padding=0, global_pooling=False,
           use_cudnn=True, ceil_mode=False, name=None, exclusive=True):
    if pool_type not in ("max", "avg"):
        raise ValueError("Unknown pool_type")
    return simple_op("pool2d", {"X": input},
                     {"pooling_type": pool_type, "ksize": _pair(pool_size), "global_pooling": global_pooling,
                      "strides": _pair(pool_stride), "paddings": _pair(pool_padding), "use_cudnn": use_cudnn,
                      "ceil_mode": ceil_mode, "exclusive": exclusive}, name=name)


@_export
def pool3d(input, pool_size=-1, pool_type="max", pool_stride=1, pool_padding=0, global_pooling=False,
           use_cudnn=True, ceil_mode=False, name=None, exclusive=True):
    return simple_op("pool3d", {"X": input},
                     {"pooling_type": pool_type, "ksize": _pair(pool_size, 3), "global_pooling": global_pooling,
                      "strides": _pair(pool_stride, 3), "paddings": _pair(pool_padding, 3),
                      "ceil_mode": ceil_mode, "exclusive": exclusive}, name=name)


@_export
def batch_norm(input, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None,
               data_layout="NCHW", in_place=False, name=None, moving_mean_name=None, moving_variance_name=None,
               do_model_average_for_mean_and_var=False, fuse_with_relu=False, use_global_stats=False):
    helper = LayerHelper("batch_norm", **locals())
    dtype = helper.input_dtype()
    input_shape = input.shape
    channel_num = input_shape[1] if data_layout == "NCHW" else input_shape[-1]
    param_shape = [channel_num]
    scale = helper.create_parameter(attr=helper.param_attr, shape=param_shape, dtype=dtype,
                                    default_initializer=ConstantInitializer(1.0))
    bias = helper.create_parameter(attr=helper.bias_attr, shape=param_shape, dtype=dtype, is_bias=True)
    mean = helper.create_parameter(attr=ParamAttr(name=moving_mean_name, initializer=ConstantInitializer(0.0),
                                                  trainable=False, do_model_average=do_model_average_for_mean_and_var),
                                   shape=param_shape, dtype=dtype)
    mean.stop_gradient = True
    variance = helper.create_parameter(attr=ParamAttr(name=moving_variance_name,
                                                      initializer=ConstantInitializer(1.0), trainable=False,
                                                      do_model_average=do_model_average_for_mean_and_var),
                                       shape=param_shape, dtype=dtype)
    variance.stop_gradient = True
    saved_mean = helper.create_variable_for_type_inference(dtype=dtype, stop_gradient=True)
    saved_variance = helper.create_variable_for_type_inference(dtype=dtype, stop_gradient=True)
    out = input if in_place else helper.create_variable_for_type_inference(dtype)
    helper.append_op(type="batch_norm",
                     inputs={"X": input, "Scale": scale, "Bias": bias, "Mean": mean, "Variance": variance},
                     outputs={"Y": out, "MeanOut": mean, "VarianceOut": variance, "SavedMean": saved_mean,
                              "SavedVariance": saved_variance},
                     attrs={"momentum": momentum, "epsilon": epsilon, "is_test": is_test,
                            "data_layout": data_layout, "fuse_with_relu": fuse_with_relu,
                            "use_global_stats": use_global_stats})
    return helper.append_activation(out)


@_export
def layer_norm(input, scale=True, shift=True, begin_norm_axis=1, epsilon=1e-05, param_attr=None, bias_attr=None,
               act=None, name=None):
    helper = LayerHelper("layer_norm", **locals())
    dtype = helper.input_dtype()
    inputs = {"X": input}
    param_shape = [int(np.prod(input.shape[begin_norm_axis:]))]
    if scale:
        inputs["Scale"] = helper.create_parameter(attr=helper.param_attr, shape=param_shape, dtype=dtype,
                                                  default_initializer=ConstantInitializer(1.0))
    if shift:
        inputs["Bias"] = helper.create_parameter(attr=helper.bias_attr, shape=param_shape, dtype=dtype,
                                                 is_bias=True)
    mean_out = helper.create_variable_for_type_inference(dtype=dtype, stop_gradient=True)
    variance_out = helper.create_variable_for_type_inference(dtype=dtype, stop_gradient=True)
    out = helper.create_variable_for_type_inference(dtype)
    helper.append_op(type="layer_norm", inputs=inputs,
                     outputs={"Y": out, "Mean": mean_out, "Variance": variance_out},
                     attrs={"epsilon": epsilon, "begin_norm_axis": begin_norm_axis})
    return helper.append_activation(out)


@_export
def softmax_with_cross_entropy(logits, label, soft_label=False, ignore_index=-100, numeric_stable_mode=False,
                               return_softmax=False):
    helper = LayerHelper("softmax_with_cross_entropy", **locals())
    softmax_ = helper.create_variable_for_type_inference(dtype=logits.dtype)
    loss = helper.create_variable_for_type_inference(dtype=logits.dtype)
    helper.append_op(type="softmax_with_cross_entropy", inputs={"Logits": logits, "Label": label},
                     outputs={"Softmax": softmax_, "Loss": loss},
                     attrs={"soft_label": soft_label, "ignore_index": ignore_index,
                            "numeric_stable_mode": numeric_stable_mode})
    if return_softmax:
        return loss, softmax_
    return loss


@_export
def sigmoid_cross_entropy_with_logits(x, label, ignore_index=-100, name=None):
    return simple_op("sigmoid_cross_entropy_with_logits", {"X": [x], "Label": [label]},
                     {"ignore_index": ignore_index}, name=name)


@_export
def matmul(x, y, transpose_x=False, transpose_y=False, alpha=1.0, name=None):
    return simple_op("matmul", {"X": x, "Y": y}, {"transpose_X": transpose_x, "transpose_Y": transpose_y,
                                                  "alpha": float(alpha)}, name=name)


@_export
def mul(x, y, x_num_col_dims=1, y_num_col_dims=1, name=None):
    return simple_op("mul", {"X": x, "Y": y}, {"x_num_col_dims": x_num_col_dims, "y_num_col_dims": y_num_col_dims},
                     name=name)


@_export
def topk(input, k, name=None):
    helper = LayerHelper("top_k", **locals())
    values = helper.create_variable_for_type_inference(dtype=input.dtype)
    indices = helper.create_variable_for_type_inference(dtype="int64", stop_gradient=True)
    helper.append_op(type="top_k", inputs={"X": [input]}, outputs={"Out": [values], "Indices": [indices]},
                     attrs={"k": k})
    values.stop_gradient = True
    return values, indices


@_export
def transpose(x, perm, name=None):
    return simple_op("transpose", {"X": [x]}, {"axis": list(perm)}, name=name)


@_export
def reshape(x, shape, actual_shape=None, act=None, inplace=False, name=None):
    helper = LayerHelper("reshape", **locals())
    inputs = {"X": x}
    if isinstance(actual_shape, Variable):
        inputs["Shape"] = actual_shape
    out = helper.create_variable_for_type_inference(dtype=x.dtype)
    helper.append_op(type="reshape", inputs=inputs, outputs={"Out": out}, attrs={"shape": list(shape)})
    return helper.append_activation(out)


@_export
def squeeze(input, axes, name=None):
    return simple_op("squeeze", {"X": input}, {"axes": list(axes)}, name=name)


@_export
def unsqueeze(input, axes, name=None):
    return simple_op("unsqueeze", {"X": input}, {"axes": list(axes)}, name=name)


@_export
def flatten(x, axis=1, name=None):
    return simple_op("flatten", {"X": x}, {"axis": axis}, name=name)


@_export
def split(input, num_or_sections, dim=-1, name=None):
    helper = LayerHelper("split", **locals())
    input_shape = input.shape
    dim = (len(input_shape) + dim) if dim < 0 else dim
    if isinstance(num_or_sections, int):
        num = num_or_sections
        sections = []
    else:
        num = len(num_or_sections)
        sections = list(num_or_sections)
    outs = [helper.create_variable_for_type_inference(dtype=input.dtype) for _ in range(num)]
    helper.append_op(type="split", inputs={"X": input}, outputs={"Out": outs},
                     attrs={"num": num if not sections else 0, "sections": sections, "axis": dim})
    return outs


@_export
def stack(x, axis=0):
    helper = LayerHelper("stack", **locals())
    if not isinstance(x, (list, tuple)):
        x = [x]
    out = helper.create_variable_for_type_inference(x[0].dtype)
    helper.append_op(type="stack", inputs={"X": x}, outputs={"Y": out}, attrs={"axis": axis})
    return out


@_export
def unstack(x, axis=0, num=None):
    helper = LayerHelper("unstack", **locals())
    if num is None:
        num = x.shape[axis]
    outs = [helper.create_variable_for_type_inference(x.dtype) for _ in range(num)]
    helper.append_op(type="unstack", inputs={"X": [x]}, outputs={"Y": outs}, attrs={"axis": axis, "num": num})
    return outs


@_export
def expand(x, expand_times, name=None):
    return simple_op("expand", {"X": x}, {"expand_times": list(expand_times)}, name=name)


@_export
def gather(input, index):
    return simple_op("gather", {"X": input, "Index": index})


@_export
def scatter(input, index, updates, name=None, overwrite=True):
    return simple_op("scatter", {"X": input, "Ids": index, "Updates": updates}, {"overwrite": overwrite}, name=name)


@_export
def slice(input, axes, starts, ends):
    return simple_op("slice", {"Input": input}, {"axes": list(axes), "starts": list(starts), "ends": list(ends)})


@_export
def shape(input):
    return simple_op("shape", {"Input": input}, dtype="int32", stop_gradient=True)


@_export
def one_hot(input, depth):
    return simple_op("one_hot", {"X": input}, {"depth": depth}, dtype="float32", stop_gradient=True)


@_export
def mean(x, name=None):
    return simple_op("mean", {"X": [x]}, {}, name=name)


def _reduce(op_type, input, dim, keep_dim, name):
    if dim is not None and not isinstance(dim, list):
        dim = [dim]
    return simple_op(op_type, {"X": input}, {"dim": dim if dim is not None else [0], "keep_dim": keep_dim,
                                             "reduce_all": dim is None}, name=name)


@_export
def reduce_sum(input, dim=None, keep_dim=False, name=None):
    return _reduce("reduce_sum", input, dim, keep_dim, name)


@_export
def reduce_mean(input, dim=None, keep_dim=False, name=None):
    return _reduce("reduce_mean", input, dim, keep_dim, name)


@_export
def reduce_max(input, dim=None, keep_dim=False, name=None):
    return _reduce("reduce_max", input, dim, keep_dim, name)


@_export
def reduce_min(input, dim=None, keep_dim=False, name=None):
    return _reduce("reduce_min", input, dim, keep_dim, name)


@_export
def reduce_prod(input, dim=None, keep_dim=False, name=None):
    return _reduce("reduce_prod", input, dim, keep_dim, name)


def _elementwise(op_type, x, y, axis, act, name):
    helper = LayerHelper(op_type, **locals())
    out = helper.create_variable_for_type_inference(dtype=x.dtype)
    helper.append_op(type=op_type, inputs={"X": x, "Y": y}, outputs={"Out": out}, attrs={"axis": axis})
    return helper.append_activation(out)


for _op in ("add", "sub", "mul", "div", "max", "min", "pow", "mod", "floordiv"):
    def _mk(op):
        def f(x, y, axis=-1, act=None, name=None):
            return _elementwise("elementwise_" + op, x, y, axis, act, name)

        f.__name__ = "elementwise_" + op
        return f

    globals()["elementwise_" + _op] = _mk(_op)
    __all__.append("elementwise_" + _op)


@_export
def clip(x, min, max, name=None):
    return simple_op("clip", {"X": x}, {"min": float(min), "max": float(max)}, name=name)


@_export
def clip_by_norm(x, max_norm, name=None):
    return simple_op("clip_by_norm", {"X": x}, {"max_norm": float(max_norm)}, name=name)


@_export
def scale(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    helper = LayerHelper("scale", **locals())
    out = helper.create_variable_for_type_inference(dtype=x.dtype)
    helper.append_op(type="scale", inputs={"X": x}, outputs={"Out": out},
                     attrs={"scale": float(scale), "bias": float(bias), "bias_after_scale": bias_after_scale})
    return helper.append_activation(out)


@_export
def sums(input, out=None):
    helper = LayerHelper("sum", **locals())
    if out is None:
        out = helper.create_variable_for_type_inference(dtype=input[0].dtype)
    helper.append_op(type="sum", inputs={"X": input}, outputs={"Out": out})
    return out


@_export
def l2_normalize(x, axis, epsilon=1e-12, name=None):
    if len(x.shape) == 1:
        axis = 0
    return simple_op("norm", {"X": x}, {"axis": 1 if axis is None else axis, "epsilon": epsilon},
                     extra_outputs=("Norm",), name=name)[0]


@_export
def lrn(input, n=5, k=1.0, alpha=1e-4, beta=0.75, name=None):
    return simple_op("lrn", {"X": input}, {"n": n, "k": k, "alpha": alpha, "beta": beta},
                     extra_outputs=("MidOut",), name=name)[0]


@_export
def pad(x, paddings, pad_value=0.0, name=None):
    return simple_op("pad", {"X": x}, {"paddings": list(paddings), "pad_value": float(pad_value)}, name=name)


@_export
def pad2d(input, paddings=[0, 0, 0, 0], mode="constant", pad_value=0.0, data_format="NCHW", name=None):
    return simple_op("pad2d", {"X": input}, {"paddings": list(paddings), "mode": mode,
                                              "pad_value": float(pad_value), "data_format": data_format}, name=name)


@_export
def pad_constant_like(x, y, pad_value=0.0, name=None):
    return simple_op("pad_constant_like", {"X": x, "Y": y}, {"pad_value": float(pad_value)}, name=name)


@_export
def crop(x, shape=None, offsets=None, name=None):
    inputs = {"X": x}
    attrs = {"offsets": list(offsets) if offsets else [0] * len(x.shape)}
    if isinstance(shape, Variable):
        inputs["Y"] = shape
    else:
        attrs["shape"] = list(shape)
    return simple_op("crop", inputs, attrs, name=name)


@_export
def label_smooth(label, prior_dist=None, epsilon=0.1, dtype="float32", name=None):
    inputs = {"X": label}
    if prior_dist is not None:
        inputs["PriorDist"] = prior_dist
    return simple_op("label_smooth", inputs, {"epsilon": float(epsilon)}, name=name)


@_export
def image_resize(input, out_shape=None, scale=None, name=None, resample="BILINEAR", actual_shape=None):
    op = "bilinear_interp" if resample == "BILINEAR" else "nearest_interp"
    attrs = {"interp_method": resample.lower()}
    if out_shape is not None:
        attrs["out_h"], attrs["out_w"] = int(out_shape[0]), int(out_shape[1])
    elif scale is not None:
        attrs["out_h"], attrs["out_w"] = int(input.shape[2] * scale), int(input.shape[3] * scale)
    inputs = {"X": input}
    if actual_shape is not None:
        inputs["OutSize"] = actual_shape
    return simple_op(op, inputs, attrs, name=name)


@_export
def resize_bilinear(input, out_shape=None, scale=None, name=None, actual_shape=None):
    return image_resize(input, out_shape, scale, name, "BILINEAR", actual_shape)


@_export
def resize_nearest(input, out_shape=None, scale=None, name=None, actual_shape=None):
    return image_resize(input, out_shape, scale, name, "NEAREST", actual_shape)


@_export
def image_resize_short(input, out_short_len, resample="BILINEAR"):
    h, w = input.shape[2], input.shape[3]
    short = min(h, w)
    ratio = out_short_len / float(short)
    return image_resize(input, [int(h * ratio + 0.5), int(w * ratio + 0.5)], resample=resample)


@_export
def prelu(x, mode, param_attr=None, name=None):
    helper = LayerHelper("prelu", **locals())
    if mode == "all":
        alpha_shape = [1]
    elif mode == "channel":
        alpha_shape = [1, x.shape[1], 1, 1]
    else:
        alpha_shape = list(x.shape)
    alpha = helper.create_parameter(attr=helper.param_attr, shape=alpha_shape, dtype="float32",
                                    default_initializer=ConstantInitializer(0.25))
    out = helper.create_variable_for_type_inference(x.dtype)
    helper.append_op(type="prelu", inputs={"X": x, "Alpha": alpha}, outputs={"Out": out}, attrs={"mode": mode})
    return out


@_export
def maxout(x, groups, name=None):
    return simple_op("maxout", {"X": x}, {"groups": groups}, name=name)


@_export
def hinge_loss(input, label):
    return simple_op("hinge_loss", {"Logits": input, "Labels": label}, out_slot="Loss")


@_export
def huber_loss(input, label, delta):
    return simple_op("huber_loss", {"X": input, "Y": label}, {"delta": delta}, extra_outputs=("Residual",))[0]


@_export
def log_loss(input, label, epsilon=1e-4, name=None):
    return simple_op("log_loss", {"Predicted": input, "Labels": label}, {"epsilon": epsilon}, out_slot="Loss",
                     name=name)


@_export
def margin_rank_loss(label, left, right, margin=0.1, name=None):
    return simple_op("margin_rank_loss", {"Label": label, "X1": left, "X2": right}, {"margin": margin},
                     extra_outputs=("Activated",), name=name)[0]


@_export
def rank_loss(label, left, right, name=None):
    return simple_op("rank_loss", {"Label": label, "Left": left, "Right": right}, name=name)


@_export
def smooth_l1(x, y, inside_weight=None, outside_weight=None, sigma=None):
    inputs = {"X": x, "Y": y}
    if inside_weight is not None:
        inputs["InsideWeight"] = inside_weight
    if outside_weight is not None:
        inputs["OutsideWeight"] = outside_weight
    return simple_op("smooth_l1_loss", inputs, {"sigma": sigma if sigma is not None else 1.0},
                     extra_outputs=("Diff",))[0]


@_export
def cos_sim(X, Y):
    return simple_op("cos_sim", {"X": [X], "Y": [Y]}, extra_outputs=("XNorm", "YNorm"))[0]


@_export
def bilinear_tensor_product(x, y, size, act=None, name=None, param_attr=None, bias_attr=None):
    helper = LayerHelper("bilinear_tensor_product", **locals())
    dtype = helper.input_dtype("x")
    w = helper.create_parameter(attr=helper.param_attr, shape=[size, x.shape[1], y.shape[1]], dtype=dtype)
    inputs = {"X": x, "Y": y, "Weight": w}
    if helper.bias_attr:
        inputs["Bias"] = helper.create_parameter(attr=helper.bias_attr, shape=[1, size], dtype=dtype, is_bias=True)
    out = helper.create_variable_for_type_inference(dtype)
    helper.append_op(type="bilinear_tensor_product", inputs=inputs, outputs={"Out": out})
    return helper.append_activation(out)


@_export
def multiplex(inputs, index):
    return simple_op("multiplex", {"X": inputs, "Ids": index})


@_export
def im2sequence(input, filter_size=1, stride=1, padding=0, input_image_size=None, out_stride=1, name=None):
    pd = _pair(padding)
    if len(pd) == 2:
        pd = pd * 2
    return simple_op("im2sequence", {"X": input}, {"kernels": _pair(filter_size), "strides": _pair(stride),
                                                    "paddings": pd}, name=name)


@_export
def row_conv(input, future_context_size, param_attr=None, act=None):
    helper = LayerHelper("row_conv", **locals())
    w = helper.create_parameter(attr=helper.param_attr, shape=[future_context_size + 1, input.shape[1]],
                                dtype=input.dtype)
    out = helper.create_variable_for_type_inference(input.dtype)
    helper.append_op(type="row_conv", inputs={"X": [input], "Filter": [w]}, outputs={"Out": [out]})
    return helper.append_activation(out)


@_export
def conv_shift(x, y):
    return simple_op("conv_shift", {"X": x, "Y": y})


@_export
def roi_pool(input, rois, pooled_height=1, pooled_width=1, spatial_scale=1.0):
    return simple_op("roi_pool", {"X": input, "ROIs": rois},
                     {"pooled_height": pooled_height, "pooled_width": pooled_width, "spatial_scale": spatial_scale},
                     extra_outputs=("Argmax",))[0]


@_export
def mean_iou(input, label, num_classes):
    helper = LayerHelper("mean_iou", **locals())
    out = helper.create_variable_for_type_inference("float32")
    wrong = helper.create_variable_for_type_inference("int32")
    correct = helper.create_variable_for_type_inference("int32")
    helper.append_op(type="mean_iou", inputs={"Predictions": input, "Labels": label},
                     outputs={"OutMeanIou": out, "OutWrong": wrong, "OutCorrect": correct},
                     attrs={"num_classes": num_classes})
    return out, wrong, correct


@_export
def random_crop(x, shape, seed=None):
    helper = LayerHelper("random_crop", **locals())
    out = helper.create_variable_for_type_inference(x.dtype)
    seed_var = helper.create_global_variable(persistable=True, dtype="int64", shape=[1])
    helper.set_variable_initializer(seed_var, ConstantInitializer(float(seed or 0)))
    seed_out = helper.create_variable_for_type_inference("int64")
    helper.append_op(type="random_crop", inputs={"X": x, "Seed": seed_var},
                     outputs={"Out": out, "SeedOut": seed_out}, attrs={"shape": list(shape)})
    return out


@_export
def shuffle_channel(x, group, name=None):
    return simple_op("shuffle_channel", {"X": x}, {"group": group}, name=name)


@_export
def kldiv_loss(x, target, reduction="mean", name=None):
    return simple_op("kldiv_loss", {"X": x, "Target": target}, {"reduction": reduction}, out_slot="Loss", name=name)


@_export
def bpr_loss(input, label, name=None):
    return simple_op("bpr_loss", {"X": input, "Label": label}, out_slot="Y", name=name)


@_export
def autoincreased_step_counter(counter_name=None, begin=1, step=1):
    from .tensor import _global_step_counter

    return _global_step_counter(counter_name, begin, step)


# ---- activations that the reference exposes from nn.py with extra attrs


@_export
def relu(x, name=None):
    return simple_op("relu", {"X": x}, name=name)


@_export
def log(x, name=None):
    return simple_op("log", {"X": x}, name=name)


@_export
def pow(x, factor=1.0, name=None):
    return simple_op("pow", {"X": x}, {"factor": float(factor)}, name=name)


@_export
def sqrt(x, name=None):
    return simple_op("sqrt", {"X": x}, name=name)


@_export
def brelu(x, t_min=0.0, t_max=24.0, name=None):
    return simple_op("brelu", {"X": x}, {"t_min": t_min, "t_max": t_max}, name=name)


@_export
def leaky_relu(x, alpha=0.02, name=None):
    return simple_op("leaky_relu", {"X": x}, {"alpha": alpha}, name=name)


@_export
def soft_relu(x, threshold=40.0, name=None):
    return simple_op("soft_relu", {"X": x}, {"threshold": threshold}, name=name)


@_export
def elu(x, alpha=1.0, name=None):
    return simple_op("elu", {"X": x}, {"alpha": alpha}, name=name)


@_export
def relu6(x, threshold=6.0, name=None):
    return simple_op("relu6", {"X": x}, {"threshold": threshold}, name=name)


@_export
def stanh(x, scale_a=2.0 / 3.0, scale_b=1.7159, name=None):
    return simple_op("stanh", {"X": x}, {"scale_a": scale_a, "scale_b": scale_b}, name=name)


@_export
def hard_sigmoid(x, slope=0.2, offset=0.5, name=None):
    return simple_op("hard_sigmoid", {"X": x}, {"slope": slope, "offset": offset}, name=name)


@_export
def swish(x, beta=1.0, name=None):
    return simple_op("swish", {"X": x}, {"beta": beta}, name=name)


@_export
def gelu(x, name=None):
    return simple_op("gelu", {"X": x}, name=name)


@_export
def conv3d_transpose(input, num_filters, output_size=None, filter_size=None, padding=0, stride=1, dilation=1,
                     groups=None, param_attr=None, bias_attr=None, use_cudnn=True, act=None, name=None):
    """3-D transposed convolution (reference nn.py conv3d_transpose; NCDHW)."""
    helper = LayerHelper("conv3d_transpose", **locals())
    dtype = helper.input_dtype()
    groups = groups or 1
    padding, stride, dilation = _pair(padding, 3), _pair(stride, 3), _pair(dilation, 3)
    if filter_size is None:
        output_size = _pair(output_size, 3)
        filter_size = [(output_size[i] - (input.shape[2 + i] - 1) * stride[i] + 2 * padding[i] - 1) // dilation[i] + 1
                       for i in range(3)]
    filter_shape = [input.shape[1], num_filters // groups] + _pair(filter_size, 3)
    w = helper.create_parameter(dtype=dtype, shape=filter_shape, attr=helper.param_attr)
    pre_bias = helper.create_variable_for_type_inference(dtype)
    helper.append_op(type="conv3d_transpose", inputs={"Input": [input], "Filter": [w]},
                     outputs={"Output": pre_bias},
                     attrs={"output_size": _pair(output_size, 3) if output_size else [], "strides": stride,
                            "paddings": padding, "dilations": dilation, "groups": groups, "use_cudnn": use_cudnn})
    out = helper.append_bias_op(pre_bias, dim_start=1, dim_end=2)
    return helper.append_activation(out)


@_export
def dice_loss(input, label, epsilon=1e-05):
    """1 - 2|X∩Y| / (|X| + |Y|) averaged over the batch; ``label`` holds class ids
    (one-hot against input's last dim), ``input`` is a probability map."""
    onehot = one_hot(label, depth=input.shape[-1])
    dims = list(range(1, len(input.shape)))
    inse = reduce_sum(elementwise_mul(input, onehot), dim=dims)
    denom = elementwise_add(reduce_sum(input, dim=dims), reduce_sum(onehot, dim=dims))
    score = scale(elementwise_div(scale(inse, scale=2.0), scale(denom, bias=epsilon)), scale=-1.0, bias=1.0)
    return reduce_mean(score)


@_export
def uniform_random_batch_size_like(input, shape, dtype="float32", input_dim_idx=0, output_dim_idx=0, min=-1.0,
                                   max=1.0, seed=0):
    from ...framework import core as _core

    return simple_op("uniform_random_batch_size_like", {"Input": input},
                     {"shape": list(shape), "dtype": _core.convert_dtype(dtype), "input_dim_idx": input_dim_idx,
                      "output_dim_idx": output_dim_idx, "min": float(min), "max": float(max), "seed": seed},
                     dtype=dtype, stop_gradient=True)


@_export
def gaussian_random_batch_size_like(input, shape, input_dim_idx=0, output_dim_idx=0, mean=0.0, std=1.0, seed=0,
                                    dtype="float32"):
    from ...framework import core as _core

    return simple_op("gaussian_random_batch_size_like", {"Input": input},
                     {"shape": list(shape), "dtype": _core.convert_dtype(dtype), "input_dim_idx": input_dim_idx,
                      "output_dim_idx": output_dim_idx, "mean": float(mean), "std": float(std), "seed": seed},
                     dtype=dtype, stop_gradient=True)


@_export
def sampling_id(x, min=0.0, max=1.0, seed=0, dtype="float32"):
    """Sample one id per row of the probability matrix ``x``."""
    return simple_op("sampling_id", {"X": x}, {"min": float(min), "max": float(max), "seed": seed},
                     dtype="int64", stop_gradient=True)


@_export
def sum(x):
    """Elementwise sum of a list of tensors (the ``sum`` op)."""
    xs = x if isinstance(x, (list, tuple)) else [x]
    return simple_op("sum", {"X": list(xs)}, dtype=xs[0].dtype)
