"""v2 layers (reference v2/layer.py over trainer_config_helpers/layers.py) built as
Fluid ops in the v2 session's program.  Defaults follow the v2 helpers: ``fc`` and
``img_conv`` use Tanh / Relu when no activation is given, sequence ``pooling``
defaults to max pooling.  Each call returns the Fluid Variable of the layer
output (v2's LayerOutput role)."""
from __future__ import annotations

import math

from .. import fluid
from . import activation as A
from . import attr as _attr
from . import pooling as P
from ._core import STATE, guard


def _name(name, kind):
    return name


def data(name, type, **kw):
    with guard():
        if type.kind == "index":
            v = fluid.layers.data(name=name, shape=[1], dtype="int64", lod_level=type.seq_type)
        else:
            v = fluid.layers.data(name=name, shape=[type.dim], dtype="float32", lod_level=type.seq_type)
    STATE["data"][name] = type
    v.v2_size = type.dim
    return v


def _act(act, default):
    return A.act_name(act if act is not None else default)


def fc(input, size, act=None, name=None, param_attr=None, bias_attr=None, layer_attr=None, **kw):
    with guard():
        out = fluid.layers.fc(input=input, size=size, act=_act(act, A.Tanh), param_attr=_attr.to_fluid(param_attr),
                              bias_attr=_attr.to_fluid(bias_attr), name=name)
        if layer_attr is not None and getattr(layer_attr, "drop_rate", None):
            out = fluid.layers.dropout(out, layer_attr.drop_rate)
    out.v2_size = size
    return out


def embedding(input, size, param_attr=None, **kw):
    vocab = STATE["data"][input.name].dim
    with guard():
        out = fluid.layers.embedding(input=input, size=[vocab, size], param_attr=_attr.to_fluid(param_attr))
    out.v2_size = size
    return out


def _as_image(input, num_channels):
    if len(input.shape) == 4:
        return input
    hw2 = getattr(input, "v2_hw", None)
    size = getattr(input, "v2_size", None) or input.shape[-1]
    if hw2 is not None:  # data_layer(height=, width=): [C, H, W] with C = size / (H W)
        h, w = hw2
        return fluid.layers.reshape(input, [-1, max(int(size) // (h * w), 1), h, w])
    hw = int(round(math.sqrt(size // num_channels)))
    return fluid.layers.reshape(input, [-1, num_channels, hw, hw])


def img_conv(input, filter_size, num_filters, num_channels=None, stride=1, padding=0, act=None, groups=1,
             param_attr=None, bias_attr=None, name=None, **kw):
    with guard():
        x = _as_image(input, num_channels or 1)
        if kw.get("trans"):  # v1 trans=True: the transposed (fractionally strided) convolution, exconvt
            out = fluid.layers.conv2d_transpose(x, num_filters, filter_size=filter_size, stride=stride,
                                                padding=padding, dilation=kw.get("dilation", 1), groups=groups,
                                                act=_act(act, A.Relu), param_attr=_attr.to_fluid(param_attr),
                                                bias_attr=_attr.to_fluid(bias_attr), name=name)
        else:
            out = fluid.layers.conv2d(x, num_filters, filter_size, stride=stride, padding=padding,
                                      dilation=kw.get("dilation", 1), groups=groups, act=_act(act, A.Relu),
                                      param_attr=_attr.to_fluid(param_attr), bias_attr=_attr.to_fluid(bias_attr),
                                      name=name)
    return out


def img_pool(input, pool_size, stride=1, padding=0, pool_type=None, num_channels=None, name=None, **kw):
    with guard():
        x = _as_image(input, num_channels or 1)
        # v1 / v2 image pooling rounds the output size up (ceil mode, reference PoolLayer)
        out = fluid.layers.pool2d(x, pool_size, (pool_type or P.Max()).img, stride, pool_padding=padding,
                                  ceil_mode=kw.get("ceil_mode", True))
    return out


def batch_norm(input, act=None, **kw):
    with guard():
        return fluid.layers.batch_norm(input, act=_act(act, A.Relu))


def dropout(input, dropout_rate, **kw):
    with guard():
        return fluid.layers.dropout(input, dropout_rate)


def concat(input, **kw):
    with guard():
        out = fluid.layers.concat(list(input), axis=1)
    return out


def pooling(input, pooling_type=None, **kw):
    with guard():
        return fluid.layers.sequence_pool(input, (pooling_type or P.Max()).seq)


def last_seq(input, **kw):
    with guard():
        return fluid.layers.sequence_last_step(input)


def first_seq(input, **kw):
    with guard():
        return fluid.layers.sequence_first_step(input)


def max_id(input, **kw):
    with guard():
        return fluid.layers.argmax(input, axis=1)


def _cost(c):
    with guard():
        return fluid.layers.mean(c)


def classification_cost(input, label, name=None, evaluator=None, **kw):
    """Cross entropy on a softmax output + the v2 default classification-error
    evaluator (reported as ``classification_error_evaluator``)."""
    from . import evaluator as E

    with guard():
        cost = fluid.layers.mean(_weighted(fluid.layers.cross_entropy(input=input, label=label), kw.get("weight")))
    E.classification_error(input, label)
    return cost


def _weighted(cost, weight):
    """Per-sample cost times the sample weight layer ([N, 1]) of a weighted v1 cost."""
    return cost if weight is None else fluid.layers.elementwise_mul(cost, weight)


def cross_entropy_cost(input, label, **kw):
    with guard():
        return fluid.layers.mean(_weighted(fluid.layers.cross_entropy(input=input, label=label), kw.get("weight")))


def square_error_cost(input, label, **kw):
    with guard():
        # per-sample sum of squares (reference SumOfSquaresCostLayer), batch mean
        c = _weighted(fluid.layers.reduce_sum(fluid.layers.square_error_cost(input=input, label=label), dim=1,
                                              keep_dim=True), kw.get("weight"))
        return fluid.layers.mean(c)


mse_cost = regression_cost = square_error_cost
