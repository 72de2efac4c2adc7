"""Composite v1 networks (reference python/paddle/trainer_config_helpers/networks.py
``__all__``): recurrent units and groups, bidirectional RNNs, attention, image
conv groups -- each one a composition of the v1 layers of this package (which build
Fluid ops on the MI355X kernels), with the reference's default names
(``__lstm_0__``, ``__gru_group_0__``, ...)."""
from __future__ import annotations

from . import layers_v1 as _v1
from ..v2 import activation as _act
from ..v2 import pooling as _pool

__all__ = []

_COUNT = {}


def _export(fn):
    __all__.append(fn.__name__)
    return fn


def _default_name(prefix, name):
    """wrap_name_default: ``__{prefix}_{i}__`` with a per-prefix counter."""
    if name:
        return name
    from . import config_proto as cp

    rec = cp.current()
    counts = rec.count if rec is not None else _COUNT
    i = counts.get(prefix, 0)
    counts[prefix] = i + 1
    return f"__{prefix}_{i}__"


def _tch():
    from .. import trainer_config_helpers as t

    return t


def _in(x):
    from .config_proto import unwrap

    return unwrap(x)


# ------------------------------------------------------------------ LSTM
@_export
def lstmemory_unit(input, out_memory=None, name=None, size=None, param_attr=None, act=None, gate_act=None,
                   state_act=None, input_proj_bias_attr=None, input_proj_layer_attr=None, lstm_bias_attr=None,
                   lstm_layer_attr=None):
    """One LSTM step inside a recurrent_group: ``input`` is the projected input
    (4 * size wide); h_{t-1} enters through a full-matrix projection."""
    input = _in(input)
    t = _tch()
    name = _default_name("lstm_unit", name)
    size = size or _v1._size(input) // 4
    out_mem = out_memory if out_memory is not None else _tch().memory(name=name, size=size)
    state_mem = _tch().memory(name=f"{name}_state", size=size)
    with t.mixed_layer(name=f"{name}_input_recurrent", size=size * 4, bias_attr=input_proj_bias_attr,
                       act=_act.Identity()) as m:
        m += t.identity_projection(input=input)
        m += t.full_matrix_projection(input=out_mem, param_attr=param_attr)
    lstm_out = _tch().lstm_step_layer(name=name, input=m.m.out, state=state_mem, size=size, bias_attr=lstm_bias_attr,
                                   act=act, gate_act=gate_act, state_act=state_act)
    _tch().get_output_layer(name=f"{name}_state", input=lstm_out, arg_name="state")
    return lstm_out


@_export
def lstmemory_group(input, size=None, name=None, out_memory=None, reverse=False, param_attr=None, act=None,
                    gate_act=None, state_act=None, input_proj_bias_attr=None, input_proj_layer_attr=None,
                    lstm_bias_attr=None, lstm_layer_attr=None):
    """lstmemory written as a recurrent_group of :func:`lstmemory_unit` steps."""
    input = _in(input)
    name = _default_name("lstm_group", name)

    def step(ipt):
        return lstmemory_unit(input=ipt, name=name, size=size, act=act, gate_act=gate_act, state_act=state_act,
                              out_memory=out_memory, input_proj_bias_attr=input_proj_bias_attr,
                              param_attr=param_attr, lstm_bias_attr=lstm_bias_attr)

    return _tch().recurrent_group(name=f"{name}_recurrent_group", step=step, reverse=reverse, input=input)


@_export
def simple_lstm(input, size, name=None, reverse=False, mat_param_attr=None, bias_param_attr=None,
                inner_param_attr=None, act=None, gate_act=None, state_act=None, mixed_layer_attr=None,
                lstm_cell_attr=None):
    """full-matrix projection to 4 * size, then lstmemory."""
    input = _in(input)
    t = _tch()
    name = _default_name("lstm", name)
    with t.mixed_layer(name=f"{name}_transform", size=size * 4, act=_act.Identity(), bias_attr=False) as m:
        m += t.full_matrix_projection(input=input, param_attr=mat_param_attr)
    return t.lstmemory(name=name, input=m.m.out, reverse=reverse, bias_attr=bias_param_attr,
                       param_attr=inner_param_attr, act=act, gate_act=gate_act, state_act=state_act)


# ------------------------------------------------------------------ GRU
@_export
def gru_unit(input, memory_boot=None, size=None, name=None, gru_bias_attr=None, gru_param_attr=None, act=None,
             gate_act=None, gru_layer_attr=None, naive=False):
    """One GRU step inside a recurrent_group (``input``: 3 * size projected gates)."""
    input = _in(input)
    name = _default_name("gru_unit", name)
    size = size or _v1._size(input) // 3
    out_mem = _tch().memory(name=name, size=size, boot_layer=memory_boot)
    step = _tch().gru_step_naive_layer if naive else _tch().gru_step_layer
    return step(name=name, input=input, output_mem=out_mem, size=size, bias_attr=gru_bias_attr,
                param_attr=gru_param_attr, act=act, gate_act=gate_act)


@_export
def gru_group(input, memory_boot=None, size=None, name=None, reverse=False, gru_bias_attr=None,
              gru_param_attr=None, act=None, gate_act=None, gru_layer_attr=None, naive=False):
    """grumemory written as a recurrent_group of :func:`gru_unit` steps."""
    input = _in(input)
    name = _default_name("gru_group", name)

    def step(ipt):
        return gru_unit(input=ipt, memory_boot=memory_boot, name=name, size=size, gru_bias_attr=gru_bias_attr,
                        gru_param_attr=gru_param_attr, act=act, gate_act=gate_act, naive=naive)

    return _tch().recurrent_group(name=f"{name}_recurrent_group", step=step, reverse=reverse, input=input)


@_export
def simple_gru(input, size, name=None, reverse=False, mixed_param_attr=None, mixed_bias_param_attr=None,
               mixed_layer_attr=None, gru_bias_attr=None, gru_param_attr=None, act=None, gate_act=None,
               gru_layer_attr=None, naive=False):
    """full-matrix projection to 3 * size, then :func:`gru_group`."""
    input = _in(input)
    t = _tch()
    name = _default_name("simple_gru", name)
    with t.mixed_layer(name=f"{name}_transform", size=size * 3, bias_attr=mixed_bias_param_attr) as m:
        m += t.full_matrix_projection(input=input, param_attr=mixed_param_attr)
    return gru_group(name=name, size=size, input=m.m.out, reverse=reverse, gru_bias_attr=gru_bias_attr,
                     gru_param_attr=gru_param_attr, act=act, gate_act=gate_act, naive=naive)


@_export
def simple_gru2(input, size, name=None, reverse=False, mixed_param_attr=None, mixed_bias_attr=None,
                gru_param_attr=None, gru_bias_attr=None, act=None, gate_act=None, mixed_layer_attr=None,
                gru_cell_attr=None):
    """full-matrix projection to 3 * size, then the fused grumemory layer."""
    input = _in(input)
    t = _tch()
    name = _default_name("simple_gru2", name)
    with t.mixed_layer(name=f"{name}_transform", size=size * 3, bias_attr=mixed_bias_attr) as m:
        m += t.full_matrix_projection(input=input, param_attr=mixed_param_attr)
    return t.grumemory(name=name, input=m.m.out, reverse=reverse, bias_attr=gru_bias_attr,
                       param_attr=gru_param_attr, act=act, gate_act=gate_act)


def _bidirectional(kind, input, size, name, return_seq, fwd_kw, bwd_kw, concat_act):
    t = _tch()
    unit = simple_gru2 if kind == "gru" else simple_lstm
    fw = unit(name=f"{name}_fw", input=input, size=size, **fwd_kw)
    bw = unit(name=f"{name}_bw", input=input, size=size, reverse=True, **bwd_kw)
    if return_seq:
        return t.concat_layer(name=name, input=[fw, bw], act=concat_act)
    return t.concat_layer(name=name, input=[t.last_seq(input=fw), t.first_seq(input=bw)], act=concat_act)


def _split_dir(kw):
    fwd = {k[4:]: v for k, v in kw.items() if k.startswith("fwd_")}
    bwd = {k[4:]: v for k, v in kw.items() if k.startswith("bwd_")}
    return fwd, bwd


@_export
def bidirectional_gru(input, size, name=None, return_seq=False, concat_act=None, **kw):
    """Forward and backward :func:`simple_gru2`, their sequences (``return_seq``) or
    last / first steps concatenated."""
    name = _default_name("bidirectional_gru", name)
    fwd, bwd = _split_dir(kw)
    return _bidirectional("gru", input, size, name, return_seq, fwd, bwd, concat_act)


@_export
def bidirectional_lstm(input, size, name=None, return_seq=False, concat_act=None, **kw):
    """Forward and backward :func:`simple_lstm` (see :func:`bidirectional_gru`)."""
    name = _default_name("bidirectional_lstm", name)
    fwd, bwd = _split_dir(kw)
    return _bidirectional("lstm", input, size, name, return_seq, fwd, bwd, concat_act)


# ------------------------------------------------------------------ attention
@_export
def simple_attention(encoded_sequence, encoded_proj, decoder_state, transform_param_attr=None,
                     softmax_param_attr=None, weight_act=None, name=None):
    """Bahdanau attention: score = v^T tanh(enc_proj + W s), softmax over the
    sequence, context = sum_t a_t enc_t."""
    t = _tch()
    name = _default_name("attention", name)
    proj_size = _v1._size(encoded_proj)
    with t.mixed_layer(size=proj_size, name=f"{name}_transform") as m:
        m += t.full_matrix_projection(input=decoder_state, param_attr=transform_param_attr)
    expanded = t.expand_layer(input=m.m.out, expand_as=encoded_sequence, name=f"{name}_expand")
    with t.mixed_layer(size=proj_size, act=weight_act or _act.Tanh(), name=f"{name}_combine") as mc:
        mc += t.identity_projection(input=expanded)
        mc += t.identity_projection(input=encoded_proj)
    attention_weight = t.fc_layer(input=mc.m.out, size=1, act=_act.SequenceSoftmax(),
                                  param_attr=softmax_param_attr, name=f"{name}_softmax", bias_attr=False)
    scaled = t.scaling_layer(weight=attention_weight, input=encoded_sequence, name=f"{name}_scaling")
    return t.pooling_layer(input=scaled, pooling_type=_pool.Sum(), name=f"{name}_pooling")


# ------------------------------------------------------------------ image groups
@_export
def img_conv_group(input, conv_num_filter, pool_size, num_channels=None, conv_padding=1, conv_filter_size=3,
                   conv_act=None, conv_with_batchnorm=False, conv_batchnorm_drop_rate=0, pool_stride=1,
                   pool_type=None, param_attr=None):
    """A stack of 3x3 convolutions (optionally + batch norm + dropout) and one pool."""
    t = _tch()
    n = len(conv_num_filter)

    def per(v):
        return list(v) if isinstance(v, (list, tuple)) else [v] * n

    pads, fsz, acts = per(conv_padding), per(conv_filter_size), per(conv_act)
    bns, drops = per(conv_with_batchnorm), per(conv_batchnorm_drop_rate)
    tmp = input
    for i in range(n):
        extra = {"num_channels": num_channels} if i == 0 else {}
        tmp = t.img_conv_layer(input=tmp, padding=pads[i], filter_size=fsz[i], num_filters=conv_num_filter[i],
                               act=_act.Linear() if bns[i] else acts[i], param_attr=param_attr, **extra)
        if bns[i]:
            tmp = t.batch_norm_layer(input=tmp, act=acts[i])
            if drops[i]:
                tmp = t.dropout_layer(input=tmp, dropout_rate=drops[i])
    return t.img_pool_layer(input=tmp, stride=pool_stride, pool_size=pool_size, pool_type=pool_type)


@_export
def vgg_16_network(input_image, num_channels, num_classes=1000):
    """VGG-16: five conv groups, two 4096-wide fc + dropout, a softmax classifier."""
    t = _tch()
    tmp = input_image
    for i, (nf, k) in enumerate(((64, 2), (128, 2), (256, 3), (512, 3), (512, 3))):
        tmp = img_conv_group(input=tmp, num_channels=num_channels if i == 0 else None, conv_padding=1,
                             conv_num_filter=[nf] * k, conv_filter_size=3, conv_act=_act.Relu(), pool_stride=2,
                             pool_size=2, pool_type=_pool.Max())
    for _ in range(2):
        tmp = t.fc_layer(input=tmp, size=4096, act=_act.Relu(), layer_attr=t.ExtraAttr(drop_rate=0.5))
    return t.fc_layer(input=tmp, size=num_classes, act=_act.Softmax())


@_export
def dropout_layer(input, dropout_rate, name=None):
    """addto of one input with layer dropout (the reference's dropout_layer)."""
    t = _tch()
    return t.addto_layer(name=name, input=input, act=_act.Linear(), bias_attr=False,
                         layer_attr=t.ExtraAttr(drop_rate=dropout_rate))
