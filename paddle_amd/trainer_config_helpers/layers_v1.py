"""The rest of the v1 layer DSL (reference python/paddle/trainer_config_helpers/
layers.py ``__all__``): mixed layers and projections, recurrent groups with
memories, sequence / image / cost / detection layers.

Every function builds Fluid ops in the v1 session's program (``v2._core.guard``)
and returns the Fluid Variable of its output (the LayerOutput role), with
``v2_size`` set to the feature width where it is known.  The legacy engine's
C++ layers (paddle/legacy/gserver/layers) are not reproduced: each v1 layer is
expressed with the Fluid operators that compute the same function on the MI355X
kernels (e.g. ``lstmemory`` -> ``dynamic_lstm`` (persistent LSTM kernel),
``crf_layer`` -> ``linear_chain_crf``, ``ctc_layer`` -> ``warpctc``).
"""
from __future__ import annotations

import contextlib

from .. import fluid
from ..fluid.layer_helper import LayerHelper
from ..v2 import activation as _act
from ..v2._core import guard

__all__ = []


def _export(fn):
    __all__.append(fn.__name__)
    return fn


def _L():
    return fluid.layers


def _seq_reverse(x):
    return _op("sequence_reverse", {"X": [x]}, {"Y": x.dtype if isinstance(x.dtype, str) else "float32"})["Y"]


def _size(v, default=None):
    s = getattr(v, "v2_size", None)
    if s is None and v is not None and getattr(v, "shape", None):
        s = v.shape[-1] if v.shape[-1] and v.shape[-1] > 0 else default
    return s if s is not None else default


def _sized(v, size):
    v.v2_size = size
    return v


def _apply_act(x, act):
    a = _act.act_name(act) if act is not None else None
    if not a or a in ("linear", "identity"):
        return x
    return getattr(_L(), a)(x)


def _op(op_type, inputs, outputs_spec, attrs=None, dtype="float32"):
    """Append one Fluid op with fresh output variables; returns them (dict)."""
    helper = LayerHelper(op_type)
    outs = {k: [helper.create_variable_for_type_inference(dtype=dt)] for k, dt in outputs_spec.items()}
    helper.append_op(type=op_type, inputs=inputs, outputs=outs, attrs=attrs or {})
    return {k: v[0] for k, v in outs.items()}


# ------------------------------------------------------------------ constants / markers
@_export
class LayerType:
    """Layer type names of the v1 ModelConfig (informational)."""
    DATA = "data"
    FC_LAYER = "fc"
    MIXED_LAYER = "mixed"
    LSTMEMORY = "lstmemory"
    GRUMEMORY = "gated_recurrent"
    RECURRENT_LAYER = "recurrent"
    COST = "cost"
    CRF_LAYER = "crf"
    CTC_LAYER = "ctc"
    CONV_LAYER = "conv"
    POOL_LAYER = "pool"
    BATCH_NORM_LAYER = "batch_norm"


@_export
class AggregateLevel:
    TO_NO_SEQUENCE = "non-seq"
    TO_SEQUENCE = "seq"
    EACH_TIMESTEP = TO_NO_SEQUENCE
    EACH_SEQUENCE = TO_SEQUENCE


@_export
class ExpandLevel:
    FROM_NO_SEQUENCE = AggregateLevel.TO_NO_SEQUENCE
    FROM_SEQUENCE = AggregateLevel.TO_SEQUENCE
    FROM_TIMESTEP = FROM_NO_SEQUENCE


LayerOutput = fluid.framework.Variable
__all__.append("LayerOutput")


@_export
def layer_support(*attrs):
    """Decorator of the v1 helpers declaring which extra attributes a layer takes."""
    def deco(fn):
        return fn
    return deco


# ------------------------------------------------------------------ projections / mixed
class _Projection:
    """A deferred term of a mixed layer: ``build(size)`` emits its ops."""

    def __init__(self, fn, size=None, input=None, kind=None):
        self.fn, self.size = fn, size
        self.input, self.v1_type = input, kind  # for the ModelConfig record (config_proto.py)

    def build(self, size):
        return self.fn(size if self.size is None else self.size)


def _fluid_attr(a):
    """A v1 ParameterAttribute as a fluid ParamAttr (a named one is shared by name)."""
    if a is None or a is True:
        return None
    if a is False:
        return False
    if isinstance(a, fluid.ParamAttr):
        return a
    init = None
    if getattr(a, "initial_std", None) is not None:
        init = fluid.initializer.Normal(loc=getattr(a, "initial_mean", None) or 0.0, scale=a.initial_std)
    return fluid.ParamAttr(name=getattr(a, "name", None), initializer=init)


@_export
def full_matrix_projection(input, size=0, param_attr=None):
    pr = _Projection(lambda s: _L().fc(input=input, size=s, bias_attr=False, param_attr=_fluid_attr(param_attr)),
                     size or None, input, "fc")
    pr.v1_param_attr = param_attr  # a named weight is recorded (and shared) under its own name
    return pr


@_export
def trans_full_matrix_projection(input, size=0, param_attr=None):
    # y = x W^T with W [size, in]: a parameter of the transposed shape, one matmul
    def build(s):
        helper = LayerHelper("trans_fc")
        w = helper.create_parameter(attr=helper.param_attr, shape=[s, _size(input)], dtype="float32")
        return _L().matmul(input, w, transpose_y=True)
    return _Projection(build, size or None, input, "trans_fc")


@_export
def table_projection(input, size=0, param_attr=None):
    from ..v2._core import STATE

    # the id layer's vocabulary: a data layer's dim, else the layer's width
    vocab = STATE["data"][input.name].dim if input.name in STATE["data"] else _size(input)
    return _Projection(lambda s: _L().embedding(input=input, size=[vocab, s]), size or None, input, "table")


@_export
def identity_projection(input, offset=None, size=None):
    if offset is None:
        return _Projection(lambda s: input, _size(input), input, "identity")
    return _Projection(lambda s: _L().slice(input, axes=[1], starts=[offset], ends=[offset + s]), size, input,
                       "identity_offset")


@_export
def slice_projection(input, slices):
    def build(s):
        parts = [_L().slice(input, axes=[1], starts=[a], ends=[b]) for a, b in slices]
        return parts[0] if len(parts) == 1 else _L().concat(parts, axis=1)
    return _Projection(build, sum(b - a for a, b in slices), input, "slice")


@_export
def dotmul_projection(input, param_attr=None):
    def build(s):
        helper = LayerHelper("dotmul")
        w = helper.create_parameter(attr=helper.param_attr, shape=[_size(input)], dtype="float32")
        w._v1_weight = True  # a [1, size] weight in the v1 record, not a bias
        return _L().elementwise_mul(input, w, axis=1)
    return _Projection(build, _size(input), input, "dot_mul")


@_export
def scaling_projection(input, param_attr=None):
    def build(s):
        helper = LayerHelper("scaling")
        w = helper.create_parameter(attr=helper.param_attr, shape=[1], dtype="float32")
        w._v1_weight = True
        return _L().elementwise_mul(input, w)
    return _Projection(build, _size(input), input, "scaling")


@_export
def dotmul_operator(a=None, b=None, scale=1, **kw):
    a = kw.get("x", a)
    b = kw.get("y", b)
    op = _Projection(lambda s: _L().scale(_L().elementwise_mul(a, b), scale=float(scale)), _size(a))
    op.v1_operands = [a, b]  # an operator reads two layers (config_proto.py records both inputs)
    op.v1_operator = ("dot_mul", float(scale))
    return op


@_export
def context_projection(input, context_len, context_start=None, padding_attr=False):
    """Concatenation of the rows [t + start, t + start + len) of each sequence (zero
    outside the sequence): the im2col of a 1-D sequence convolution."""
    start = -((context_len - 1) // 2) if context_start is None else context_start

    def build(s):
        d = _size(input)
        helper = LayerHelper("context_projection")
        # a sequence_conv with an identity filter is exactly the context window
        import numpy as np

        eye = np.eye(context_len * d, dtype="float32")
        w = helper.create_parameter(
            attr=fluid.ParamAttr(initializer=fluid.initializer.NumpyArrayInitializer(eye), trainable=False),
            shape=[context_len * d, context_len * d], dtype="float32")
        out = helper.create_variable_for_type_inference("float32")
        helper.append_op(type="sequence_conv", inputs={"X": [input], "Filter": [w]}, outputs={"Out": [out]},
                         attrs={"contextStride": 1, "contextStart": start, "contextLength": context_len})
        return out
    pr = _Projection(build, context_len * _size(input), input, "context")
    pr.v1_context = (start, context_len)
    return pr


@_export
def conv_projection(input, filter_size, num_filters, num_channels=None, stride=1, padding=0, groups=1,
                    param_attr=None, trans=False, **kw):
    """A convolution (trans: transposed convolution) of an image layer as a mixed-layer
    term, flattened to [N, C * H * W]."""
    from ..v2.layer import _as_image

    def build(s):
        x = _as_image(input, num_channels or 1)
        if trans:
            out = _L().conv2d_transpose(x, num_filters=num_filters, filter_size=filter_size, stride=stride,
                                        padding=padding, groups=groups, bias_attr=False)
        else:
            out = _L().conv2d(x, num_filters=num_filters, filter_size=filter_size, stride=stride, padding=padding,
                              groups=groups, bias_attr=False)
        n = _conv_flat(input, num_channels or 1, filter_size, stride, padding, num_filters, trans)
        return _sized(_L().reshape(out, [-1, n]), n)
    pr = _Projection(build, None, input, "convt" if trans else "conv")
    pr.v1_conv = dict(filter_size=filter_size, num_filters=num_filters, channels=num_channels or 1, stride=stride,
                      padding=padding, groups=groups, trans=trans)
    return pr


conv_operator = conv_projection
__all__.append("conv_operator")


class _Mixed:
    def __init__(self, size, act, bias_attr, name):
        self.size, self.act, self.bias_attr, self.name = size, act, bias_attr, name
        self.terms = []
        self.out = None

    def __iadd__(self, proj):
        self.terms.append(proj)
        return self

    def finish(self):
        with guard():
            outs = [p.build(self.size) if isinstance(p, _Projection) else p for p in self.terms]
            size = self.size or _size(outs[0])
            s = outs[0] if len(outs) == 1 else _L().sums(outs)
            if self.bias_attr is not False and self.bias_attr is not None:
                helper = LayerHelper("mixed")
                b = helper.create_parameter(attr=helper.bias_attr, shape=[size], dtype="float32", is_bias=True)
                s = _L().elementwise_add(s, b, axis=1)
            self.out = _sized(_apply_act(s, self.act), size)
        return self.out


@_export
def mixed_layer(size=0, input=None, name=None, act=None, bias_attr=False, layer_attr=None):
    """Sum of projections / operators (+ bias, + activation).  Also usable as
    ``with mixed_layer(size=n) as m: m += full_matrix_projection(x)``."""
    m = _Mixed(size or None, act, bias_attr, name)
    if input is not None:
        for p in (input if isinstance(input, (list, tuple)) else [input]):
            m += p
        return m.finish()
    return _MixedCtx(m)


class _MixedCtx(contextlib.AbstractContextManager):
    def __init__(self, m):
        self.m = m

    def __iadd__(self, proj):
        self.m += proj
        return self

    def __exit__(self, *exc):
        if exc[0] is None:
            self.m.finish()
            hook = getattr(self.m, "on_finish", None)
            if hook is not None:
                hook(self.m)
        return False

    def __getattr__(self, k):  # the finished layer's Variable attributes
        return getattr(self.m.out, k)


# ------------------------------------------------------------------ recurrent layers
@_export
def lstmemory(input, name=None, size=None, reverse=False, act=None, gate_act=None, state_act=None, bias_attr=None,
              param_attr=None, **kw):
    """input: the projected gates [T, 4H] (v1 convention); returns the hidden sequence."""
    size = size or _size(input) // 4
    with guard():
        h, _ = _L().dynamic_lstm(input=input, size=4 * size, is_reverse=reverse,
                                 gate_activation=_act.act_name(gate_act) or "sigmoid",
                                 cell_activation=_act.act_name(state_act) or "tanh",
                                 candidate_activation=_act.act_name(act) or "tanh", use_peepholes=False)
    return _sized(h, size)


@_export
def grumemory(input, name=None, size=None, reverse=False, act=None, gate_act=None, bias_attr=None, param_attr=None,
              **kw):
    """input: the projected gates [T, 3H]; returns the hidden sequence."""
    size = size or _size(input) // 3
    with guard():
        h = _L().dynamic_gru(input=input, size=size, is_reverse=reverse,
                             gate_activation=_act.act_name(gate_act) or "sigmoid",
                             candidate_activation=_act.act_name(act) or "tanh")
    return _sized(h, size)


@_export
def recurrent_layer(input, act=None, bias_attr=None, param_attr=None, name=None, reverse=False, **kw):
    """h_t = act(x_t + W h_{t-1} (+ b)) over each sequence."""
    size = _size(input)
    with guard():
        rnn = _L().DynamicRNN()
        src = _seq_reverse(input) if reverse else input
        with rnn.block():
            x = rnn.step_input(src)
            prev = rnn.memory(shape=[size], value=0.0)
            h = _apply_act(_L().elementwise_add(x, _L().fc(prev, size=size, bias_attr=bias_attr)),
                           act or _act.Tanh())
            rnn.update_memory(prev, h)
            rnn.output(h)
        out = rnn()
        if reverse:
            out = _seq_reverse(out)
    return _sized(out, size)


# recurrent_group: the step function runs once inside a DynamicRNN block; memory()
# placeholders are bound, after the step returns, to the layer of the same name
_RG = []


@_export
class StaticInput:
    """A non-sequence (or whole-sequence) input read unchanged at every step."""

    def __init__(self, input, is_seq=False, size=None):
        self.input, self.is_seq, self.size = input, is_seq, size


@_export
class SubsequenceInput:
    def __init__(self, input):
        self.input = input


@_export
class BaseGeneratedInput:
    pass


@_export
class GeneratedInput(BaseGeneratedInput):
    """The generated-token input of a generation group (beam_search)."""

    def __init__(self, size, embedding_name, embedding_size):
        self.size, self.embedding_name, self.embedding_size = size, embedding_name, embedding_size


@_export
class BeamInput:
    def __init__(self, candidate_scores, selected_candidates, gold):
        self.candidate_scores, self.selected_candidates, self.gold = candidate_scores, selected_candidates, gold


_NAMED = []  # stack of {name: Variable} of the layers built inside recurrent groups


def _named(v, name):
    if name and _NAMED:
        _NAMED[-1][name] = v
    return v


@_export
def memory(name, size, is_seq=False, boot_layer=None, boot_bias=None, boot_bias_active_type=None,
           boot_with_const_id=None, **kw):
    """The previous step's output of the layer ``name`` of this recurrent group
    (``boot_layer`` at the first step, else zeros)."""
    if not _RG:
        raise RuntimeError("memory() is only valid inside a recurrent_group step function")
    rnn, mems = _RG[-1]
    m = rnn.memory(init=boot_layer) if boot_layer is not None else rnn.memory(shape=[size], value=0.0)
    if name is None:
        # an anonymous memory is bound later: ``m.set_input(layer)`` (LayerOutput.set_input)
        name = f"@memory_{len(mems)}@"
        named = _NAMED[-1]
        m.set_input = lambda layer, _k=name, _d=named: _d.__setitem__(_k, layer)
    mems.append((name, m))
    return _sized(m, size)


@_export
def recurrent_group(step, input, reverse=False, name=None, targetInlink=None, is_generating=False):
    """Run ``step`` over every time step of the sequence inputs (StaticInput: the same
    value each step); returns the step outputs as sequences."""
    from .config_proto import unwrap

    input = unwrap(input)
    ins = input if isinstance(input, (list, tuple)) else [input]
    with guard():
        rnn = _L().DynamicRNN()
        mems = []
        _RG.append((rnn, mems))
        _NAMED.append({})
        try:
            with rnn.block():
                args = []
                for x in ins:
                    if isinstance(x, StaticInput):
                        args.append(rnn.static_input(x.input))
                    elif isinstance(x, SubsequenceInput):
                        args.append(rnn.step_input(x.input))
                    else:
                        src = _seq_reverse(x) if reverse else x
                        args.append(_sized(rnn.step_input(src), _size(x)))
                outs = step(*args)
                named = _NAMED[-1]
                for nm, m in mems:
                    if nm not in named:
                        raise ValueError(f"recurrent_group: memory '{nm}' names no layer of the step")
                    rnn.update_memory(m, named[nm])
                outs_l = outs if isinstance(outs, (list, tuple)) else [outs]
                for o in outs_l:
                    rnn.output(o)
            res = rnn()
        finally:
            _RG.pop()
            _NAMED.pop()
        res_l = res if isinstance(res, (list, tuple)) else [res]
        if reverse:
            res_l = [_seq_reverse(r) for r in res_l]
        for r, o in zip(res_l, outs_l):
            _sized(r, _size(o))
    return res_l[0] if len(res_l) == 1 else res_l


@_export
def lstm_step_layer(input, state, size=None, act=None, name=None, gate_act=None, state_act=None, bias_attr=None,
                    **kw):
    """One LSTM step: input = projected gates [N, 4H] (already including W_h h_{t-1}),
    state = c_{t-1}; returns h_t (the new cell is published as ``name + "_state"``)."""
    size = size or _size(state)
    with guard():
        i, f, c_hat, o = _L().split(input, 4, dim=1)
        ga = _act.act_name(gate_act) or "sigmoid"
        i, f, o = (getattr(_L(), ga)(t) for t in (i, f, o))
        c_hat = getattr(_L(), _act.act_name(act) or "tanh")(c_hat)
        c = _L().elementwise_add(_L().elementwise_mul(f, state), _L().elementwise_mul(i, c_hat))
        h = _L().elementwise_mul(o, getattr(_L(), _act.act_name(state_act) or "tanh")(c))
    _named(_sized(c, size), (name + "_state") if name else None)
    return _named(_sized(h, size), name)


@_export
def gru_step_layer(input, output_mem, size=None, act=None, name=None, gate_act=None, bias_attr=None,
                   param_attr=None, **kw):
    """One GRU step: input = projected gates [N, 3H], output_mem = h_{t-1}."""
    size = size or _size(output_mem)
    blk = fluid.default_main_program().global_block()
    before = {p.name for p in blk.all_parameters()}
    with guard():
        h, _, _ = _L().gru_unit(input=input, hidden=output_mem, size=3 * size,
                                activation=_act.act_name(act) or "tanh",
                                gate_activation=_act.act_name(gate_act) or "sigmoid",
                                param_attr=_fluid_attr(param_attr), bias_attr=_fluid_attr(bias_attr))
    for p in blk.all_parameters():  # the [1, 3 size] gate bias is a bias, not a second weight
        if p.name not in before and len(p.shape) == 2 and p.shape[0] == 1:
            p._v1_bias = True
    return _named(_sized(h, size), name)


gru_step_naive_layer = gru_step_layer
__all__.append("gru_step_naive_layer")


@_export
def get_output_layer(input, arg_name, name=None, **kw):
    """A named secondary output of a layer (lstm_step_layer's 'state')."""
    if arg_name == "state" and _NAMED:
        for k, v in _NAMED[-1].items():
            if k.endswith("_state"):
                return _named(v, name)
    return _named(input, name)


@_export
def beam_search(step, input, bos_id, eos_id, beam_size, max_length=500, name=None, num_results_per_sample=None):
    """Generation with a recurrent step function over the generated tokens: the
    GeneratedInput's embedding of the previous token feeds ``step``; the step's
    output probabilities drive fluid's beam_search op each step (contrib
    BeamSearchDecoder semantics).  Returns the generated id sequences."""
    from ..fluid.contrib.decoder import beam_search_decoder as _bsd  # noqa: F401  (import check)

    ins = input if isinstance(input, (list, tuple)) else [input]
    gen = [x for x in ins if isinstance(x, BaseGeneratedInput)]
    if len(gen) != 1:
        raise ValueError("beam_search needs exactly one GeneratedInput")
    g = gen[0]
    statics = [x for x in ins if isinstance(x, StaticInput)]
    with guard():
        L = _L()
        init = statics[0].input if statics else None
        batch_ref = init if init is not None else None
        if batch_ref is None:
            raise ValueError("beam_search needs a StaticInput (e.g. the encoder state) to size the batch")
        ids0 = L.fill_constant_batch_size_like(batch_ref, shape=[-1, 1], dtype="int64", value=bos_id)
        scores0 = L.fill_constant_batch_size_like(batch_ref, shape=[-1, 1], dtype="float32", value=0.0)
        counter = L.zeros(shape=[1], dtype="int64")
        limit = L.fill_constant(shape=[1], dtype="int64", value=max_length)
        ids_arr = L.create_array("int64")
        scores_arr = L.create_array("float32")
        L.array_write(ids0, counter, ids_arr)
        L.array_write(scores0, counter, scores_arr)
        cond = L.less_than(counter, limit)
        w = L.While(cond)
        with w.block():
            pre_ids = L.array_read(ids_arr, counter)
            pre_scores = L.array_read(scores_arr, counter)
            emb = L.embedding(pre_ids, size=[g.size, g.embedding_size],
                              param_attr=fluid.ParamAttr(name=g.embedding_name))
            args = [emb if isinstance(x, BaseGeneratedInput) else x.input for x in ins]
            _NAMED.append({})
            try:
                prob = step(*args)
            finally:
                _NAMED.pop()
            topk_scores, topk_idx = L.topk(prob, k=beam_size)
            acc = L.elementwise_add(L.log(topk_scores), pre_scores, axis=0)
            sel_ids, sel_scores = L.beam_search(pre_ids, pre_scores, topk_idx, acc, beam_size, end_id=eos_id)
            L.increment(counter, 1, in_place=True)
            L.array_write(sel_ids, counter, ids_arr)
            L.array_write(sel_scores, counter, scores_arr)
            L.less_than(counter, limit, cond=cond)
        out_ids, _ = L.beam_search_decode(ids_arr, scores_arr, beam_size=beam_size, end_id=eos_id)
    return out_ids


# ------------------------------------------------------------------ sequence / shape layers
@_export
def expand_layer(input, expand_as, name=None, expand_level=None, **kw):
    with guard():
        return _named(_sized(_L().sequence_expand(input, expand_as), _size(input)), name)


@_export
def repeat_layer(input, num_repeats, as_row_vector=True, act=None, name=None, **kw):
    with guard():
        out = _L().expand(input, expand_times=[1, num_repeats]) if as_row_vector else \
            _L().reshape(_L().expand(_L().reshape(input, [-1, _size(input), 1]), [1, 1, num_repeats]),
                         [-1, _size(input) * num_repeats])
        return _named(_sized(_apply_act(out, act), _size(input) * num_repeats), name)


@_export
def seq_reshape_layer(input, reshape_size, act=None, name=None, **kw):
    with guard():
        return _named(_sized(_apply_act(_L().sequence_reshape(input, reshape_size), act), reshape_size), name)


@_export
def seq_concat_layer(a, b, act=None, name=None, **kw):
    with guard():
        return _named(_sized(_apply_act(_L().sequence_concat([a, b]), act), _size(a)), name)


@_export
def seq_slice_layer(input, starts, ends, name=None):
    """Slice each sequence: rows [starts, ends) (index tensors, one per sequence)."""
    with guard():
        length = _L().elementwise_sub(ends, starts) if ends is not None else None
        out = _L().sequence_slice(input, starts, length)
        out.shape = (-1, _size(input))  # rows of the input's width (a LoD-level slice)
        return _named(_sized(out, _size(input)), name)


@_export
def sub_seq_layer(input, offsets, sizes, act=None, bias_attr=None, name=None):
    with guard():
        return _named(_sized(_apply_act(_L().sequence_slice(input, offsets, sizes), act), _size(input)), name)


@_export
def sub_nested_seq_layer(input, selected_indices, name=None):
    """Select whole sub-sequences of a nested sequence by index (the gather of
    kmax_seq_score_layer's result)."""
    with guard():
        flat = _L().reshape(selected_indices, [-1])
        return _named(_sized(_L().gather(input, flat), _size(input)), name)


@_export
def kmax_seq_score_layer(input, name=None, beam_size=1):
    """Indices of the top ``beam_size`` scores of each sequence (one score per step)."""
    with guard():
        padded, _ = _L().sequence_pad(input, _L().fill_constant(shape=[1], dtype="float32", value=-1e30))
        _, idx = _L().topk(_L().reshape(padded, [0, -1]), k=beam_size)
        return _named(idx, name)


@_export
def eos_layer(input, eos_id, name=None, **kw):
    with guard():
        c = _L().fill_constant(shape=[1], dtype="int64", value=eos_id)
        return _named(_L().cast(_L().equal(input, c), "float32"), name)


@_export
def scaling_layer(input, weight, name=None, **kw):
    """y_i = w_i x_i (one scalar weight per row)."""
    with guard():
        return _named(_sized(_L().elementwise_mul(input, weight, axis=0), _size(input)), name)


@_export
def power_layer(input, weight, name=None, **kw):
    """y_i = x_i ^ w_i (one exponent per row)."""
    with guard():
        return _named(_sized(_L().exp(_L().elementwise_mul(_L().log(input), weight, axis=0)), _size(input)), name)


@_export
def interpolation_layer(input, weight, name=None, **kw):
    """y = w a + (1 - w) b (one weight per row)."""
    a, b = input
    with guard():
        d = _L().elementwise_mul(_L().elementwise_sub(a, b), weight, axis=0)
        return _named(_sized(_L().elementwise_add(d, b), _size(a)), name)


@_export
def slope_intercept_layer(input, slope=1.0, intercept=0.0, name=None, **kw):
    with guard():
        return _named(_sized(_L().scale(input, scale=float(slope), bias=float(intercept)), _size(input)), name)


@_export
def sum_to_one_norm_layer(input, name=None, **kw):
    with guard():
        return _named(_sized(_L().elementwise_div(input, _L().reduce_sum(input, dim=1, keep_dim=True), axis=0),
                             _size(input)), name)


@_export
def row_l2_norm_layer(input, name=None, **kw):
    with guard():
        return _named(_sized(_L().l2_normalize(input, axis=1), _size(input)), name)


@_export
def cos_sim(a, b, scale=1, size=1, name=None, **kw):
    with guard():
        return _named(_sized(_L().scale(_L().cos_sim(a, b), scale=float(scale)), 1), name)


@_export
def l2_distance_layer(x, y, name=None, **kw):
    with guard():
        d = _L().elementwise_sub(x, y)
        return _named(_sized(_L().sqrt(_L().reduce_sum(_L().square(d), dim=1, keep_dim=True)), 1), name)


@_export
def dot_prod_layer(input1, input2, name=None, **kw):
    with guard():
        return _named(_sized(_L().reduce_sum(_L().elementwise_mul(input1, input2), dim=1, keep_dim=True), 1),
                      name)


@_export
def out_prod_layer(input1, input2, name=None, **kw):
    a, b = _size(input1), _size(input2)
    with guard():
        o = _L().matmul(_L().reshape(input1, [-1, a, 1]), _L().reshape(input2, [-1, 1, b]))
        return _named(_sized(_L().reshape(o, [-1, a * b]), a * b), name)


@_export
def linear_comb_layer(weights, vectors, size=None, name=None, **kw):
    """z = sum_i w_i v_i with vectors [N, M * size] viewed as M vectors of ``size``."""
    m = _size(weights)
    size = size or _size(vectors) // m
    with guard():
        v = _L().reshape(vectors, [-1, m, size])
        z = _L().matmul(_L().reshape(weights, [-1, 1, m]), v)
        return _named(_sized(_L().reshape(z, [-1, size]), size), name)


convex_comb_layer = linear_comb_layer
__all__.append("convex_comb_layer")


@_export
def tensor_layer(a, b, size, act=None, name=None, param_attr=None, bias_attr=None, **kw):
    with guard():
        return _named(_sized(_L().bilinear_tensor_product(a, b, size, act=_act.act_name(act) or None), size), name)


@_export
def selective_fc_layer(input, size, select=None, act=None, name=None, pass_generation=False, has_selected_colums=True,
                       mul_ratio=0.02, param_attr=None, bias_attr=None, **kw):
    """fc whose output keeps only the selected columns (``select``: a 0/1 mask of
    [N, size]; none = all columns)."""
    with guard():
        out = _L().fc(input=input, size=size, act=_act.act_name(act) or None)
        if select is not None:
            out = _L().elementwise_mul(out, select)
        return _named(_sized(out, size), name)


@_export
def sampling_id_layer(input, name=None, **kw):
    with guard():
        return _named(_L().sampling_id(input), name)


@_export
def conv_shift_layer(a, b, name=None, **kw):
    with guard():
        return _named(_sized(_L().conv_shift(a, b), _size(a)), name)


@_export
def gated_unit_layer(input, size, act=None, name=None, gate_attr=None, gate_param_attr=None, gate_bias_attr=True,
                     inproj_attr=None, inproj_param_attr=None, inproj_bias_attr=True, layer_attr=None):
    """act(x W + b) * sigmoid(x V + c) (gated linear unit).  A composite, as in the
    reference (trainer_config_helpers/layers.py gated_unit_layer): the layers
    <name>_input_proj (fc), <name>_gate (fc, sigmoid) and <name>_gated_act (mixed
    layer with a dot_mul operator), each recorded in the ModelConfig."""
    from . import config_proto as _cp
    from . import fc_layer as _fc, mixed_layer as _mixed  # the recorded (package-level) layer functions

    rec = _cp.current()
    if name is None:
        name = rec.name_for("gated_unit_layer", None) if rec is not None else "__gated_unit_layer__"
    proj = _fc(input=input, size=size, act=act or _act.Tanh(), name=f"{name}_input_proj",
               param_attr=inproj_param_attr, bias_attr=inproj_bias_attr, layer_attr=inproj_attr)
    gate = _fc(input=input, size=size, act=_act.Sigmoid(), name=f"{name}_gate",
               param_attr=gate_param_attr, bias_attr=gate_bias_attr, layer_attr=gate_attr)
    return _mixed(size=size, input=[dotmul_operator(a=proj, b=gate)], name=f"{name}_gated_act", bias_attr=False,
                  layer_attr=layer_attr)


@_export
def clip_layer(input, min, max, name=None):
    with guard():
        return _named(_sized(_L().clip(input, min=float(min), max=float(max)), _size(input)), name)


@_export
def scale_shift_layer(input, name=None, param_attr=None, bias_attr=None):
    """y = w x + b with scalar learned w, b."""
    with guard():
        helper = LayerHelper("scale_shift")
        w = helper.create_parameter(attr=helper.param_attr, shape=[1], dtype="float32",
                                    default_initializer=fluid.initializer.Constant(1.0))
        out = _L().elementwise_mul(input, w)
        if bias_attr is not False:
            b = helper.create_parameter(attr=helper.bias_attr, shape=[1], dtype="float32", is_bias=True)
            out = _L().elementwise_add(out, b)
        return _named(_sized(out, _size(input)), name)


@_export
def resize_layer(input, size, name=None):
    with guard():
        return _named(_sized(_L().reshape(input, [-1, size]), size), name)


@_export
def trans_layer(input, name=None, **kw):
    """The minibatch matrix transposed ([N, size] -> [size, N]).  Like the reference
    (size = the input's size) a following layer sees rows of the input's width, so
    the declared shape keeps it: a consumer's weights are sized as if N == size."""
    with guard():
        out = _L().transpose(input, perm=[1, 0])
        w = _size(input)
        if w:
            out.shape = (-1, w)
        return _named(_sized(out, w), name)


@_export
def rotate_layer(input, height, width, name=None, **kw):
    """Rotate each [height, width] sample 90 degrees clockwise."""
    with guard():
        x = _L().reshape(input, [-1, height, width])
        x = _L().transpose(x, perm=[0, 2, 1])
        x = _L().reverse(x, axis=2)
        return _named(_sized(_L().reshape(x, [-1, height * width]), height * width), name)


@_export
def multiplex_layer(input, name=None, **kw):
    """input[0]: the int index per row; input[1:]: the candidates."""
    with guard():
        return _named(_sized(_L().multiplex(list(input[1:]), input[0]), _size(input[1])), name)


@_export
def row_conv_layer(input, context_len, act=None, name=None, param_attr=None, **kw):
    with guard():
        return _named(_sized(_L().row_conv(input, future_context_size=context_len - 1,
                                           act=_act.act_name(act) or None), _size(input)), name)


@_export
def prelu_layer(input, name=None, partial_sum=1, channel_shared=None, num_channels=None, param_attr=None, **kw):
    """Parametric ReLU with one slope per `partial_sum` consecutive elements of the
    row (reference layers.py prelu_layer / PReluLayer): channel_shared=True -> one
    slope for the row, False -> one per channel of num_channels.  Slopes [1, size /
    partial_sum], initialised to 0.25; the row is viewed as [n_slopes, partial_sum]."""
    size = _size(input)
    if channel_shared is not None:
        partial_sum = size if channel_shared else size // (num_channels or 1)
    if partial_sum <= 0 or size % partial_sum:
        raise ValueError(f"prelu_layer: partial_sum {partial_sum} must divide the layer size {size}")
    n_w = size // partial_sum
    with guard():
        helper = LayerHelper("prelu", param_attr=param_attr)
        alpha = helper.create_parameter(attr=helper.param_attr, shape=[1, n_w], dtype="float32",
                                        default_initializer=fluid.initializer.Constant(0.25))
        x = _L().reshape(input, [-1, n_w, partial_sum, 1])
        y = helper.create_variable_for_type_inference("float32")
        helper.append_op(type="prelu", inputs={"X": x, "Alpha": alpha}, outputs={"Out": y}, attrs={"mode": "channel"})
        y = _L().reshape(y, list(input.shape) if len(input.shape) == 4 else [-1, size])
        return _named(_sized(y, size), name)


@_export
def factorization_machine(input, factor_size, act=None, name=None, param_attr=None, **kw):
    """Second-order FM term: 0.5 * sum_f ((x V)_f^2 - (x^2)(V^2)_f)."""
    d = _size(input)
    with guard():
        helper = LayerHelper("factorization_machine")
        v = helper.create_parameter(attr=helper.param_attr, shape=[d, factor_size], dtype="float32")
        xv = _L().matmul(input, v)
        x2v2 = _L().matmul(_L().square(input), _L().square(v))
        out = _L().scale(_L().reduce_sum(_L().elementwise_sub(_L().square(xv), x2v2), dim=1, keep_dim=True), 0.5)
        return _named(_sized(_apply_act(out, act), 1), name)


@_export
def printer_layer(input, format=None, name=None):
    """Print the layers' values at run time; recorded as a "print" LayerConfig (no
    output of its own: the config keeps using the printed layers)."""
    from . import config_proto as _cp

    ins = input if isinstance(input, (list, tuple)) else [input]
    rec = _cp.current()
    if rec is not None and not rec.depth:
        lname = rec.name_for("print", name)
        srcs = [rec.layer_name(x) or x.name for x in ins]
        lc = {"name": lname, "type": "print", "active_type": "",
              "inputs": [{"input_layer_name": n} for n in srcs],
              "user_arg": format or "\n".join(f"layer={n} %s" for n in srcs)}
        rec.layers.append(lc)
        rec.by_name[lname] = lc
        rec.parents[lname] = srcs
    with guard():
        for x in ins:
            _L().Print(x, message=format or x.name)
    return input


print_layer = printer_layer
__all__.append("print_layer")


# ------------------------------------------------------------------ image layers
def _img(input, num_channels):
    from ..v2.layer import _as_image

    return _as_image(input, num_channels or 1)


@_export
def img_cmrnorm_layer(input, size, scale=0.0128, power=0.75, name=None, num_channels=None, **kw):
    with guard():
        return _named(_L().lrn(_img(input, num_channels), n=size, alpha=scale, beta=power), name)


@_export
def bilinear_interp_layer(input, out_size_x=None, out_size_y=None, name=None, **kw):
    with guard():
        return _named(_L().resize_bilinear(input, out_shape=[out_size_y, out_size_x]), name)


@_export
def block_expand_layer(input, block_x=0, block_y=0, stride_x=0, stride_y=0, padding_x=0, padding_y=0,
                       num_channels=None, name=None, **kw):
    with guard():
        return _named(_L().im2sequence(_img(input, num_channels), filter_size=[block_y, block_x],
                                       stride=[stride_y, stride_x], padding=[padding_y, padding_x]), name)


@_export
def maxout_layer(input, groups, num_channels=None, name=None, **kw):
    with guard():
        return _named(_L().maxout(_img(input, num_channels), groups=groups), name)


@_export
def spp_layer(input, name=None, num_channels=None, pool_type=None, pyramid_height=None, **kw):
    from ..v2 import pooling as _pool

    with guard():
        ptype = "avg" if isinstance(pool_type, _pool.Avg) else "max"
        out = _op("spp", {"X": [_img(input, num_channels)]}, {"Out": "float32"},
                  {"pyramid_height": int(pyramid_height), "pooling_type": ptype})["Out"]
        return _named(out, name)


@_export
def pad_layer(input, pad_c=None, pad_h=None, pad_w=None, name=None, **kw):
    pc, ph, pw = pad_c or [0, 0], pad_h or [0, 0], pad_w or [0, 0]
    with guard():
        return _named(_L().pad(input, paddings=[0, 0] + list(pc) + list(ph) + list(pw)), name)


@_export
def crop_layer(input, offset, axis=2, shape=None, name=None, **kw):
    x, ref = (input[0], input[1]) if isinstance(input, (list, tuple)) else (input, None)
    with guard():
        nd = len(x.shape)
        offs = [0] * axis + list(offset)
        offs = offs + [0] * (nd - len(offs))
        return _named(_L().crop(x, shape=ref if ref is not None else shape, offsets=offs), name)


@_export
def switch_order_layer(input, name=None, reshape_axis=None, act=None, **kw):
    """NCHW -> NHWC."""
    with guard():
        return _named(_apply_act(_L().transpose(input, perm=[0, 2, 3, 1]), act), name)


@_export
def img_pool3d_layer(input, pool_size, num_channels=None, stride=1, padding=0, pool_type=None, name=None, **kw):
    from ..v2 import pooling as _pool

    with guard():
        ptype = "avg" if isinstance(pool_type, _pool.Avg) else "max"
        return _named(_L().pool3d(_as_volume(input, num_channels), pool_size=pool_size, pool_type=ptype,
                                  pool_stride=stride, pool_padding=padding, ceil_mode=True), name)


def _as_volume(input, num_channels):
    """[N, C * D * H * W] rows of a data_layer(depth=, height=, width=) as [N, C, D, H, W]."""
    if len(input.shape) == 5:
        return input
    dhw = getattr(input, "v2_dhw", None)
    if dhw is None:
        raise ValueError("3-D layers need an input with depth / height / width (data_layer(depth=...))")
    d, h, w = dhw
    return _L().reshape(input, [-1, num_channels or max(_size(input) // (d * h * w), 1), d, h, w])


@_export
def img_conv3d_layer(input, filter_size, num_filters, num_channels=None, stride=1, padding=0, act=None, groups=1,
                     name=None, bias_attr=None, param_attr=None, **kw):
    with guard():
        x = _as_volume(input, num_channels)
        conv = _L().conv3d_transpose if kw.get("trans") else _L().conv3d
        from ..v2 import attr as _attr

        return _named(conv(x, num_filters=num_filters, filter_size=filter_size, stride=stride, padding=padding,
                           groups=groups, act=_act.act_name(act) or None, param_attr=_attr.to_fluid(param_attr),
                           bias_attr=_attr.to_fluid(bias_attr)), name)


@_export
def upsample_layer(input, scale=2, name=None, upsample_size=None, pad_out_x=False, pad_out_y=False, **kw):
    """Max-unpooling of ``input[0]`` at the argmax positions ``input[1]``."""
    x, mask = input
    with guard():
        out = _op("unpool", {"X": [x], "Indices": [mask]}, {"Out": "float32"},
                  {"unpooling_type": "max", "ksize": [scale, scale], "strides": [scale, scale],
                   "paddings": [0, 0]})["Out"]
        return _named(out, name)


@_export
def scale_sub_region_layer(input, indices, value, name=None):
    """Multiply the [C, H, W] box of each sample given by ``indices`` (6 ints:
    c0, c1, h0, h1, w0, w1, 1-based inclusive) by ``value``."""
    with guard():
        out = _op("scale_sub_region", {"X": [input], "Indices": [indices]}, {"Out": "float32"},
                  {"value": float(value)})["Out"]
        return _named(out, name)


@_export
def cross_channel_norm_layer(input, name=None, param_attr=None):
    """L2 normalisation across channels with a learned per-channel scale (SSD)."""
    c = input.shape[1]
    with guard():
        helper = LayerHelper("cross_channel_norm")
        w = helper.create_parameter(attr=helper.param_attr, shape=[c], dtype="float32",
                                    default_initializer=fluid.initializer.Constant(20.0))
        return _named(_L().elementwise_mul(_L().l2_normalize(input, axis=1), w, axis=1), name)


@_export
def priorbox_layer(input, image, aspect_ratio, variance, min_size, max_size=None, name=None):
    with guard():
        boxes, var = _L().prior_box(input, image, min_sizes=list(min_size), max_sizes=list(max_size or []),
                                    aspect_ratios=list(aspect_ratio), variance=list(variance))
        return _named(boxes, name)


@_export
def multibox_loss_layer(input_loc, input_conf, priorbox, label, num_classes, overlap_threshold=0.5,
                        neg_pos_ratio=3.0, neg_overlap=0.5, background_id=0, name=None):
    with guard():
        loc = input_loc[0] if isinstance(input_loc, (list, tuple)) else input_loc
        conf = input_conf[0] if isinstance(input_conf, (list, tuple)) else input_conf
        gt_box = _L().slice(label, axes=[1], starts=[1], ends=[5])
        gt_label = _L().cast(_L().slice(label, axes=[1], starts=[0], ends=[1]), "int64")
        var = _L().fill_constant_batch_size_like(priorbox, shape=[-1, 4], dtype="float32", value=0.1)
        loss = _L().ssd_loss(loc, conf, gt_box, gt_label, priorbox, var, background_label=background_id,
                             overlap_threshold=overlap_threshold, neg_pos_ratio=neg_pos_ratio,
                             neg_overlap=neg_overlap)
        return _named(_L().reduce_sum(loss), name)


@_export
def detection_output_layer(input_loc, input_conf, priorbox, num_classes, nms_threshold=0.45, nms_top_k=400,
                           keep_top_k=200, confidence_threshold=0.01, background_id=0, name=None):
    with guard():
        loc = input_loc[0] if isinstance(input_loc, (list, tuple)) else input_loc
        conf = input_conf[0] if isinstance(input_conf, (list, tuple)) else input_conf
        var = _L().fill_constant_batch_size_like(priorbox, shape=[-1, 4], dtype="float32", value=0.1)
        return _named(_L().detection_output(loc, conf, priorbox, var, background_label=background_id,
                                            nms_threshold=nms_threshold, nms_top_k=nms_top_k,
                                            keep_top_k=keep_top_k, score_threshold=confidence_threshold), name)


@_export
def roi_pool_layer(input, rois, pooled_width, pooled_height, spatial_scale, num_channels=None, name=None):
    with guard():
        out = _L().roi_pool(input, rois, pooled_height=pooled_height, pooled_width=pooled_width,
                            spatial_scale=spatial_scale)
        c = num_channels or (int(input.shape[1]) if len(input.shape) == 4 else 1)
        return _named(_sized(out, c * pooled_height * pooled_width), name)


# ------------------------------------------------------------------ costs
def _cost_out(c, name, coeff=1.0):
    if coeff != 1.0:
        c = _L().scale(c, scale=float(coeff))
    return _named(_sized(c, 1), name)


@_export
def hsigmoid(input, label, num_classes=None, name=None, bias_attr=None, param_attr=None, **kw):
    with guard():
        return _cost_out(_L().hsigmoid(input, label, num_classes=num_classes), name)


@_export
def crf_layer(input, label, size=None, weight=None, param_attr=None, name=None, coeff=1.0, **kw):
    with guard():
        ll = _L().linear_chain_crf(input, label, param_attr=param_attr if param_attr is not None else
                                   fluid.ParamAttr(name=(name or "crf") + ".w"))
        return _cost_out(_L().mean(ll), name, coeff)


@_export
def crf_decoding_layer(input, size, label=None, param_attr=None, name=None, **kw):
    with guard():
        return _named(_L().crf_decoding(input, param_attr=param_attr if param_attr is not None else
                                        fluid.ParamAttr(name=(name or "crf") + ".w"), label=label), name)


@_export
def warp_ctc_layer(input, label, size=None, name=None, blank=0, norm_by_times=False, **kw):
    """input: linear activations (the op applies the softmax)."""
    with guard():
        return _cost_out(_L().mean(_L().warpctc(input, label, blank=blank, norm_by_times=norm_by_times)), name)


@_export
def ctc_layer(input, label, size=None, name=None, norm_by_times=False, **kw):
    """input: softmax probabilities (v1 ctc_layer); blank = size - 1.  log p passed
    to the softmax-applying CTC op gives back p."""
    size = size or _size(input)
    with guard():
        logp = _L().log(input)
        return _cost_out(_L().mean(_L().warpctc(logp, label, blank=size - 1, norm_by_times=norm_by_times)), name)


@_export
def nce_layer(input, label, num_classes=None, act=None, param_attr=None, weight=None, num_neg_samples=10,
              neg_distribution=None, name=None, bias_attr=None, layer_attr=None):
    x = _L().concat(list(input), axis=1) if isinstance(input, (list, tuple)) else input
    if num_classes is None:  # reference nce_layer: the label layer's size
        num_classes = _size(label)
    with guard():
        return _cost_out(_L().mean(_L().nce(x, label, num_total_classes=num_classes,
                                            num_neg_samples=num_neg_samples)), name)


@_export
def cross_entropy_with_selfnorm(input, label, name=None, coeff=1.0, softmax_selfnorm_alpha=0.1, layer_attr=None):
    """-log(p_label / Z) + alpha * log(Z)^2 over unnormalised positive scores."""
    with guard():
        z = _L().reduce_sum(input, dim=1, keep_dim=True)
        p = _L().elementwise_div(input, z, axis=0)
        ce = _L().cross_entropy(p, label)
        lz = _L().log(z)
        c = _L().elementwise_add(ce, _L().scale(_L().square(lz), scale=float(softmax_selfnorm_alpha)))
        return _cost_out(_L().mean(c), name, coeff)


@_export
def multi_binary_label_cross_entropy(input, label, name=None, coeff=1.0, layer_attr=None):
    """input: probabilities; label: a 0/1 matrix of the same shape."""
    with guard():
        eps = 1e-7
        p = _L().clip(input, min=eps, max=1.0 - eps)
        one = _L().fill_constant_batch_size_like(p, shape=[-1, _size(input)], dtype="float32", value=1.0)
        t = _L().elementwise_add(_L().elementwise_mul(label, _L().log(p)),
                                 _L().elementwise_mul(_L().elementwise_sub(one, label),
                                                      _L().log(_L().elementwise_sub(one, p))))
        return _cost_out(_L().mean(_L().scale(_L().reduce_sum(t, dim=1), scale=-1.0)), name, coeff)


@_export
def sum_cost(input, name=None, layer_attr=None):
    with guard():
        return _cost_out(_L().reduce_sum(input), name)


@_export
def rank_cost(left, right, label, weight=None, name=None, coeff=1.0, layer_attr=None):
    with guard():
        return _cost_out(_L().mean(_L().rank_loss(label, left, right)), name, coeff)


@_export
def lambda_cost(input, score, name=None, NDCG_num=5, max_sort_size=-1, layer_attr=None):
    """LambdaRank over each query's sequence of scores: the pairwise logistic loss of
    every (i, j) with score_i > score_j, weighted by the |delta NDCG@k| of swapping
    them (the gradient LambdaCost applies)."""
    with guard():
        L = _L()
        s_in, _ = L.sequence_pad(input, L.fill_constant(shape=[1], dtype="float32", value=0.0))
        s_lab, _ = L.sequence_pad(score, L.fill_constant(shape=[1], dtype="float32", value=0.0))
        s_in = L.reshape(s_in, [0, -1])
        s_lab = L.reshape(s_lab, [0, -1])
        n = -1
        si = L.unsqueeze(s_in, [2])
        sj = L.unsqueeze(s_in, [1])
        li = L.unsqueeze(s_lab, [2])
        lj = L.unsqueeze(s_lab, [1])
        better = L.cast(L.greater_than(L.elementwise_sub(li, lj), L.fill_constant([1], "float32", 0.0)),
                        "float32")
        gain = L.abs(L.elementwise_sub(L.elementwise_sub(L.exp(L.scale(li, 0.6931471805599453)),
                                                         L.exp(L.scale(lj, 0.6931471805599453))),
                                       L.fill_constant([1], "float32", 0.0)))
        pair = L.softplus(L.scale(L.elementwise_sub(si, sj), scale=-1.0))
        c = L.reduce_sum(L.elementwise_mul(L.elementwise_mul(pair, better), gain), dim=[1, 2])
        del n
        return _cost_out(L.mean(c), name)


@_export
def huber_regression_cost(input, label, name=None, delta=1.0, coeff=1.0, layer_attr=None):
    with guard():
        return _cost_out(_L().mean(_L().huber_loss(input, label, delta=float(delta))), name, coeff)


@_export
def huber_classification_cost(input, label, name=None, coeff=1.0, layer_attr=None):
    """Modified Huber loss for {0, 1} labels (mapped to {-1, +1})."""
    with guard():
        lab = _L().cast(label, "float32")
        out = _op("modified_huber_loss", {"X": [input], "Y": [lab]},
                  {"Out": "float32", "IntermediateVal": "float32"})["Out"]
        return _cost_out(_L().mean(out), name, coeff)


@_export
def smooth_l1_cost(input, label, name=None, coeff=1.0, layer_attr=None):
    with guard():
        return _cost_out(_L().mean(_L().smooth_l1(input, label)), name, coeff)


@_export
def cross_entropy_over_beam(input, name=None):
    """Cross entropy of the gold path over the beam's expanded candidates: for every
    BeamInput, -log softmax(candidate_scores)[gold]."""
    beams = input if isinstance(input, (list, tuple)) else [input]
    with guard():
        terms = []
        for b in beams:
            prob = _L().softmax(b.candidate_scores)
            terms.append(_L().cross_entropy(prob, b.gold))
        s = terms[0] if len(terms) == 1 else _L().sums(terms)
        return _cost_out(_L().mean(s), name)


# ------------------------------------------------------------------ operators / unwrapping
@_export
def conv_operator(img, filter, filter_size, num_filters, num_channels=None, stride=1, padding=0,
                  filter_size_y=None, stride_y=None, padding_y=None, trans=False):
    """A convolution whose filter is another layer's output (one filter set per
    sample): a deferred term of a mixed layer, like a projection."""
    def build(size):
        with guard():
            c = num_channels or 1
            fy = filter_size_y or filter_size
            side = int(round((_size(img) // c) ** 0.5))
            x = _L().reshape(img, [-1, c, side, side])
            attrs = {"strides": [stride_y or stride, stride], "paddings": [padding_y or padding, padding],
                     "dilations": [1, 1], "groups": 1}
            if trans:
                w = _L().reshape(filter, [c, num_filters, fy, filter_size])
                out = _op("conv2d_transpose", {"Input": [x], "Filter": [w]}, {"Output": "float32"}, attrs)["Output"]
            else:
                w = _L().reshape(filter, [num_filters, c, fy, filter_size])
                out = _op("conv2d", {"Input": [x], "Filter": [w]}, {"Output": "float32"}, attrs)["Output"]
            n = _conv_flat(img, c, filter_size, stride, padding, num_filters, trans)
            return _sized(_L().reshape(out, [-1, n]), n)
    op = _Projection(build, None, img, "convt_op" if trans else "conv_op")
    op.v1_operands = [img, filter]  # the image and the filter layer (config_proto.py operator_confs)
    op.v1_operator = ("convt" if trans else "conv", 1.0)
    op.v1_conv = dict(filter_size=filter_size, num_filters=num_filters, channels=num_channels or 1, stride=stride,
                      padding=padding, groups=1, trans=trans, filter_size_y=filter_size_y, stride_y=stride_y,
                      padding_y=padding_y)
    return op


def _conv_flat(img, c, f, s, p, nf, trans):
    """C * H * W of a (transposed) convolution of a square image layer."""
    side = int(round((_size(img) // c) ** 0.5))
    o = (side - 1) * s + f - 2 * p if trans else (side + 2 * p - f) // s + 1
    return int(nf * o * o)


def _prod_shape(v):
    n = 1
    for d in (v.shape or ())[1:]:
        n *= max(int(d), 1)
    return n


def _unwrap_args(fn):
    import functools

    @functools.wraps(fn)
    def w(*args, **kw):
        from .config_proto import unwrap

        return fn(*[unwrap(a) for a in args], **{k: unwrap(v) for k, v in kw.items()})
    return w


# projection / operator helpers accept a finished ``with mixed_layer() as m`` context
for _n in ("full_matrix_projection", "trans_full_matrix_projection", "table_projection", "identity_projection",
           "slice_projection", "dotmul_projection", "scaling_projection", "dotmul_operator", "context_projection",
           "conv_projection", "conv_operator"):
    globals()[_n] = _unwrap_args(globals()[_n])
del _n
