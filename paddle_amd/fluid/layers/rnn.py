"""Recurrent, structured-prediction, sampled-loss and decoding layers
(python/paddle/fluid/layers/nn.py: dynamic_lstm, dynamic_lstmp, dynamic_gru,
gru_unit, lstm_unit, linear_chain_crf, crf_decoding, chunk_eval, warpctc,
ctc_greedy_decoder, edit_distance, nce, hsigmoid, beam_search,
beam_search_decode).  Parameter shapes and return values follow the reference
layers; the ops live in operators/{rnn,structured}_ops.py."""
from __future__ import annotations

from ..framework import Variable
from ..layer_helper import LayerHelper
from ..param_attr import ParamAttr

__all__ = ["dynamic_lstm", "dynamic_lstmp", "dynamic_gru", "gru_unit", "lstm_unit", "linear_chain_crf",
           "crf_decoding", "chunk_eval", "warpctc", "ctc_greedy_decoder", "edit_distance", "nce", "hsigmoid",
           "beam_search", "beam_search_decode"]


def _tmp(helper, dtype, stop_gradient=False):
    return helper.create_variable_for_type_inference(dtype=dtype, stop_gradient=stop_gradient)


def dynamic_lstm(input, size, h_0=None, c_0=None, param_attr=None, bias_attr=None, use_peepholes=True,
                 is_reverse=False, gate_activation="sigmoid", cell_activation="tanh",
                 candidate_activation="tanh", dtype="float32", name=None):
    helper = LayerHelper("lstm", **locals())
    D = size // 4
    w = helper.create_parameter(attr=helper.param_attr, shape=[D, 4 * D], dtype=dtype)
    b = helper.create_parameter(attr=helper.bias_attr, shape=[1, 7 * D if use_peepholes else 4 * D], dtype=dtype,
                                is_bias=True)
    hidden, cell = _tmp(helper, dtype), _tmp(helper, dtype)
    bg, bc = _tmp(helper, dtype, True), _tmp(helper, dtype, True)
    ins = {"Input": input, "Weight": w, "Bias": b}
    if h_0 is not None:
        ins["H0"] = h_0
    if c_0 is not None:
        ins["C0"] = c_0
    helper.append_op(type="lstm", inputs=ins,
                     outputs={"Hidden": hidden, "Cell": cell, "BatchGate": bg, "BatchCellPreAct": bc},
                     attrs={"use_peepholes": use_peepholes, "is_reverse": is_reverse,
                            "gate_activation": gate_activation, "cell_activation": cell_activation,
                            "candidate_activation": candidate_activation})
    return hidden, cell


def dynamic_lstmp(input, size, proj_size, param_attr=None, bias_attr=None, use_peepholes=True, is_reverse=False,
                  gate_activation="sigmoid", cell_activation="tanh", candidate_activation="tanh",
                  proj_activation="tanh", dtype="float32", name=None):
    helper = LayerHelper("lstmp", **locals())
    D = size // 4
    w = helper.create_parameter(attr=helper.param_attr, shape=[proj_size, 4 * D], dtype=dtype)
    pw = helper.create_parameter(attr=helper.param_attr, shape=[D, proj_size], dtype=dtype)
    b = helper.create_parameter(attr=helper.bias_attr, shape=[1, 7 * D if use_peepholes else 4 * D], dtype=dtype,
                                is_bias=True)
    proj, cell = _tmp(helper, dtype), _tmp(helper, dtype)
    outs = {"Projection": proj, "Cell": cell}
    for s in ("BatchGate", "BatchCellPreAct", "BatchHidden"):
        outs[s] = _tmp(helper, dtype, True)
    helper.append_op(type="lstmp", inputs={"Input": input, "Weight": w, "ProjWeight": pw, "Bias": b},
                     outputs=outs,
                     attrs={"use_peepholes": use_peepholes, "is_reverse": is_reverse,
                            "gate_activation": gate_activation, "cell_activation": cell_activation,
                            "candidate_activation": candidate_activation, "proj_activation": proj_activation})
    return proj, cell


def dynamic_gru(input, size, param_attr=None, bias_attr=None, is_reverse=False, gate_activation="sigmoid",
                candidate_activation="tanh", h_0=None):
    helper = LayerHelper("gru", **locals())
    dtype = helper.input_dtype()
    w = helper.create_parameter(attr=helper.param_attr, shape=[size, 3 * size], dtype=dtype)
    b = helper.create_parameter(attr=helper.bias_attr, shape=[1, 3 * size], dtype=dtype, is_bias=True)
    ins = {"Input": input, "Weight": w, "Bias": b}
    if h_0 is not None:
        ins["H0"] = h_0
    hidden = _tmp(helper, dtype)
    outs = {"Hidden": hidden}
    for s in ("BatchGate", "BatchResetHiddenPrev", "BatchHidden"):
        outs[s] = _tmp(helper, dtype, True)
    helper.append_op(type="gru", inputs=ins, outputs=outs,
                     attrs={"is_reverse": is_reverse, "gate_activation": gate_activation,
                            "activation": candidate_activation})
    return hidden


_ACT = {"identity": 0, "sigmoid": 1, "tanh": 2, "relu": 3}


def gru_unit(input, hidden, size, param_attr=None, bias_attr=None, activation="tanh", gate_activation="sigmoid"):
    helper = LayerHelper("gru_unit", **locals())
    dtype = helper.input_dtype()
    D = size // 3
    w = helper.create_parameter(attr=helper.param_attr, shape=[D, 3 * D], dtype=dtype)
    ins = {"Input": input, "HiddenPrev": hidden, "Weight": w}
    if helper.bias_attr:
        ins["Bias"] = helper.create_parameter(attr=helper.bias_attr, shape=[1, 3 * D], dtype=dtype, is_bias=True)
    gate, reset, upd = _tmp(helper, dtype), _tmp(helper, dtype), _tmp(helper, dtype)
    helper.append_op(type="gru_unit", inputs=ins, outputs={"Gate": gate, "ResetHiddenPrev": reset, "Hidden": upd},
                     attrs={"activation": _ACT[activation], "gate_activation": _ACT[gate_activation]})
    return upd, reset, gate


def lstm_unit(x_t, hidden_t_prev, cell_t_prev, forget_bias=0.0, param_attr=None, bias_attr=None, name=None):
    from .nn import fc
    from .tensor import concat

    helper = LayerHelper("lstm_unit", **locals())
    size = cell_t_prev.shape[1]
    fc_out = fc(input=concat([x_t, hidden_t_prev], axis=1), size=4 * size, param_attr=param_attr,
                bias_attr=bias_attr)
    dtype = x_t.dtype
    c, h = _tmp(helper, dtype), _tmp(helper, dtype)
    helper.append_op(type="lstm_unit", inputs={"X": fc_out, "C_prev": cell_t_prev}, outputs={"C": c, "H": h},
                     attrs={"forget_bias": forget_bias})
    return h, c


def linear_chain_crf(input, label, param_attr=None):
    helper = LayerHelper("linear_chain_crf", **locals())
    size = input.shape[1]
    trans = helper.create_parameter(attr=helper.param_attr, shape=[size + 2, size], dtype=helper.input_dtype())
    ll = _tmp(helper, helper.input_dtype())
    outs = {"LogLikelihood": ll}
    for s in ("Alpha", "EmissionExps", "TransitionExps"):
        outs[s] = _tmp(helper, helper.input_dtype(), True)
    helper.append_op(type="linear_chain_crf", inputs={"Emission": [input], "Transition": trans, "Label": label},
                     outputs=outs)
    return ll


def crf_decoding(input, param_attr, label=None):
    helper = LayerHelper("crf_decoding", **locals())
    pa = param_attr if isinstance(param_attr, ParamAttr) else ParamAttr(name=param_attr)
    trans = helper.main_program.global_block().var(pa.name)
    path = helper.create_variable_for_type_inference(dtype="int64", stop_gradient=True)
    ins = {"Emission": [input], "Transition": trans}
    if label is not None:
        ins["Label"] = label
    helper.append_op(type="crf_decoding", inputs=ins, outputs={"ViterbiPath": [path]})
    return path


def chunk_eval(input, label, chunk_scheme, num_chunk_types, excluded_chunk_types=None):
    helper = LayerHelper("chunk_eval", **locals())
    outs = {}
    res = []
    for s, dt in (("Precision", "float32"), ("Recall", "float32"), ("F1-Score", "float32"),
                  ("NumInferChunks", "int64"), ("NumLabelChunks", "int64"), ("NumCorrectChunks", "int64")):
        v = helper.create_variable_for_type_inference(dtype=dt, stop_gradient=True)
        outs[s] = [v]
        res.append(v)
    helper.append_op(type="chunk_eval", inputs={"Inference": [input], "Label": [label]}, outputs=outs,
                     attrs={"num_chunk_types": num_chunk_types, "chunk_scheme": chunk_scheme,
                            "excluded_chunk_types": excluded_chunk_types or []})
    return tuple(res)


def warpctc(input, label, blank=0, norm_by_times=False):
    helper = LayerHelper("warpctc", **locals())
    loss = _tmp(helper, input.dtype)
    grad = _tmp(helper, input.dtype, True)
    helper.append_op(type="warpctc", inputs={"Logits": [input], "Label": [label]},
                     outputs={"WarpCTCGrad": [grad], "Loss": [loss]},
                     attrs={"blank": blank, "norm_by_times": norm_by_times})
    return loss


def ctc_greedy_decoder(input, blank, name=None):
    from .nn import topk

    helper = LayerHelper("ctc_greedy_decoder", **locals())
    _, idx = topk(input, k=1)
    out = helper.create_variable_for_type_inference(dtype="int64", stop_gradient=True)
    helper.append_op(type="ctc_align", inputs={"Input": [idx]}, outputs={"Output": [out]},
                     attrs={"merge_repeated": True, "blank": blank})
    return out


def edit_distance(input, label, normalized=True, ignored_tokens=None):
    helper = LayerHelper("edit_distance", **locals())
    if ignored_tokens:
        ei = helper.create_variable_for_type_inference(dtype="int64", stop_gradient=True)
        el = helper.create_variable_for_type_inference(dtype="int64", stop_gradient=True)
        helper.append_op(type="sequence_erase", inputs={"X": [input]}, outputs={"Out": [ei]},
                         attrs={"tokens": ignored_tokens})
        helper.append_op(type="sequence_erase", inputs={"X": [label]}, outputs={"Out": [el]},
                         attrs={"tokens": ignored_tokens})
        input, label = ei, el
    out = helper.create_variable_for_type_inference(dtype="float32", stop_gradient=True)
    num = helper.create_variable_for_type_inference(dtype="int64", stop_gradient=True)
    helper.append_op(type="edit_distance", inputs={"Hyps": [input], "Refs": [label]},
                     outputs={"Out": [out], "SequenceNum": [num]}, attrs={"normalized": normalized})
    return out, num


def nce(input, label, num_total_classes, sample_weight=None, param_attr=None, bias_attr=None, num_neg_samples=None):
    helper = LayerHelper("nce", **locals())
    dim = input.shape[1]
    w = helper.create_parameter(attr=helper.param_attr, shape=[num_total_classes, dim], dtype=input.dtype)
    b = helper.create_parameter(attr=helper.bias_attr, shape=[num_total_classes, 1], dtype=input.dtype,
                                is_bias=True)
    num_neg_samples = 10 if num_neg_samples is None else int(num_neg_samples)
    cost = _tmp(helper, input.dtype)
    sl, slab = _tmp(helper, input.dtype, True), helper.create_variable_for_type_inference("int64", True)
    ins = {"Input": input, "Label": label, "Weight": w, "Bias": b}
    if sample_weight is not None:
        ins["SampleWeight"] = sample_weight
    helper.append_op(type="nce", inputs=ins, outputs={"Cost": cost, "SampleLogits": sl, "SampleLabels": slab},
                     attrs={"num_total_classes": int(num_total_classes), "num_neg_samples": num_neg_samples})
    return cost / (num_neg_samples + 1)


def hsigmoid(input, label, num_classes, param_attr=None, bias_attr=None):
    helper = LayerHelper("hierarchical_sigmoid", **locals())
    if num_classes < 2:
        raise ValueError("num_classes must not be less than 2.")
    dtype = helper.input_dtype()
    w = helper.create_parameter(attr=helper.param_attr, shape=[num_classes - 1, input.shape[1]], dtype=dtype)
    ins = {"X": input, "W": w, "Label": label}
    if helper.bias_attr:
        ins["Bias"] = helper.create_parameter(attr=helper.bias_attr, shape=[1, num_classes - 1], dtype=dtype,
                                              is_bias=True)
    out, pre = _tmp(helper, dtype), _tmp(helper, dtype, True)
    helper.append_op(type="hierarchical_sigmoid", inputs=ins, outputs={"Out": out, "PreOut": pre},
                     attrs={"num_classes": num_classes})
    return out


def beam_search(pre_ids, pre_scores, ids, scores, beam_size, end_id, level=0):
    helper = LayerHelper("beam_search", **locals())
    sid = helper.create_variable_for_type_inference(dtype="int64", stop_gradient=True)
    ssc = helper.create_variable_for_type_inference(dtype="float32", stop_gradient=True)
    helper.append_op(type="beam_search",
                     inputs={"pre_ids": pre_ids, "pre_scores": pre_scores, "ids": ids, "scores": scores},
                     outputs={"selected_ids": sid, "selected_scores": ssc},
                     attrs={"level": level, "beam_size": beam_size, "end_id": end_id})
    return sid, ssc


def beam_search_decode(ids, scores, beam_size, end_id, name=None):
    helper = LayerHelper("beam_search_decode", **locals())
    sid = helper.create_variable_for_type_inference(dtype="int64", stop_gradient=True)
    ssc = helper.create_variable_for_type_inference(dtype="float32", stop_gradient=True)
    helper.append_op(type="beam_search_decode", inputs={"Ids": ids, "Scores": scores},
                     outputs={"SentenceIds": sid, "SentenceScores": ssc},
                     attrs={"beam_size": beam_size, "end_id": end_id})
    return sid, ssc
