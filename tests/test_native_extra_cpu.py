"""ops_extra.hip and the transposed convolutions of ops_conv3d.hip on the C++
executor vs the interpreter: conv2d / depthwise / conv3d transpose (+grads), spp
(+grad, max and avg), fused_elemwise_activation in all four functor orders (+grads),
prior_box / anchor_generator, auc / precision_recall / positive_negative_pair,
fake_quantize_range_abs_max, bipartite_match + target_assign, host layer_norm (+grad),
ModelAverage's average_accumulates, reduce_*_grad, elementwise max / min / pow grads,
floordiv / mod, size, sequence_reverse / sequence_scatter (+grads), kldiv / bpr
losses (+grads), shuffle_channel / scale_sub_region (+grads) and lars_momentum;
3 steps, fetches to 1e-5, no Python fallback.  test_native_extra_gpu.py runs the same cases on a HIP place."""
import numpy as np
import pytest
import torch

import paddle_amd.fluid as fluid
from paddle_amd.fluid.layers.layer_utils import simple_op
from paddle_amd.framework import core

from native_control_cases import run

L = fluid.layers


def _head(x, n=6):
    return L.fc(x, n, bias_attr=False)


def _img(x, c, h, w):
    return L.reshape(_head(x, c * h * w), [-1, c, h, w])


def _sq(v):
    return L.mean(L.square(v))


def _sum(*vs):
    tot = vs[0]
    for v in vs[1:]:
        tot = L.elementwise_add(tot, v)
    return tot


def _convt(op, x, w, **attrs):
    a = {"strides": [1, 1], "paddings": [0, 0], "dilations": [1, 1], "groups": 1}
    a.update(attrs)
    return simple_op(op, {"Input": [x], "Filter": [w]}, a, out_slot="Output")


def case_conv2d_transpose(x, lab, idx):
    img = _img(x, 2, 3, 3)
    a = _convt("conv2d_transpose", img, L.create_parameter([2, 3, 2, 2], "float32"), strides=[2, 2],
               paddings=[1, 1])
    b = _convt("conv2d_transpose", img, L.create_parameter([2, 2, 3, 3], "float32"), paddings=[1, 1],
               dilations=[2, 2], groups=2)
    c = _convt("depthwise_conv2d_transpose", img, L.create_parameter([2, 1, 2, 2], "float32"), strides=[2, 1],
               groups=2)
    return _sum(_sq(a), _sq(b), _sq(c))


def case_conv3d_transpose(x, lab, idx):
    vol = L.reshape(_head(x, 16), [-1, 2, 2, 2, 2])
    w = L.create_parameter([2, 2, 2, 2, 2], "float32")
    y = _convt("conv3d_transpose", vol, w, strides=[2, 1, 1], paddings=[0, 1, 0], dilations=[1, 1, 1])
    return _sq(y)


def case_spp(x, lab, idx):
    img = _img(x, 2, 4, 4)
    m = simple_op("spp", {"X": [img]}, {"pyramid_height": 3, "pooling_type": "max"})
    a = simple_op("spp", {"X": [img]}, {"pyramid_height": 2, "pooling_type": "avg"})
    odd = simple_op("spp", {"X": [_img(x, 1, 3, 5)]}, {"pyramid_height": 2, "pooling_type": "max"})
    return _sum(_sq(m), _sq(a), _sq(odd))


def _fused(x, y, fl, **attrs):
    a = {"functor_list": fl, "axis": -1, "scale": 0.0, "save_intermediate_out": True}
    a.update(attrs)
    out, _ = simple_op("fused_elemwise_activation", {"X": [x], "Y": [y]}, a, extra_outputs=("IntermediateOut",))
    return out


def case_fused_elemwise_activation(x, lab, idx):
    h = _head(x)
    yb = L.create_parameter([6], "float32")
    a = _fused(h, _head(x), ["elementwise_add", "relu"])
    b = _fused(h, yb, ["elementwise_mul", "scale"], scale=0.7)
    c = _fused(h, _head(x), ["relu", "elementwise_add"])
    d = _fused(L.reshape(_head(x, 12), [-1, 3, 4]), L.create_parameter([3], "float32"),
               ["scale", "elementwise_mul"], scale=-1.5, axis=1)
    return _sum(_sq(a), _sq(b), _sq(c), _sq(d))


def case_priors(x, lab, idx):
    h = _head(x)
    feat = L.reshape(_head(x, 12), [-1, 2, 3, 2])
    image = L.reshape(_head(x, 48), [-1, 1, 8, 6])
    pb, pv = simple_op("prior_box", {"Input": [feat], "Image": [image]},
                       {"min_sizes": [2.0, 4.0], "max_sizes": [5.0, 7.0], "aspect_ratios": [2.0, 3.0],
                        "variances": [0.1, 0.1, 0.2, 0.2], "flip": True, "clip": True, "step_w": 0.0, "step_h": 0.0,
                        "offset": 0.5, "min_max_aspect_ratios_order": False},
                       out_slot="Boxes", extra_outputs=("Variances",), stop_gradient=True)
    qb, _ = simple_op("prior_box", {"Input": [feat], "Image": [image]},
                      {"min_sizes": [3.0], "max_sizes": [6.0], "aspect_ratios": [0.5], "variances": [0.1, 0.2, 0.3, 0.4],
                       "flip": False, "clip": False, "step_w": 3.0, "step_h": 2.5, "offset": 0.25,
                       "min_max_aspect_ratios_order": True},
                      out_slot="Boxes", extra_outputs=("Variances",), stop_gradient=True)
    an, av = simple_op("anchor_generator", {"Input": [feat]},
                       {"anchor_sizes": [8.0, 16.0], "aspect_ratios": [0.5, 1.0, 2.0],
                        "variances": [0.1, 0.1, 0.2, 0.2], "stride": [4.0, 6.0], "offset": 0.5},
                       out_slot="Anchors", extra_outputs=("Variances",), stop_gradient=True)
    extra = _sum(L.mean(pb), L.mean(pv), L.mean(qb), L.scale(L.mean(an), 0.01), L.mean(av))
    return L.elementwise_add(_sq(h), extra)


def case_metrics(x, lab, idx):
    h = _head(x)
    prob = L.softmax(_head(x, 2))
    bin_lab = L.cast(L.greater_than(L.slice(lab, axes=[1], starts=[0], ends=[1]), L.fill_constant([1], "float32", 0.0)),
                     "int64")
    outs = simple_op("auc", {"Predict": [prob], "Label": [bin_lab]}, {"curve": "ROC", "num_thresholds": 50},
                     out_slot="AUC", dtype="float64", extra_outputs=("TPOut", "FPOut", "TNOut", "FNOut"),
                     stop_gradient=True)
    pr_auc = simple_op("auc", {"Predict": [prob], "Label": [bin_lab]}, {"curve": "PR", "num_thresholds": 20},
                       out_slot="AUC", dtype="float64", extra_outputs=("TPOut", "FPOut", "TNOut", "FNOut"),
                       stop_gradient=True)[0]
    pred = L.argmax(_head(x, 4), axis=1)
    probs = L.reduce_max(L.softmax(_head(x, 4)), dim=1)
    bm, am, st = simple_op("precision_recall", {"MaxProbs": [probs], "Indices": [pred], "Labels": [idx]},
                           {"class_number": 4}, out_slot="BatchMetrics", extra_outputs=("AccumMetrics", "AccumStatesInfo"),
                           stop_gradient=True)
    score = _head(x, 2)
    pp, npair, neu = simple_op("positive_negative_pair",
                               {"Score": [score], "Label": [L.slice(lab, axes=[1], starts=[1], ends=[2])],
                                "QueryID": [L.cast(L.greater_than(L.cast(idx, "float32"),
                                                                  L.fill_constant([1], "float32", 1.0)), "int64")]},
                               {"column": 1}, out_slot="PositivePair", extra_outputs=("NegativePair", "NeutralPair"),
                               stop_gradient=True)
    q, s = simple_op("fake_quantize_range_abs_max", {"X": [h], "InScale": [L.fill_constant([1], "float32", 0.5)]},
                     {"bit_length": 8, "window_size": 4, "is_test": False}, extra_outputs=("OutScale",),
                     stop_gradient=True)
    extra = _sum(L.cast(outs[0], "float32"), L.cast(pr_auc, "float32"), L.mean(bm), L.mean(am), L.mean(st),
                 pp, npair, neu, L.scale(L.mean(q), 0.001), s)
    return L.elementwise_add(_sq(h), extra)


def case_match_assign(x, lab, idx):
    h = _head(x)
    dist = L.abs(_head(x, 6))
    dist.stop_gradient = True
    mi, md = simple_op("bipartite_match", {"DistMat": [dist]}, {"match_type": "bipartite", "dist_threshold": 0.5},
                       out_slot="ColToRowMatchIndices", dtype="int32", extra_outputs=("ColToRowMatchDist",),
                       stop_gradient=True)
    pi, pd = simple_op("bipartite_match", {"DistMat": [dist]}, {"match_type": "per_prediction",
                                                                 "dist_threshold": 0.1},
                       out_slot="ColToRowMatchIndices", dtype="int32", extra_outputs=("ColToRowMatchDist",),
                       stop_gradient=True)
    tgt = _head(x, 3)
    tgt.stop_gradient = True
    out, w = simple_op("target_assign", {"X": [tgt], "MatchIndices": [pi]}, {"mismatch_value": 2},
                       extra_outputs=("OutWeight",), stop_gradient=True)
    extra = _sum(L.mean(md), L.mean(pd), L.mean(L.cast(mi, "float32")), L.mean(out), L.mean(w))
    return L.elementwise_add(_sq(h), extra)


def case_layer_norm(x, lab, idx):
    a = L.layer_norm(L.reshape(_head(x, 12), [-1, 3, 4]), begin_norm_axis=1)
    b = L.layer_norm(L.reshape(_head(x, 12), [-1, 3, 4]), begin_norm_axis=2, scale=False)
    return L.elementwise_add(_sq(L.elementwise_mul(L.reshape(a, [-1, 12]), _head(x, 12))), L.mean(L.exp(b)))


def case_reduce_grads(x, lab, idx):
    h = L.reshape(_head(x, 12), [-1, 3, 4])
    a = L.reduce_sum(h, dim=[1])
    b = L.reduce_mean(h, dim=[-1], keep_dim=True)
    c = L.reduce_max(h, dim=[1, 2])
    d = L.reduce_min(h)
    e = L.reduce_prod(L.elementwise_add(L.scale(h, 0.1), L.fill_constant([1], "float32", 1.0)), dim=[2])
    return _sum(_sq(a), _sq(b), _sq(c), d, _sq(e))


def case_ew_max_min_pow(x, lab, idx):
    h = _head(x)
    w = L.create_parameter([6], "float32")
    a = simple_op("elementwise_max", {"X": [h], "Y": [w]}, {"axis": -1})
    b = simple_op("elementwise_min", {"X": [h], "Y": [L.elementwise_add(_head(x), lab)]}, {"axis": -1})
    base = L.exp(L.scale(_head(x), 0.3))
    c = simple_op("elementwise_pow", {"X": [base], "Y": [L.create_parameter([6], "float32")]}, {"axis": -1})
    return _sum(_sq(a), _sq(b), L.mean(c))


def case_floordiv_mod(x, lab, idx):
    h = _head(x)
    two = L.fill_constant([1], "int64", 2)
    neg = L.fill_constant([1], "int64", -3)
    fi = simple_op("elementwise_floordiv", {"X": [idx], "Y": [neg]}, {"axis": -1}, dtype="int64", stop_gradient=True)
    mi = simple_op("elementwise_mod", {"X": [L.elementwise_sub(idx, two)], "Y": [neg]}, {"axis": -1}, dtype="int64",
                   stop_gradient=True)
    ff = simple_op("elementwise_floordiv", {"X": [lab], "Y": [L.fill_constant([1], "float32", 0.7)]}, {"axis": -1},
                   stop_gradient=True)
    mf = simple_op("elementwise_mod", {"X": [lab], "Y": [L.fill_constant([1], "float32", -0.6)]}, {"axis": -1},
                   stop_gradient=True)
    sz = simple_op("size", {"Input": [h]}, {}, dtype="int64", stop_gradient=True)
    extra = _sum(L.mean(L.cast(fi, "float32")), L.mean(L.cast(mi, "float32")), L.mean(ff), L.mean(mf),
                 L.scale(L.cast(sz, "float32"), 0.01))
    return L.elementwise_add(_sq(h), extra)


def case_seq_reverse_scatter(x, lab, idx):
    h = L.lod_reset(_head(x), target_lod=[0, 1, 4])
    rv = simple_op("sequence_reverse", {"X": [h]}, {}, out_slot="Y")
    tbl = L.reshape(_head(x, 3), [2, 6])
    ids = L.lod_reset(idx, target_lod=[0, 2, 4])
    ids.stop_gradient = True
    up = L.lod_reset(_head(x, 1), target_lod=[0, 2, 4])
    sc = simple_op("sequence_scatter", {"X": [tbl], "Ids": [ids], "Updates": [up]}, {})
    return L.elementwise_add(_sq(L.elementwise_mul(rv, lab)), _sq(sc))


def case_kldiv_bpr(x, lab, idx):
    h = _head(x)
    t = L.softmax(lab)
    outs = [simple_op("kldiv_loss", {"X": [h], "Target": [t]}, {"reduction": red}, out_slot="Loss")
            for red in ("mean", "sum", "batchmean")]
    none = simple_op("kldiv_loss", {"X": [h], "Target": [t]}, {"reduction": "none"}, out_slot="Loss")
    bpr = simple_op("bpr_loss", {"X": [_head(x)], "Label": [idx]}, {}, out_slot="Y")
    return _sum(outs[0], L.scale(outs[1], 0.1), outs[2], _sq(none), L.mean(bpr))


def case_shuffle_scale_sub(x, lab, idx):
    img = _img(x, 4, 3, 2)
    sh = simple_op("shuffle_channel", {"X": [img]}, {"group": 2})
    box = simple_op("assign_value", {}, {"shape": [4, 6], "dtype": 2,
                                         "int32_values": [1, 2, 1, 3, 1, 1, 2, 4, 2, 2, 1, 2,
                                                          1, 1, 1, 1, 2, 2, 3, 4, 1, 3, 1, 2]},
                    dtype="int32", stop_gradient=True)
    ss = simple_op("scale_sub_region", {"X": [sh], "Indices": [box]}, {"value": -2.5})
    return _sq(L.elementwise_mul(ss, _img(x, 4, 3, 2)))


def case_pool3d_index(x, lab, idx):
    vol = L.reshape(_head(x, 2 * 4 * 4 * 2), [-1, 2, 4, 4, 2])
    a, _ = simple_op("max_pool3d_with_index", {"X": [vol]}, {"ksize": [2, 2, 2], "strides": [2, 2, 2],
                                                              "paddings": [0, 0, 0], "global_pooling": False},
                     extra_outputs=("Mask",))
    b, _ = simple_op("max_pool3d_with_index", {"X": [vol]}, {"ksize": [3, 2, 2], "strides": [1, 2, 1],
                                                              "paddings": [1, 0, 1], "global_pooling": False},
                     extra_outputs=("Mask",))
    return L.elementwise_add(_sq(a), _sq(b))


def _tags(vals, lod):
    t = simple_op("assign_value", {}, {"shape": [len(vals), 1], "dtype": 2, "int32_values": vals}, dtype="int32",
                  stop_gradient=True)
    return L.lod_reset(t, target_lod=lod)


def case_chunk_eval(x, lab, idx):
    h = _head(x)
    lod = [0, 4, 9, 12]
    inf = _tags([0, 1, 4, 2, 3, 3, 0, 1, 1, 4, 0, 2], lod)
    gold = _tags([0, 1, 4, 2, 2, 3, 0, 1, 4, 4, 0, 1], lod)
    outs = simple_op("chunk_eval", {"Inference": [inf], "Label": [gold]},
                     {"num_chunk_types": 2, "chunk_scheme": "IOB", "excluded_chunk_types": []}, out_slot="Precision",
                     extra_outputs=("Recall", "F1-Score", "NumInferChunks", "NumLabelChunks", "NumCorrectChunks"),
                     stop_gradient=True)
    inf2 = _tags([0, 1, 2, 8, 3, 4, 5, 6, 7, 8, 4, 6], lod)
    gold2 = _tags([0, 1, 2, 8, 3, 4, 6, 6, 7, 8, 4, 7], lod)
    outs2 = simple_op("chunk_eval", {"Inference": [inf2], "Label": [gold2]},
                      {"num_chunk_types": 2, "chunk_scheme": "IOBES", "excluded_chunk_types": [1]},
                      out_slot="Precision",
                      extra_outputs=("Recall", "F1-Score", "NumInferChunks", "NumLabelChunks", "NumCorrectChunks"),
                      stop_gradient=True)
    extra = _sum(*[L.cast(o, "float32") for o in list(outs) + list(outs2)])
    return L.elementwise_add(_sq(h), extra)


def case_nms_mining(x, lab, idx):
    h = _head(x)
    corner = L.reshape(_head(x, 12), [-1, 3, 4])
    lo = L.slice(corner, axes=[2], starts=[0], ends=[2])
    boxes = L.concat([lo, L.elementwise_add(lo, L.exp(L.slice(corner, axes=[2], starts=[2], ends=[4])))], axis=2)
    boxes.stop_gradient = True
    scores = L.sigmoid(L.reshape(_head(x, 9), [-1, 3, 3]))
    scores.stop_gradient = True
    nms = simple_op("multiclass_nms", {"BBoxes": [boxes], "Scores": [scores]},
                    {"background_label": 0, "score_threshold": 0.3, "nms_top_k": 2, "nms_threshold": 0.4,
                     "nms_eta": 1.0, "keep_top_k": 3, "normalized": False}, stop_gradient=True)
    cls = L.abs(_head(x, 6))
    cls.stop_gradient = True
    match = simple_op("assign_value", {}, {"shape": [4, 6], "dtype": 2,
                                           "int32_values": [0, -1, -1, 1, -1, -1, -1, -1, -1, -1, -1, 2,
                                                            1, 0, -1, -1, -1, -1, -1, 3, -1, -1, 0, -1]},
                      dtype="int32", stop_gradient=True)
    dist = L.scale(L.sigmoid(_head(x, 6)), 0.8)
    dist.stop_gradient = True
    neg, upd = simple_op("mine_hard_examples", {"ClsLoss": [cls], "MatchIndices": [match], "MatchDist": [dist]},
                         {"neg_pos_ratio": 2.0, "neg_dist_threshold": 0.5, "sample_size": 0,
                          "mining_type": "max_negative"}, out_slot="NegIndices", dtype="int32",
                         extra_outputs=("UpdatedMatchIndices",), stop_gradient=True)
    hneg, hupd = simple_op("mine_hard_examples", {"ClsLoss": [cls], "LocLoss": [L.abs(_head(x, 6))],
                                                  "MatchIndices": [match], "MatchDist": [dist]},
                           {"neg_pos_ratio": 1.0, "neg_dist_threshold": 0.5, "sample_size": 3,
                            "mining_type": "hard_example"}, out_slot="NegIndices", dtype="int32",
                           extra_outputs=("UpdatedMatchIndices",), stop_gradient=True)
    extra = _sum(L.mean(nms), *[L.mean(L.cast(t, "float32")) for t in (neg, upd, hneg, hupd)])
    return L.elementwise_add(_sq(h), extra)


def _fconst(vals, shape, lod):
    t = simple_op("assign_value", {}, {"shape": shape, "dtype": 5, "fp32_values": vals}, dtype="float32",
                  stop_gradient=True)
    return L.lod_reset(t, target_lod=lod)


def case_detection_map(x, lab, idx):
    h = _head(x)
    det = _fconst([1, 0.9, 0.1, 0.1, 0.5, 0.5, 1, 0.8, 0.12, 0.1, 0.5, 0.52, 2, 0.7, 0.5, 0.5, 0.9, 0.9,
                   2, 0.95, 0.0, 0.0, 0.3, 0.3, 1, 0.6, 0.55, 0.5, 0.9, 0.95, 2, 0.3, 0.1, 0.1, 0.2, 0.2],
                  [6, 6], [0, 3, 6])
    gt = _fconst([1, 0, 0.1, 0.1, 0.5, 0.5, 2, 1, 0.5, 0.5, 0.9, 0.9, 2, 0, 0.0, 0.0, 0.3, 0.3,
                  1, 0, 0.5, 0.5, 0.9, 0.9, 2, 0, 0.6, 0.6, 0.8, 0.8],
                 [5, 6], [0, 2, 5])
    outs = []
    for ap, diff in (("integral", True), ("11point", False)):
        m, pc, tp, fp = simple_op("detection_map", {"DetectRes": [det], "Label": [gt]},
                                  {"class_num": 3, "background_label": 0, "overlap_threshold": 0.5,
                                   "evaluate_difficult": diff, "ap_type": ap}, out_slot="MAP",
                                  extra_outputs=("AccumPosCount", "AccumTruePos", "AccumFalsePos"),
                                  stop_gradient=True)
        outs += [m, L.mean(L.cast(pc, "float32")), L.mean(tp), L.mean(fp)]
    return L.elementwise_add(_sq(h), _sum(*outs))


def case_generate_proposals(x, lab, idx):
    h = _head(x)
    sc = L.sigmoid(L.reshape(_head(x, 2 * 2 * 3), [-1, 2, 2, 3]))
    dl = L.scale(L.reshape(_head(x, 8 * 2 * 3), [-1, 8, 2, 3]), 0.3)
    feat = L.reshape(_head(x, 6), [-1, 1, 2, 3])
    anchors, var = simple_op("anchor_generator", {"Input": [feat]},
                             {"anchor_sizes": [8.0, 16.0], "aspect_ratios": [1.0], "variances": [1.0, 1.0, 1.0, 1.0],
                              "stride": [8.0, 8.0], "offset": 0.5}, out_slot="Anchors",
                             extra_outputs=("Variances",), stop_gradient=True)
    info = simple_op("assign_value", {}, {"shape": [4, 3], "dtype": 5,
                                          "fp32_values": [20.0, 28.0, 1.0, 24.0, 24.0, 0.5, 16.0, 30.0, 2.0,
                                                          30.0, 30.0, 1.0]}, dtype="float32", stop_gradient=True)
    for v in (sc, dl):
        v.stop_gradient = True
    rois, probs = simple_op("generate_proposals", {"Scores": [sc], "BboxDeltas": [dl], "ImInfo": [info],
                                                   "Anchors": [anchors], "Variances": [var]},
                            {"pre_nms_topN": 10, "post_nms_topN": 5, "nms_thresh": 0.6, "min_size": 2.0, "eta": 1.0},
                            out_slot="RpnRois", extra_outputs=("RpnRoiProbs",), stop_gradient=True)
    return L.elementwise_add(_sq(h), L.elementwise_add(L.scale(L.mean(rois), 0.01), L.mean(probs)))


CASES = {k[5:]: v for k, v in globals().items() if k.startswith("case_")}


def net(case):
    def build():
        x = L.data(name="x", shape=[5], dtype="float32")
        lab = L.data(name="lab", shape=[6], dtype="float32")
        idx = L.data(name="idx", shape=[1], dtype="int64")
        loss = CASES[case](x, lab, idx)
        fluid.optimizer.SGD(learning_rate=0.1).minimize(loss)
        return [loss]
    return build


def model_average_net():
    """SGD + ModelAverage: average_accumulates over every parameter, window rolled
    within the 3 steps (min / max window 2)."""
    def build():
        x = L.data(name="x", shape=[5], dtype="float32")
        lab = L.data(name="lab", shape=[6], dtype="float32")
        L.data(name="idx", shape=[1], dtype="int64")
        loss = L.mean(L.square(L.elementwise_sub(L.fc(x, 6), lab)))
        fluid.optimizer.SGD(learning_rate=0.1).minimize(loss)
        ma = fluid.optimizer.ModelAverage(0.5, min_average_window=2, max_average_window=2)
        fetch = [loss]
        for p, _ in ma.params_grads:
            fetch += [ma._get_accumulator(k, p) for k in ("sum_1", "sum_2", "sum_3", "num_accumulates",
                                                           "old_num_accumulates", "num_updates")]
        return fetch
    return build


def feeds(steps=3):
    out = []
    for s in range(steps):
        rs = np.random.RandomState(80 + s)
        out.append({"x": core.LoDTensor(torch.from_numpy(rs.randn(4, 5).astype("float32"))),
                    "lab": core.LoDTensor(torch.from_numpy(rs.randn(4, 6).astype("float32"))),
                    "idx": core.LoDTensor(torch.from_numpy(np.array([[2], [0], [3], [2]], dtype="int64")))})
    return out


def lars_net():
    """fc + square loss; every parameter updated by lars_momentum."""
    def build():
        x = L.data(name="x", shape=[5], dtype="float32")
        lab = L.data(name="lab", shape=[6], dtype="float32")
        L.data(name="idx", shape=[1], dtype="int64")
        loss = L.mean(L.square(L.elementwise_sub(L.fc(x, 6), lab)))
        pg = fluid.backward.append_backward(loss)
        lr = L.fill_constant([1], "float32", 0.5)
        blk = fluid.default_main_program().global_block()
        for p, g in pg:
            v = L.create_global_var(shape=list(p.shape), value=0.05, dtype="float32", persistable=True)
            blk.append_op(type="lars_momentum", inputs={"Param": [p], "Grad": [g], "Velocity": [v],
                                                         "LearningRate": [lr]},
                          outputs={"ParamOut": [p], "VelocityOut": [v]},
                          attrs={"mu": 0.8, "lars_coeff": 0.01, "lars_weight_decay": 0.001})
        return [loss]
    return build


BUILDS = dict({k: net(k) for k in CASES}, model_average=model_average_net(), lars_momentum=lars_net())


def check(case, place, rtol, atol):
    fd = feeds()
    ref, init, _ = run(BUILDS[case], fd, "python", place)
    got, _, exe = run(BUILDS[case], fd, "native", place, init)
    for a, b in zip(ref, got):
        for u, v in zip(a, b):
            np.testing.assert_allclose(v, u, rtol=rtol, atol=atol)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    return exe


@pytest.mark.parametrize("case", sorted(BUILDS))
def test_extra_op_native_host(case):
    check(case, fluid.CPUPlace(), 1e-5, 1e-6)


def test_batch_size_like_random_native():
    """uniform / gaussian_random_batch_size_like: the batch dim comes from Input, the
    values from the executor's RNG (range / moments only, the engines' RNGs differ)."""
    def build():
        x = L.data(name="x", shape=[5], dtype="float32")
        u = L.uniform_random_batch_size_like(x, [-1, 300], min=-2.0, max=3.0)
        g = simple_op("gaussian_random_batch_size_like", {"Input": [x]},
                      {"shape": [7, -1, 200], "mean": 1.0, "std": 0.5, "seed": 3, "dtype": 5, "input_dim_idx": 0,
                       "output_dim_idx": 1}, stop_gradient=True)
        return [u, g]
    fd = [{"x": core.LoDTensor(torch.zeros(4, 5))}]
    got, _, exe = run(build, fd, "native", fluid.CPUPlace())
    u, g = got[0]
    assert u.shape == (4, 300) and g.shape == (7, 4, 200)
    assert u.min() >= -2.0 and u.max() <= 3.0 and abs(u.mean() - 0.5) < 0.1
    assert abs(g.mean() - 1.0) < 0.05 and abs(g.std() - 0.5) < 0.05
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_dropout_grad_native_host():
    """host dropout + dropout_grad: Mask is 0 / 1, the upscale factor applies to Out
    and to X@GRAD (X@GRAD == Out@GRAD * Out / X elementwise)."""
    def build():
        x = L.data(name="x", shape=[50], dtype="float32")
        x.stop_gradient = False
        y = L.dropout(x, 0.3, dropout_implementation="upscale_in_train")
        loss = L.reduce_sum(L.elementwise_mul(y, L.fill_constant([50], "float32", 2.0)))
        fluid.backward.append_backward(loss)
        return [y, "x@GRAD"]
    xv = np.random.RandomState(0).rand(8, 50).astype("float32") + 0.5
    got, _, exe = run(build, [{"x": core.LoDTensor(torch.from_numpy(xv))}], "native", fluid.CPUPlace())
    y, gx = got[0]
    keep = y != 0
    np.testing.assert_allclose(y[keep], xv[keep] / 0.7, rtol=1e-6)
    np.testing.assert_allclose(gx, np.where(keep, 2.0 / 0.7, 0.0), rtol=1e-6)
    assert 0.5 < keep.mean() < 0.9
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_sampling_crop_print_native(capfd):
    """sampling_id (a valid column per row, biased to the heavy one), random_crop (a
    window of X), print (the message on stdout, Out sharing In) on the C++ executor."""
    def build():
        p = L.data(name="p", shape=[4], dtype="float32")
        v = L.data(name="v", shape=[3, 5], dtype="float32")
        ids = simple_op("sampling_id", {"X": [p]}, {"min": 0.0, "max": 1.0, "seed": 5}, dtype="int64",
                        stop_gradient=True)
        seed = L.fill_constant([1], "int64", 7)
        crop, _ = simple_op("random_crop", {"X": [v], "Seed": [seed]}, {"shape": [2, 3], "startup_seed": 0},
                            extra_outputs=("SeedOut",), stop_gradient=True)
        shown = simple_op("print", {"In": [crop]}, {"message": "crop-native", "summarize": 4}, stop_gradient=True)
        return [ids, crop, shown]
    probs = np.tile(np.array([[0.05, 0.05, 0.85, 0.05]], "float32"), (400, 1))
    vol = np.arange(8 * 15, dtype="float32").reshape(8, 3, 5)
    got, _, exe = run(build, [{"p": core.LoDTensor(torch.from_numpy(probs)),
                               "v": core.LoDTensor(torch.from_numpy(vol))}], "native", fluid.CPUPlace())
    ids, crop, shown = got[0]
    assert ids.shape == (400,) and ids.min() >= 0 and ids.max() <= 3 and (ids == 2).mean() > 0.75
    assert crop.shape == (8, 2, 3)
    r0, c0 = divmod(int(crop[0, 0, 0]) % 15, 5)
    np.testing.assert_array_equal(crop, vol[:, r0:r0 + 2, c0:c0 + 3])
    np.testing.assert_array_equal(shown, crop)
    assert "crop-native" in capfd.readouterr().out
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def fusion_rnn_build():
    """fusion_lstm / fusion_gru (inference ops: XX = X WeightX, then the recurrence) and
    fusion_seqexpand_concat_fc, attention_lstm."""
    x = L.data(name="xs", shape=[5], dtype="float32", lod_level=1)
    D = 3
    cp = lambda shape: L.create_parameter(shape, "float32")  # noqa: E731
    h, c, _ = simple_op("fusion_lstm", {"X": [x], "WeightX": [cp([5, 4 * D])], "WeightH": [cp([D, 4 * D])],
                                        "Bias": [cp([1, 4 * D])]},
                        {"use_peepholes": False, "is_reverse": False, "gate_activation": "sigmoid",
                         "cell_activation": "tanh", "candidate_activation": "tanh", "use_seq": True},
                        out_slot="Hidden", extra_outputs=("Cell", "XX"), stop_gradient=True)
    g, _ = simple_op("fusion_gru", {"X": [x], "WeightX": [cp([5, 3 * D])], "WeightH": [cp([D, 3 * D])],
                                    "Bias": [cp([1, 3 * D])]},
                     {"activation": "tanh", "gate_activation": "sigmoid", "is_reverse": True, "use_seq": True},
                     out_slot="Hidden", extra_outputs=("XX",), stop_gradient=True)
    y = L.data(name="ys", shape=[2], dtype="float32")
    fo, _ = simple_op("fusion_seqexpand_concat_fc", {"X": [x, y], "FCWeight": [cp([7, 4])], "FCBias": [cp([4])]},
                      {"fc_activation": "tanh"}, extra_outputs=("FCOut",), stop_gradient=True)
    c0 = L.data(name="c0", shape=[D], dtype="float32")
    ah, ac, _, _, _, _ = simple_op(
        "attention_lstm", {"X": [x], "C0": [c0], "AttentionWeight": [cp([5 + D, 1])], "AttentionBias": [cp([1, 1])],
                           "AttentionScalar": [cp([1, 1])], "AttentionScalarBias": [cp([1, 1])],
                           "LSTMWeight": [cp([D + 5, 4 * D])], "LSTMBias": [cp([1, 4 * D])]},
        {"gate_activation": "sigmoid", "cell_activation": "tanh", "candidate_activation": "tanh"},
        out_slot="Hidden", extra_outputs=("Cell", "AttentionedX", "AttentionFCOut", "LSTMX", "LSTMOUT"),
        stop_gradient=True)
    return [h, c, g, fo, ah, ac]


def fusion_feeds():
    rs = np.random.RandomState(3)
    t = core.LoDTensor(torch.from_numpy(rs.randn(9, 5).astype("float32")))
    t.set_lod([[0, 3, 5, 9]])
    return [{"xs": t, "ys": core.LoDTensor(torch.from_numpy(rs.randn(3, 2).astype("float32"))),
             "c0": core.LoDTensor(torch.from_numpy(rs.randn(3, 3).astype("float32")))}]


def test_fusion_rnn_native_host():
    ref, init, _ = run(fusion_rnn_build, fusion_feeds(), "python", fluid.CPUPlace())
    got, _, exe = run(fusion_rnn_build, fusion_feeds(), "native", fluid.CPUPlace(), init)
    for u, v in zip(ref[0], got[0]):
        np.testing.assert_allclose(v, u, rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
