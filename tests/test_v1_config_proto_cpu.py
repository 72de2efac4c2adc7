"""The v1 config parser's ModelConfig / TrainerConfig output
(trainer_config_helpers/config_proto.py) against the reference's own expected
outputs: python/paddle/trainer_config_helpers/tests/configs/protostr/*.protostr
(text-format ModelConfig files, read as data).  Each config below builds the
topology of the reference test config of the same name; the layer names, types,
sizes, activations, inputs, parameter names / sizes / dims and input / output
layer names must match.  Also: proto2 wire round trip of a whole TrainerConfig."""
import os

import pytest

import paddle_amd.trainer_config_helpers as tch
from paddle_amd.trainer_config_helpers import config_proto as cp

PROTOSTR = "/root/reference/python/paddle/trainer_config_helpers/tests/configs/protostr"


def _fc():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    din = tch.data_layer(name="data", size=100)
    trans = tch.trans_layer(input=din)
    hidden = tch.fc_layer(input=trans, size=100, bias_attr=False)
    mask = tch.data_layer(name="mask", size=100)
    sel = tch.selective_fc_layer(input=din, select=mask, size=100, act=tch.SigmoidActivation())
    tch.outputs(hidden, sel)


def _activations():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    din = tch.data_layer(name="input", size=100)
    acts = [tch.TanhActivation, tch.SigmoidActivation, tch.SoftmaxActivation, tch.IdentityActivation,
            tch.LinearActivation, tch.ExpActivation, tch.ReluActivation, tch.BReluActivation,
            tch.SoftReluActivation, tch.STanhActivation, tch.AbsActivation, tch.SquareActivation]
    tch.outputs([tch.fc_layer(input=din, size=100, act=a(), name="layer_%d" % i) for i, a in enumerate(acts)])


def _util():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    a = tch.data_layer(name="a", size=10)
    b = tch.data_layer(name="b", size=10)
    r = tch.addto_layer(input=[a, b])
    c1 = tch.concat_layer(input=[a, b])
    c2 = tch.concat_layer(input=[tch.identity_projection(input=a), tch.identity_projection(input=b)])
    tch.outputs(r, c1, c2)


def _last_first_seq():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    din = tch.data_layer(name="data", size=30)
    outs = []
    for op in (tch.first_seq, tch.last_seq):
        for al in (tch.AggregateLevel.TO_SEQUENCE, tch.AggregateLevel.TO_NO_SEQUENCE):
            outs.append(op(input=din, agg_level=al))
    for op in (tch.first_seq, tch.last_seq):
        outs.append(op(input=din, agg_level=tch.AggregateLevel.TO_NO_SEQUENCE, stride=5))
    tch.outputs(outs)


def _l2_distance():
    tch.outputs(tch.l2_distance_layer(x=tch.data_layer(name="x", size=128), y=tch.data_layer(name="y", size=128)))


def _repeat():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    din = tch.data_layer(name="data", size=30)
    tch.outputs(tch.repeat_layer(input=din, num_repeats=10, as_row_vector=True),
                tch.repeat_layer(input=din, num_repeats=10, act=tch.TanhActivation(), as_row_vector=False))


def _clip():
    tch.outputs(tch.clip_layer(input=tch.data_layer(name="input", size=300), min=-10, max=10))


def _dot_prod():
    v1 = tch.data_layer(name="vector1", size=10)
    v2 = tch.data_layer(name="vector2", size=10)
    tch.outputs(tch.dot_prod_layer(input1=v1, input2=v2))


def _row_l2_norm():
    tch.outputs(tch.row_l2_norm_layer(input=tch.data_layer(name="input", size=300)))


def _fm():
    tch.outputs(tch.factorization_machine(input=tch.data_layer(name="data", size=1024), factor_size=10))


def _smooth_l1():
    tch.outputs(tch.smooth_l1_cost(input=tch.data_layer(name="input", size=300),
                                   label=tch.data_layer(name="label", size=300)))


def _hsigmoid():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    din = tch.data_layer(name="data", size=100)
    label = tch.data_layer(name="label", size=10)
    tch.outputs(tch.hsigmoid(input=din, label=label, num_classes=10))


def _row_conv():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    tch.outputs(tch.row_conv_layer(input=tch.data_layer(name="data", size=2560), context_len=19,
                                   act=tch.ReluActivation()))


def _scale_shift():
    din = tch.data_layer(name="data", size=100)
    tch.outputs(tch.scale_shift_layer(input=din, bias_attr=False), tch.scale_shift_layer(input=din))


def _prelu():
    din = tch.data_layer(name="input", size=300, height=10, width=10)
    tch.prelu_layer(input=din, num_channels=3)
    tch.prelu_layer(input=din, partial_sum=1, num_channels=3)
    tch.prelu_layer(input=din, partial_sum=5, num_channels=3)
    tch.prelu_layer(input=din, channel_shared=True, num_channels=3)
    tch.outputs(tch.prelu_layer(input=din, channel_shared=False, num_channels=3))


def _resize():
    tch.outputs(tch.resize_layer(input=tch.data_layer(name="input", size=300), size=150))


def _multiplex():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    index = tch.data_layer(name="index", size=1)
    ds = [tch.data_layer(name="data%d" % i, size=30) for i in (1, 2, 3)]
    tch.outputs(tch.multiplex_layer([index] + ds))


def _expand():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    din = tch.data_layer(name="data", size=30)
    seq = tch.data_layer(name="data_seq", size=30)
    tch.outputs(tch.expand_layer(input=din, expand_as=seq, expand_level=tch.ExpandLevel.FROM_SEQUENCE),
                tch.expand_layer(input=din, expand_as=seq, expand_level=tch.ExpandLevel.FROM_NO_SEQUENCE))


def _gated_unit():
    ex = tch.ExtraLayerAttribute(error_clipping_threshold=100.0)
    tch.outputs(tch.gated_unit_layer(size=512, input=tch.data_layer(name="input", size=256),
                                     act=tch.TanhActivation(), gate_attr=ex,
                                     gate_param_attr=tch.ParamAttr(initial_std=1e-4),
                                     gate_bias_attr=tch.ParamAttr(initial_std=1), inproj_attr=ex,
                                     inproj_param_attr=tch.ParamAttr(initial_std=1e-4),
                                     inproj_bias_attr=tch.ParamAttr(initial_std=1), layer_attr=ex))


def _seq_slice():
    seq = tch.data_layer("word", size=128)
    starts = tch.data_layer("starts", size=5)
    ends = tch.data_layer("ends", size=5)
    tch.outputs(tch.seq_slice_layer(input=seq, starts=starts, ends=ends),
                tch.seq_slice_layer(input=seq, starts=starts, ends=None),
                tch.seq_slice_layer(input=seq, starts=None, ends=ends))


def _kmax_seq_score():
    scores = tch.fc_layer(input=tch.data_layer(name="input_seq", size=128), size=1, act=tch.ExpActivation())
    tch.outputs(tch.kmax_seq_score_layer(input=scores, beam_size=5))


def _bi_gru():
    tch.settings(batch_size=1000, learning_rate=1e-4)
    tch.outputs(tch.bidirectional_gru(input=tch.data_layer(name="data", size=120), size=40, return_seq=True))


def _gru():
    tch.settings(batch_size=1000, learning_rate=1e-4)
    tch.outputs(tch.grumemory(input=tch.data_layer(name="data", size=120), size=40, reverse=True,
                              gate_act=tch.TanhActivation(), act=tch.SigmoidActivation()))


def _lstm():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    tch.outputs(tch.lstmemory(input=tch.data_layer(name="data", size=128), reverse=True,
                              gate_act=tch.TanhActivation(), act=tch.TanhActivation(), size=32))


def _cost_weight():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    data = tch.data_layer(name="input", size=300)
    lbl = tch.data_layer(name="label", size=1)
    wt = tch.data_layer(name="weight", size=1)
    fc = tch.fc_layer(input=data, size=10, act=tch.SoftmaxActivation())
    tch.outputs(tch.classification_cost(input=fc, label=lbl, weight=wt),
                tch.square_error_cost(input=fc, label=lbl, weight=wt),
                tch.nce_layer(input=fc, label=tch.data_layer(name="multi_class_label", size=500), weight=wt))


def _pad():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    data = tch.data_layer(name="data", size=2016, height=48, width=42)
    conv = tch.img_conv_layer(input=data, filter_size=3, num_channels=1, num_filters=16, padding=1,
                              act=tch.LinearActivation(), bias_attr=True)
    pool = tch.img_pool_layer(input=conv, pool_size=2, stride=2, pool_type=tch.MaxPooling())
    tch.outputs(tch.pad_layer(input=pool, pad_c=[2, 3], pad_h=[1, 2], pad_w=[3, 1]))


def _print():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    din = tch.data_layer(name="input", size=100)
    tch.print_layer(input=din)
    tch.outputs(din)


def _seq_concat_reshape():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    d1 = tch.data_layer(name="data1", size=30)
    d2 = tch.data_layer(name="data2", size=30)
    tch.outputs([tch.seq_concat_layer(a=d1, b=d2), tch.seq_reshape_layer(input=d1, reshape_size=5)])


def _spp():
    tch.settings(batch_size=100, learning_rate=1e-5)
    data = tch.data_layer(name="data", size=3200, height=20, width=10)
    tch.outputs(tch.spp_layer(input=data, pyramid_height=2, num_channels=16, pool_type=tch.MaxPooling()))


def _bn3d():
    tch.settings(batch_size=1000, learning_rate=1e-4)
    d = tch.data_layer(name="data3D", size=120 * 3, width=20, height=6, depth=3)
    tch.outputs(tch.batch_norm_layer(d, num_channels=1, img3D=True))


def _scale_sub_region():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    data = tch.data_layer(name="data", size=2016, height=48, width=42)
    indices = tch.data_layer(name="indices", size=6)
    tch.outputs(tch.scale_sub_region_layer(input=data, indices=indices, value=0.0))


def _unused():
    tch.settings(batch_size=1000, learning_rate=1e-4)
    tch.outputs(tch.sampling_id_layer(input=tch.data_layer(name="probs", size=100)))


def _sub_nested_seq():
    data = tch.data_layer(name="input_seq", size=300)
    sel = tch.data_layer(name="input", size=5)
    tch.outputs(tch.sub_nested_seq_layer(input=data, selected_indices=sel))


def _conv(inp, nc, nf, **kw):
    return tch.img_conv_layer(input=inp, filter_size=kw.pop("filter_size", 3), num_channels=nc, num_filters=nf,
                              padding=kw.pop("padding", 1), act=tch.LinearActivation(),
                              bias_attr=kw.pop("bias_attr", True), **kw)


def _maxout():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    data = tch.data_layer(name="data", size=2304, height=48, width=48)
    mo = tch.maxout_layer(input=_conv(data, 1, 16), num_channels=16, groups=2)
    pool = tch.img_pool_layer(input=mo, num_channels=8, pool_size=2, stride=2, pool_type=tch.MaxPooling())
    mo2 = tch.maxout_layer(input=_conv(pool, 8, 128), num_channels=128, groups=4)
    block = tch.block_expand_layer(input=mo2, num_channels=32, stride_x=1, stride_y=1, block_x=1, block_y=6)
    tch.outputs(tch.fc_layer(input=block, size=384, bias_attr=False))


def _bilinear():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    data = tch.data_layer(name="data", size=2304)
    bil = tch.bilinear_interp_layer(input=_conv(data, 1, 16), out_size_x=64, out_size_y=64)
    pool = tch.img_pool_layer(input=bil, num_channels=16, pool_size=2, stride=2, pool_type=tch.MaxPooling())
    tch.outputs(tch.fc_layer(input=pool, size=384, bias_attr=False))


def _img(trans):
    def f():
        tch.settings(learning_rate=1e-3, batch_size=1000)
        n = 227 if trans else 256
        img = tch.data_layer(name="image", size=n * n)
        kw = {"trans": True} if trans else {"dilation": (1, 1)}
        conv = tch.img_conv_layer(input=img, num_channels=1, num_filters=64, filter_size=(32, 32), padding=(1, 1),
                                  stride=(1, 1), act=tch.LinearActivation(), **kw)
        bn = tch.batch_norm_layer(input=conv, act=tch.ReluActivation())
        norm = tch.img_cmrnorm_layer(input=bn, size=32)
        pool = tch.img_pool_layer(input=conv, pool_size=32, pool_type=tch.MaxPooling())
        tch.outputs(pool, norm)
    return f


def _seq_pooling():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    din = tch.data_layer(name="dat_in", size=100)
    pts = [tch.MaxPooling, tch.AvgPooling, tch.SumPooling]
    opts = [tch.pooling_layer(input=din, agg_level=al, pooling_type=pt())
            for pt in pts for al in (tch.AggregateLevel.TO_SEQUENCE, tch.AggregateLevel.TO_NO_SEQUENCE)]
    opts += [tch.pooling_layer(input=din, agg_level=tch.AggregateLevel.TO_NO_SEQUENCE, pooling_type=pt(), stride=5)
             for pt in pts]
    opts.append(tch.pooling_layer(input=din, pooling_type=tch.MaxPooling(output_max_index=True)))
    tch.outputs(opts)


def _shared_fc():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    a = tch.data_layer(name="feature_a", size=200)
    b = tch.data_layer(name="feature_b", size=200)
    fc_p = tch.ParamAttr(name="fc_param", initial_max=1.0, initial_min=-1.0)
    b_p = tch.ParamAttr(name="bias_param", initial_mean=0.0, initial_std=0.0)
    sm_p = tch.ParamAttr(name="softmax_param", initial_max=1.0, initial_min=-1.0)
    ha = tch.fc_layer(input=a, size=200, param_attr=fc_p, bias_attr=b_p)
    hb = tch.fc_layer(input=b, size=200, param_attr=fc_p, bias_attr=b_p)
    pred = tch.fc_layer(input=[ha, hb], param_attr=[sm_p, sm_p], bias_attr=False, size=10,
                        act=tch.SoftmaxActivation())
    tch.outputs(tch.classification_cost(input=pred, label=tch.data_layer(name="label", size=10)))


def _roi_pool():
    data = tch.data_layer(name="data", size=3 * 14 * 14, height=14, width=14)
    rois = tch.data_layer(name="rois", size=10)
    tch.outputs(tch.roi_pool_layer(input=_conv(data, 3, 16), rois=rois, pooled_width=7, pooled_height=7,
                                   spatial_scale=1. / 16))


def _math_ops():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    lm = tch.layer_math
    x = tch.data_layer(name="data", size=100)
    for f in (lm.exp, lm.sqrt, lm.reciprocal, lm.log, lm.abs, lm.sigmoid, lm.tanh, lm.square, lm.relu):
        x = f(x)
    y = 1 + x
    y = y + 1
    y = x + y
    y = y - x
    y = y - 2
    y = 2 - y
    y = 2 * y
    y = y * 3
    z = tch.data_layer(name="data_2", size=1)
    y = y * z
    y = z * y
    y = y + z
    y = z + y
    tch.outputs(y)


def _cost_layers():
    tch.settings(learning_rate=1e-4, batch_size=1000)
    seq_in = tch.data_layer(name="input", size=200)
    labels = tch.data_layer(name="labels", size=5000)
    probs = tch.data_layer(name="probs", size=10)
    xe_label = tch.data_layer(name="xe-label", size=10)
    hidden = tch.fc_layer(input=seq_in, size=4)
    tch.outputs(
        tch.ctc_layer(input=seq_in, label=labels),
        tch.warp_ctc_layer(input=seq_in, label=labels, blank=0),
        tch.crf_layer(input=hidden, label=tch.data_layer(name="crf_label", size=4)),
        tch.rank_cost(left=tch.data_layer(name="left", size=1), right=tch.data_layer(name="right", size=1),
                      label=tch.data_layer(name="label", size=1)),
        tch.lambda_cost(input=tch.data_layer(name="list_feature", size=100),
                        score=tch.data_layer(name="list_scores", size=1)),
        tch.cross_entropy(input=probs, label=xe_label),
        tch.cross_entropy_with_selfnorm(input=probs, label=xe_label),
        tch.huber_regression_cost(input=seq_in, label=labels),
        tch.huber_classification_cost(input=tch.data_layer(name="huber_probs", size=1),
                                      label=tch.data_layer(name="huber_label", size=1)),
        tch.multi_binary_label_cross_entropy(input=probs, label=xe_label),
        tch.sum_cost(input=hidden),
        tch.nce_layer(input=hidden, label=labels))


def _recursive():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    enc = tch.data_layer(name="data", size=100)
    for _ in range(32):
        enc = tch.addto_layer([enc, enc])
    tch.outputs(tch.fc_layer(input=tch.fc_layer(input=enc, size=32, act=tch.ReluActivation()), size=10,
                             act=tch.SoftmaxActivation()))


def _split_ds():
    tch.define_py_data_sources2(train_list="train.list", test_list="test.list", module=["a", "b"], obj=("c", "d"))
    tch.settings(learning_rate=1e-3, batch_size=1000)
    tch.outputs(tch.data_layer(name="a", size=10))


def _ntm():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    w = tch.data_layer(name="w", size=1)
    a = tch.data_layer(name="a", size=100)
    b = tch.data_layer(name="b", size=100)
    c = tch.data_layer(name="c", size=200)
    d = tch.data_layer(name="d", size=31)
    tch.outputs(tch.interpolation_layer(input=[a, b], weight=w), tch.power_layer(input=a, weight=w),
                tch.scaling_layer(input=a, weight=w), tch.cos_sim(a=a, b=b), tch.cos_sim(a=a, b=c, size=2),
                tch.sum_to_one_norm_layer(input=a), tch.conv_shift_layer(a=a, b=d),
                tch.tensor_layer(a=a, b=b, size=1000), tch.slope_intercept_layer(input=a, slope=0.7, intercept=0.9),
                tch.linear_comb_layer(weights=b, vectors=c))


def _pool3d():
    tch.settings(batch_size=100, learning_rate=1e-5)
    d2 = tch.data_layer(name="data_2d", size=6000, height=20, width=10)
    tch.outputs(tch.img_pool_layer(name="pool___2d", input=d2, num_channels=30, pool_size=5, stride=3, padding=1,
                                   pool_type=tch.AvgPooling()))
    d3 = tch.data_layer(name="data_3d_1", size=60000, depth=10, height=20, width=10)
    tch.outputs(tch.img_pool3d_layer(name="pool_3d_1", input=d3, num_channels=30, pool_size=5, stride=3, padding=1,
                                     pool_type=tch.AvgPooling()))
    tch.outputs(tch.img_pool3d_layer(name="pool_3d_2", input=d3, num_channels=30, pool_size=[5, 5, 5],
                                     stride=[3, 3, 3], padding=[1, 1, 1], pool_type=tch.MaxPooling()))


def _conv3d(trans):
    def f():
        tch.settings(batch_size=1000, learning_rate=1e-5)
        data = tch.data_layer(name="data", size=12096 * 3, height=48, width=42, depth=6)
        pre = "deconv3d" if trans else "conv3d"
        kw = dict(input=data, num_filters=16, num_channels=3, groups=1, bias_attr=True, shared_biases=True,
                  trans=trans, layer_type=pre, act=tch.LinearActivation())
        tch.img_conv3d_layer(name=pre + "_1", filter_size=3, stride=2, padding=1, **kw)
        tch.outputs(tch.img_conv3d_layer(name=pre + "_2", filter_size=[3, 3, 3], stride=[2, 2, 2],
                                         padding=[1, 1, 1], **kw))
    return f


def _multibox():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    loc = tch.data_layer(name="input_loc", size=16, height=16, width=1)
    conf = tch.data_layer(name="input_conf", size=8, height=1, width=8)
    prior = tch.data_layer(name="priorbox", size=32, height=4, width=8)
    label = tch.data_layer(name="label", size=24, height=4, width=6)
    tch.outputs(tch.multibox_loss_layer(input_loc=loc, input_conf=conf, priorbox=prior, label=label, num_classes=21,
                                        overlap_threshold=0.5, neg_pos_ratio=3.0, neg_overlap=0.5, background_id=0,
                                        name="test_multibox_loss"))


def _detection_output():
    tch.settings(batch_size=1000, learning_rate=1e-5)
    loc = tch.data_layer(name="input_loc", size=16, height=16, width=1)
    conf = tch.data_layer(name="input_conf", size=8, height=1, width=8)
    prior = tch.data_layer(name="priorbox", size=32, height=4, width=8)
    tch.outputs(tch.detection_output_layer(input_loc=loc, input_conf=conf, priorbox=prior, num_classes=21,
                                           nms_threshold=0.45, nms_top_k=400, keep_top_k=200,
                                           confidence_threshold=0.01, background_id=0, name="test_detection_output"))


def _xe_over_beam():
    states = tch.data_layer(name="sentence_states", size=32)
    scores = tch.data_layer(name="sentence_scores", size=1)
    top_sent = tch.kmax_seq_score_layer(input=scores, beam_size=5)
    top_sen = tch.sub_nested_seq_layer(input=states, selected_indices=top_sent)
    start_scores = tch.fc_layer(input=top_sen, size=1, act=tch.LinearActivation())
    top_start = tch.kmax_seq_score_layer(input=scores, beam_size=5)
    spans = tch.seq_slice_layer(input=top_sen, starts=top_start, ends=None)
    end_scores = tch.fc_layer(input=spans, size=1, act=tch.LinearActivation())
    top_end = tch.kmax_seq_score_layer(input=end_scores, beam_size=5)
    sid = tch.data_layer(name="sentences_ids", size=1)
    st = tch.data_layer(name="start_ids", size=1)
    en = tch.data_layer(name="end_ids", size=1)
    tch.outputs(tch.cross_entropy_over_beam(input=[
        tch.BeamInput(candidate_scores=scores, selected_candidates=top_sent, gold=sid),
        tch.BeamInput(candidate_scores=start_scores, selected_candidates=top_start, gold=st),
        tch.BeamInput(candidate_scores=end_scores, selected_candidates=top_end, gold=en)]))


CONFIGS = {"test_fc": _fc, "layer_activations": _activations, "util_layers": _util,
           "last_first_seq": _last_first_seq, "test_l2_distance_layer": _l2_distance,
           "test_repeat_layer": _repeat, "test_clip_layer": _clip, "test_dot_prod_layer": _dot_prod,
           "test_row_l2_norm_layer": _row_l2_norm, "test_factorization_machine": _fm,
           "test_smooth_l1": _smooth_l1, "test_hsigmoid": _hsigmoid, "test_row_conv": _row_conv,
           "test_scale_shift_layer": _scale_shift, "test_prelu_layer": _prelu, "test_resize_layer": _resize,
           "test_multiplex_layer": _multiplex, "test_expand_layer": _expand, "test_gated_unit_layer": _gated_unit,
           "test_seq_slice_layer": _seq_slice, "test_kmax_seq_socre_layer": _kmax_seq_score,
           "test_bi_grumemory": _bi_gru, "test_grumemory_layer": _gru, "test_lstmemory_layer": _lstm,
           "test_cost_layers_with_weight": _cost_weight, "test_pad": _pad, "test_print_layer": _print,
           "test_seq_concat_reshape": _seq_concat_reshape, "test_spp_layer": _spp, "test_BatchNorm3D": _bn3d,
           "test_scale_sub_region_layer": _scale_sub_region, "unused_layers": _unused,
           "test_sub_nested_seq_select_layer": _sub_nested_seq, "test_maxout": _maxout,
           "test_bilinear_interp": _bilinear, "img_layers": _img(False), "img_trans_layers": _img(True),
           "test_sequence_pooling": _seq_pooling, "shared_fc": _shared_fc, "test_roi_pool_layer": _roi_pool,
           "math_ops": _math_ops, "test_cost_layers": _cost_layers, "test_recursive_topology": _recursive,
           "test_split_datasource": _split_ds, "test_ntm_layers": _ntm, "test_pooling3D_layer": _pool3d,
           "test_conv3d_layer": _conv3d(False), "test_deconv3d_layer": _conv3d(True),
           "test_multibox_loss_layer": _multibox, "test_detection_output_layer": _detection_output,
           "test_cross_entropy_over_beam": _xe_over_beam}


def _core(mc):
    layers = [(lc["name"], lc["type"], lc.get("size"), lc.get("active_type", ""),
               tuple((i["input_layer_name"], i.get("input_parameter_name")) for i in lc.get("inputs", [])),
               lc.get("bias_parameter_name")) for lc in mc.get("layers", [])]
    params = sorted((p["name"], p.get("size"), tuple(p.get("dims", []))) for p in mc.get("parameters", []))
    return layers, params, mc.get("input_layer_names", []), mc.get("output_layer_names", [])


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_model_config_matches_reference_protostr(name):
    path = os.path.join(PROTOSTR, name + ".protostr")
    if not os.path.exists(path):
        pytest.skip("reference protostr not present")
    c = tch.parse_config(CONFIGS[name])
    got = _core(c.model_config())
    text = open(path).read()
    if text.startswith("model_config {"):  # a whole TrainerConfig: its data configs must match too
        tc = cp.from_text("TrainerConfig", text)
        mine = c.trainer_config()
        for k in ("data_config", "test_data_config"):
            if k in tc:
                assert {f: mine[k].get(f) for f in tc[k]} == tc[k], k
        exp = _core(tc["model_config"])
    else:
        exp = _core(cp.from_text("ModelConfig", text))
    assert got[0] == exp[0]
    assert got[1] == exp[1]
    assert got[2:] == exp[2:]
    # the same message through the wire format and back
    mc = c.model_config()
    assert cp.decode("ModelConfig", cp.encode("ModelConfig", mc)) == cp.from_text("ModelConfig", cp.to_text(
        "ModelConfig", mc))


def test_trainer_config_wire_round_trip_and_text():
    def conf():
        tch.settings(batch_size=64, learning_rate=2e-3, learning_method=tch.AdamOptimizer(beta1=0.8),
                     regularization=tch.L2Regularization(1e-4))
        x = tch.data_layer(name="x", size=8)
        h = tch.fc_layer(input=x, size=16, act=tch.ReluActivation())
        p = tch.fc_layer(input=h, size=3, act=tch.SoftmaxActivation())
        tch.outputs(tch.classification_cost(input=p, label=tch.data_layer(name="label", size=3)))

    c = tch.parse_config(conf)
    tc = cp.decode("TrainerConfig", c.proto())
    oc = tc["opt_config"]
    assert oc["batch_size"] == 64 and oc["learning_method"] == "adam" and abs(oc["adam_beta1"] - 0.8) < 1e-12
    assert abs(oc["learning_rate"] - 2e-3) < 1e-15
    mc = tc["model_config"]
    assert [lc["type"] for lc in mc["layers"]] == ["data", "fc", "fc", "data", "multi-class-cross-entropy"]
    assert mc["layers"][1]["bias_parameter_name"] == "___fc_layer_0__.wbias"
    assert mc["input_layer_names"] == ["x", "label"]
    # every v1 parameter name maps onto the Fluid parameter that holds it, with its shape
    from paddle_amd.v2._core import STATE

    fluid_params = {p.name: tuple(p.shape) for p in STATE["main"].global_block().all_parameters()}
    for p in mc["parameters"]:
        fp = c.parameter_name_map[p["name"]]
        assert fp in fluid_params and int(p["size"]) == int(__import__("numpy").prod(fluid_params[fp]))
    txt = c.to_text(whole=True)
    assert cp.from_text("TrainerConfig", txt) == tc


def test_negative_and_packed_fields_decode():
    msg = {"name": "p", "size": 6, "dims": [2, 3], "device": -1, "initial_std": 0.5}
    b = cp.encode("ParameterConfig", msg)
    assert cp.decode("ParameterConfig", b) == msg
    # packed repeated dims (field 9, wire type 2) as another encoder may write them
    packed = cp._key(1, 2) + bytes([1]) + b"p" + cp._key(9, 2) + bytes([2, 2, 3])
    assert cp.decode("ParameterConfig", packed) == {"name": "p", "dims": [2, 3]}


def test_dump_config_cli(tmp_path, capsys):
    from paddle_amd.utils import dump_config

    cfg = tmp_path / "conf.py"
    cfg.write_text("from paddle_amd.trainer_config_helpers import *\n"
                   "settings(batch_size=10, learning_rate=0.1)\n"
                   "n = get_config_arg('n', int, 4)\n"
                   "x = data_layer(name='x', size=6)\n"
                   "outputs(fc_layer(input=x, size=n, act=SoftmaxActivation()))\n")
    assert dump_config.main([str(cfg), "n=5"]) == 0
    mc = cp.from_text("ModelConfig", capsys.readouterr().out)
    assert mc["layers"][1]["size"] == 5 and mc["layers"][1]["active_type"] == "softmax"
    assert dump_config.main([str(cfg), "n=5", "--whole"]) == 0
    tc = cp.from_text("TrainerConfig", capsys.readouterr().out)
    assert tc["opt_config"]["batch_size"] == 10 and "config_files" not in tc  # (only Import()-ed files)
