"""ops_more.hip on the C++ executor vs the interpreter: pointwise losses, reverse /
pad / pad_constant_like, prelu (three modes), iou_similarity, arg_min, fill /
assign_value (and their gradients, where they have one) inside a small trained net,
matmul's gradient (transposes, batch broadcast, vectors), cos_sim, multiplex, crop,
norm, conv_shift, bilinear_tensor_product, maxout, fake (de)quantisation,
plus the proximal optimizers; 3 steps, losses to 1e-5, no Python fallback.
test_native_more_gpu.py runs the same cases on a HIP place."""
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


def _binary(lab):
    return L.cast(L.greater_than(lab, L.fill_constant([1], "float32", 0.0)), "float32")


def case_hinge(x, lab, idx):
    return L.mean(simple_op("hinge_loss", {"Logits": [_head(x)], "Labels": [_binary(lab)]}, {}, out_slot="Loss"))


def case_modified_huber(x, lab, idx):
    out, _ = simple_op("modified_huber_loss", {"X": [_head(x)], "Y": [_binary(lab)]}, {},
                       extra_outputs=("IntermediateVal",))
    return L.mean(out)


def case_rank_loss(x, lab, idx):
    return L.mean(simple_op("rank_loss", {"Label": [_binary(lab)], "Left": [_head(x)], "Right": [_head(x)]}, {}))


def case_margin_rank(x, lab, idx):
    sgn = L.scale(_binary(lab), 2.0, bias=-1.0)
    out, _ = simple_op("margin_rank_loss", {"X1": [_head(x)], "X2": [_head(x)], "Label": [sgn]}, {"margin": 0.3},
                       extra_outputs=("Activated",))
    return L.mean(out)


def case_l1_norm(x, lab, idx):
    return L.scale(simple_op("l1_norm", {"X": [_head(x)]}, {}), 0.1)


def case_reverse(x, lab, idx):
    h = _head(x)
    a = simple_op("reverse", {"X": [h]}, {"axis": [1]})
    b = simple_op("reverse", {"X": [h]}, {"axis": [0, -1]})
    return L.mean(L.square(L.elementwise_add(L.elementwise_mul(a, lab), b)))


def case_pad(x, lab, idx):
    p = simple_op("pad", {"X": [_head(x)]}, {"paddings": [1, 0, 2, 1], "pad_value": 0.5})
    return L.mean(L.square(p))


def case_pad_constant_like(x, lab, idx):
    big = simple_op("pad", {"X": [lab]}, {"paddings": [0, 2, 0, 3], "pad_value": 0.0}, stop_gradient=True)
    out = simple_op("pad_constant_like", {"X": [big], "Y": [_head(x)]}, {"pad_value": -0.25})
    return L.mean(L.square(L.elementwise_add(out, big)))


def _prelu(x, mode, shape):
    h = L.reshape(_head(x, 12), [-1, 3, 2, 2])
    a = L.create_parameter(shape, "float32", default_initializer=fluid.initializer.Constant(0.25))
    return L.mean(L.square(simple_op("prelu", {"X": [h], "Alpha": [a]}, {"mode": mode})))


def case_prelu_all(x, lab, idx):
    return _prelu(x, "all", [1])


def case_prelu_channel(x, lab, idx):
    return _prelu(x, "channel", [3])


def case_prelu_element(x, lab, idx):
    return _prelu(x, "element", [12])


def case_iou_argmin_fill(x, lab, idx):
    h = _head(x)
    bx = L.slice(lab, axes=[1], starts=[0], ends=[4])
    by = L.slice(lab, axes=[1], starts=[2], ends=[6])
    iou = simple_op("iou_similarity", {"X": [bx], "Y": [by]}, {"box_normalized": False}, stop_gradient=True)
    am = L.cast(simple_op("arg_min", {"X": [h]}, {"axis": 1}, dtype="int64", stop_gradient=True), "float32")
    f = simple_op("fill", {}, {"shape": [1], "dtype": 5, "value": [0.75]}, dtype="float32", stop_gradient=True)
    av = simple_op("assign_value", {}, {"shape": [2], "dtype": 5, "fp32_values": [0.5, -1.5]}, dtype="float32",
                   stop_gradient=True)
    extra = L.elementwise_add(L.elementwise_add(L.mean(iou), L.mean(am)), L.elementwise_add(f, L.mean(av)))
    return L.elementwise_add(L.mean(L.square(h)), extra)


def case_matmul(x, lab, idx):
    h = L.reshape(_head(x, 12), [-1, 3, 4])              # [4, 3, 4]
    w = L.create_parameter([4, 5], "float32")             # broadcast over the batch
    a = L.matmul(h, w)                                     # [4, 3, 5]
    b = L.matmul(h, h, transpose_y=True, alpha=0.5)        # [4, 3, 3]
    c = L.matmul(w, h, transpose_x=True, transpose_y=True)  # [4, 5, 3]
    v = L.matmul(L.reshape(lab, [-1]), L.reshape(lab, [-1]))  # vector . vector
    return L.elementwise_add(L.elementwise_add(L.mean(L.square(a)), L.mean(b)),
                             L.elementwise_add(L.mean(L.square(c)), L.scale(v, 0.01)))


def case_cos_sim(x, lab, idx):
    h = _head(x)
    one = L.slice(lab, axes=[0], starts=[0], ends=[1])
    o1, _, _ = simple_op("cos_sim", {"X": [h], "Y": [lab]}, {}, extra_outputs=("XNorm", "YNorm"))
    o2, _, _ = simple_op("cos_sim", {"X": [h], "Y": [L.scale(one, 2.0)]}, {}, extra_outputs=("XNorm", "YNorm"))
    return L.elementwise_add(L.mean(o1), L.mean(L.square(o2)))


def case_multiplex(x, lab, idx):
    a, b, c, d = _head(x), _head(x), L.scale(_head(x), -1.0), _head(x)
    return L.mean(L.square(simple_op("multiplex", {"Ids": [idx], "X": [a, b, c, d]}, {})))


def case_crop_norm(x, lab, idx):
    h = _head(x)
    c = simple_op("crop", {"X": [h]}, {"offsets": [1, 2], "shape": [2, 3]})
    n, _ = simple_op("norm", {"X": [h]}, {"axis": 1, "epsilon": 1e-6}, extra_outputs=("Norm",))
    return L.elementwise_add(L.mean(L.square(c)), L.mean(L.elementwise_mul(n, lab)))


def case_conv_shift(x, lab, idx):
    k = L.slice(_head(x), axes=[1], starts=[0], ends=[3])
    return L.mean(L.square(simple_op("conv_shift", {"X": [_head(x)], "Y": [k]}, {})))


def case_bilinear_tensor_product(x, lab, idx):
    w = L.create_parameter([3, 6, 5], "float32")
    b = L.create_parameter([1, 3], "float32")
    out = simple_op("bilinear_tensor_product", {"X": [_head(x)], "Y": [x], "Weight": [w], "Bias": [b]}, {})
    return L.mean(L.square(out))


def case_maxout(x, lab, idx):
    h = L.reshape(_head(x, 12), [-1, 6, 2, 1])
    return L.mean(L.square(simple_op("maxout", {"X": [h]}, {"groups": 3})))


def case_fake_quant(x, lab, idx):
    h = _head(x)
    q, s = simple_op("fake_quantize_abs_max", {"X": [h]}, {"bit_length": 8}, extra_outputs=("OutScale",),
                     stop_gradient=True)
    dq = simple_op("fake_dequantize_max_abs", {"X": [h], "Scale": [s]}, {"max_range": 127.0})
    return L.elementwise_add(L.mean(L.square(dq)), L.scale(L.mean(q), 0.001))


def case_scatter_grads(x, lab, idx):
    h = _head(x)
    up = L.slice(_head(x), axes=[0], starts=[0], ends=[2])
    ids = L.slice(idx, axes=[0], starts=[0], ends=[2])
    ids.stop_gradient = True
    a = simple_op("scatter", {"X": [h], "Ids": [ids], "Updates": [up]}, {"overwrite": True})
    b = simple_op("scatter", {"X": [h], "Ids": [ids], "Updates": [up]}, {"overwrite": False})
    return L.mean(L.square(L.elementwise_add(a, L.scale(b, 0.5))))


def case_memory_helper_lod_reset(x, lab, idx):
    h = simple_op("rnn_memory_helper", {"X": [_head(x)]}, {"dtype": 5})
    rs = simple_op("lod_reset", {"X": [h]}, {"target_lod": [0, 1, 4]})
    return L.mean(L.square(rs))


def case_row_conv_lrn(x, lab, idx):
    w = L.create_parameter([3, 6], "float32")
    rc = simple_op("row_conv", {"X": [_head(x)], "Filter": [w]}, {})
    img = L.reshape(L.elementwise_add(_head(x, 12), L.fill_constant([1], "float32", 1.0)), [-1, 6, 2, 1])
    ln, _ = simple_op("lrn", {"X": [img]}, {"n": 3, "k": 1.0, "alpha": 0.1, "beta": 0.75}, extra_outputs=("MidOut",))
    return L.elementwise_add(L.mean(L.square(rc)), L.mean(L.square(ln)))


def case_argsort_polygon(x, lab, idx):
    h = _head(x)
    v, i = simple_op("argsort", {"X": [h]}, {"axis": 1}, extra_outputs=("Indices",), stop_gradient=True)
    pb = simple_op("polygon_box_transform", {"Input": [L.reshape(h, [-1, 2, 3, 1])]}, {}, out_slot="Output",
                   stop_gradient=True)
    return L.elementwise_add(L.mean(L.square(h)), L.elementwise_add(L.mean(v), L.mean(pb)))


def case_ifelse(x, lab, idx):
    h = _head(x)
    col = L.slice(lab, axes=[1], starts=[0], ends=[1])
    cond = L.less_than(col, L.fill_constant([1], "float32", 0.0))
    ie = L.IfElse(cond)
    with ie.true_block():
        t = ie.input(h)
        ie.output(L.scale(t, 2.0))
    with ie.false_block():
        f = ie.input(h)
        ie.output(L.square(f))
    out = ie()[0]
    return L.mean(out)


def case_pool_index_unpool(x, lab, idx):
    img = L.reshape(_head(x, 16), [-1, 1, 4, 4])
    p, m = simple_op("max_pool2d_with_index", {"X": [img]}, {"ksize": [2, 2], "strides": [2, 2], "paddings": [0, 0],
                                                             "global_pooling": False}, extra_outputs=("Mask",))
    up = simple_op("unpool", {"X": [p], "Indices": [m]}, {"unpooling_type": "max", "ksize": [2, 2],
                                                          "strides": [2, 2], "paddings": [0, 0]})
    return L.elementwise_add(L.mean(L.square(up)), L.mean(p))


def case_box_coder_mean_iou(x, lab, idx):
    h = _head(x)
    a = L.slice(lab, axes=[1], starts=[0], ends=[2])
    prior = L.concat([a, L.elementwise_add(a, L.exp(L.slice(lab, axes=[1], starts=[2], ends=[4])))], axis=1)
    tb = L.concat([a, L.elementwise_add(a, L.exp(L.slice(lab, axes=[1], starts=[4], ends=[6])))], axis=1)
    enc = simple_op("box_coder", {"PriorBox": [prior], "TargetBox": [tb]},
                    {"code_type": "encode_center_size", "box_normalized": False}, out_slot="OutputBox",
                    stop_gradient=True)
    dec = simple_op("box_coder", {"PriorBox": [prior], "TargetBox": [L.slice(h, axes=[1], starts=[0], ends=[4])]},
                    {"code_type": "decode_center_size", "box_normalized": True}, out_slot="OutputBox",
                    stop_gradient=True)
    pred = L.slice(idx, axes=[0], starts=[0], ends=[4])
    miou, _, _ = simple_op("mean_iou", {"Predictions": [pred], "Labels": [L.fill_constant([4, 1], "int64", 2)]},
                           {"num_classes": 4}, out_slot="OutMeanIou", dtype="float32",
                           extra_outputs=("OutWrong", "OutCorrect"), stop_gradient=True)
    extra = L.elementwise_add(L.elementwise_add(L.mean(enc), L.mean(dec)), miou)
    return L.elementwise_add(L.mean(L.square(h)), extra)


def _img(x, c=2, h=3, w=2):
    return L.reshape(_head(x, c * h * w), [-1, c, h, w])


def case_interp(x, lab, idx):
    img = _img(x)
    a = simple_op("bilinear_interp", {"X": [img]}, {"out_h": 5, "out_w": 4, "interp_method": "bilinear",
                                                     "align_corners": True})
    b = simple_op("bilinear_interp", {"X": [img]}, {"out_h": 4, "out_w": 3, "interp_method": "bilinear",
                                                     "align_corners": False})
    c = simple_op("nearest_interp", {"X": [img]}, {"out_h": 6, "out_w": 5, "interp_method": "nearest",
                                                    "align_corners": False})
    return L.elementwise_add(L.elementwise_add(L.mean(L.square(a)), L.mean(L.square(b))), L.mean(L.square(c)))


def case_pad2d(x, lab, idx):
    img = _img(x)
    outs = [simple_op("pad2d", {"X": [img]}, {"paddings": [1, 0, 1, 1], "mode": m, "pad_value": 0.3,
                                               "data_format": "NCHW"}) for m in ("constant", "reflect", "edge")]
    nhwc = simple_op("pad2d", {"X": [L.transpose(img, [0, 2, 3, 1])]},
                     {"paddings": [0, 1, 1, 0], "mode": "edge", "pad_value": 0.0, "data_format": "NHWC"})
    tot = L.mean(L.square(nhwc))
    for o in outs:
        tot = L.elementwise_add(tot, L.mean(L.square(o)))
    return tot


def case_im2sequence(x, lab, idx):
    img = _img(x, 2, 3, 3)
    seq = simple_op("im2sequence", {"X": [img]}, {"kernels": [2, 2], "strides": [1, 1], "paddings": [0, 1, 1, 0]})
    return L.mean(L.square(seq))


def case_fc_grad(x, lab, idx):
    w = L.create_parameter([5, 4], "float32")
    b = L.create_parameter([4], "float32")
    o1 = simple_op("fc", {"Input": [x], "W": [w], "Bias": [b]}, {"in_num_col_dims": 1, "activation_type": "relu"})
    o2 = simple_op("fc", {"Input": [x], "W": [w]}, {"in_num_col_dims": 1, "activation_type": ""})
    return L.elementwise_add(L.mean(L.square(o1)), L.mean(o2))


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


def prox_net(kind):
    """fc + square loss; every parameter updated by proximal_gd / proximal_adagrad."""
    def build():
        x = L.data(name="x", shape=[5], dtype="float32")
        lab = L.data(name="lab", shape=[6], dtype="float32")
        L.data(name="idx", shape=[1], dtype="int64")
        loss = L.mean(L.square(L.elementwise_sub(_head(x), lab)))
        pg = fluid.backward.append_backward(loss)
        lr = L.fill_constant([1], "float32", 0.2)
        blk = fluid.default_main_program().global_block()
        for p, g in pg:
            if kind == "gd":
                blk.append_op(type="proximal_gd", inputs={"Param": [p], "Grad": [g], "LearningRate": [lr]},
                              outputs={"ParamOut": [p]}, attrs={"l1": 0.01, "l2": 0.05})
            else:
                m = L.create_global_var(shape=list(p.shape), value=0.1, dtype="float32", persistable=True)
                blk.append_op(type="proximal_adagrad",
                              inputs={"Param": [p], "Moment": [m], "Grad": [g], "LearningRate": [lr]},
                              outputs={"ParamOut": [p], "MomentOut": [m]}, attrs={"l1": 0.01, "l2": 0.05})
        return [loss]
    return build


def feeds(steps=3):
    out = []
    for s in range(steps):
        rs = np.random.RandomState(60 + s)
        out.append({"x": core.LoDTensor(torch.from_numpy(rs.randn(4, 5).astype("float32"))),
                    "lab": core.LoDTensor(torch.from_numpy(rs.randn(4, 6).astype("float32"))),
                    "idx": core.LoDTensor(torch.from_numpy(np.array([[2], [0], [3], [2]], dtype="int64")))})
    return out


BUILDS = dict({k: net(k) for k in CASES}, proximal_gd=prox_net("gd"), proximal_adagrad=prox_net("adagrad"))


@pytest.mark.parametrize("case", sorted(BUILDS))
def test_more_op_native_host(case):
    fd = feeds()
    place = fluid.CPUPlace()
    ref, init, _ = run(BUILDS[case], fd, "python", place)
    got, _, exe = run(BUILDS[case], fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
