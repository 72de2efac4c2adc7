"""detect.hip kernels vs the host implementations of the same operators (which
follow the reference's detection ops): iou_similarity, box_coder encode / decode
(normalized and pixel boxes, with and without variances) and multiclass_nms (the
batched bitmask NMS vs the per-class host loop, including LoD offsets)."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid
from op_test import OpTest
from paddle_amd.framework import core

pytestmark = pytest.mark.gpu


def _run(op, inputs, out_slots, attrs, place):
    t = OpTest()
    t.op_type, t.inputs, t.attrs = op, inputs, attrs
    t.outputs = {s: np.zeros(1, "float32") for s in out_slots}
    prog, _, feed, _, ov, _ = t._build()
    res = fluid.Executor(place).run(prog, feed=feed, fetch_list=[ov[s][0] for s in out_slots], scope=core.Scope(),
                                    return_numpy=False)
    return [(np.asarray(r.numpy() if hasattr(r, "numpy") else r), r.lod() if hasattr(r, "lod") else None)
            for r in res]


def _both(op, inputs, out_slots, attrs):
    return (_run(op, inputs, out_slots, attrs, fluid.CPUPlace()),
            _run(op, inputs, out_slots, attrs, fluid.CUDAPlace(0)))


def _boxes(rng, n, scale=1.0):
    xy = rng.uniform(0, 0.7, (n, 2)) * scale
    wh = rng.uniform(0.05, 0.3, (n, 2)) * scale
    return np.concatenate([xy, xy + wh], 1).astype("float32")


@pytest.mark.parametrize("normalized", [True, False])
def test_iou_similarity(normalized):
    rng = np.random.RandomState(0)
    sc = 1.0 if normalized else 100.0
    x, y = _boxes(rng, 37, sc), _boxes(rng, 53, sc)
    cpu, gpu = _both("iou_similarity", {"X": x, "Y": y}, ["Out"], {"box_normalized": normalized})
    np.testing.assert_allclose(gpu[0][0], cpu[0][0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("normalized", [True, False])
@pytest.mark.parametrize("with_var", [True, False])
def test_box_coder(normalized, with_var):
    rng = np.random.RandomState(1)
    sc = 1.0 if normalized else 100.0
    prior = _boxes(rng, 19, sc)
    var = rng.uniform(0.1, 0.3, (19, 4)).astype("float32")
    tgt = _boxes(rng, 7, sc)
    ins = {"PriorBox": prior, "TargetBox": tgt}
    if with_var:
        ins["PriorBoxVar"] = var
    cpu, gpu = _both("box_coder", ins, ["OutputBox"], {"code_type": "encode_center_size",
                                                      "box_normalized": normalized})
    np.testing.assert_allclose(gpu[0][0], cpu[0][0], rtol=1e-4, atol=1e-5)
    deltas = rng.uniform(-0.5, 0.5, (7, 19, 4)).astype("float32")
    ins["TargetBox"] = deltas
    cpu, gpu = _both("box_coder", ins, ["OutputBox"], {"code_type": "decode_center_size",
                                                      "box_normalized": normalized})
    np.testing.assert_allclose(gpu[0][0], cpu[0][0], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("N,C,M,top_k,keep", [(2, 5, 60, 40, 25), (3, 4, 300, 400, -1), (1, 3, 20, -1, 5)])
def test_multiclass_nms_matches_host(N, C, M, top_k, keep):
    rng = np.random.RandomState(M)
    boxes = np.stack([_boxes(rng, M) for _ in range(N)])
    # clusters of near-duplicates so NMS suppresses something
    boxes[:, 1::3] = boxes[:, 0::3][:, :boxes[:, 1::3].shape[1]] + 0.01
    scores = rng.uniform(0, 1, (N, C, M)).astype("float32")
    attrs = {"background_label": 0, "score_threshold": 0.2, "nms_top_k": top_k, "nms_threshold": 0.4,
             "keep_top_k": keep, "normalized": True}
    cpu, gpu = _both("multiclass_nms", {"BBoxes": boxes, "Scores": scores}, ["Out"], attrs)
    (co, cl), (go, gl) = cpu[0], gpu[0]
    assert cl == gl
    np.testing.assert_allclose(go, co, rtol=1e-6, atol=1e-6)


def test_multiclass_nms_nothing_survives():
    boxes = np.random.RandomState(0).uniform(0, 1, (1, 10, 4)).astype("float32")
    scores = np.zeros((1, 3, 10), "float32")
    _, gpu = _both("multiclass_nms", {"BBoxes": boxes, "Scores": scores}, ["Out"],
                   {"score_threshold": 0.5})
    np.testing.assert_array_equal(gpu[0][0], -np.ones((1, 6), "float32"))
