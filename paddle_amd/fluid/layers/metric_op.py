"""Metric layers (python/paddle/fluid/layers/metric_op.py): accuracy, auc."""
from __future__ import annotations

from ..initializer import ConstantInitializer
from ..layer_helper import LayerHelper
from .nn import topk

__all__ = ["accuracy", "auc"]


def accuracy(input, label, k=1, correct=None, total=None):
    helper = LayerHelper("accuracy", **locals())
    topk_out, topk_indices = topk(input, k=k)
    acc_out = helper.create_variable_for_type_inference(dtype="float32")
    if correct is None:
        correct = helper.create_variable_for_type_inference(dtype="int32")
    if total is None:
        total = helper.create_variable_for_type_inference(dtype="int32")
    helper.append_op(type="accuracy", inputs={"Out": [topk_out], "Indices": [topk_indices], "Label": [label]},
                     outputs={"Accuracy": [acc_out], "Correct": [correct], "Total": [total]})
    acc_out.stop_gradient = True
    return acc_out


def auc(input, label, curve="ROC", num_thresholds=2 ** 12 - 1, topk=1, slide_steps=1):
    helper = LayerHelper("auc", **locals())
    auc_out = helper.create_variable_for_type_inference(dtype="float64")
    batch_auc_out = helper.create_variable_for_type_inference(dtype="float64")
    stat_pos = helper.create_global_variable(persistable=True, dtype="int64", shape=[num_thresholds + 1])
    stat_neg = helper.create_global_variable(persistable=True, dtype="int64", shape=[num_thresholds + 1])
    for v in (stat_pos, stat_neg):
        helper.set_variable_initializer(v, ConstantInitializer(0.0))
    helper.append_op(type="auc", inputs={"Predict": [input], "Label": [label], "StatPos": [stat_pos],
                                         "StatNeg": [stat_neg]},
                     attrs={"curve": curve, "num_thresholds": num_thresholds},
                     outputs={"AUC": [auc_out], "StatPosOut": [stat_pos], "StatNegOut": [stat_neg]})
    return auc_out, batch_auc_out, [stat_pos, stat_neg]
