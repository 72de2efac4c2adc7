"""Detection layers (python/paddle/fluid/layers/detection.py) over operators/detection_ops.py:
prior_box, multi_box_head, anchor_generator, box_coder, iou_similarity,
bipartite_match, target_assign, detection_output, ssd_loss, detection_map,
rpn_target_assign, generate_proposals, generate_proposal_labels,
polygon_box_transform."""
from __future__ import annotations

from ..layer_helper import LayerHelper

__all__ = ["prior_box", "multi_box_head", "anchor_generator", "box_coder", "iou_similarity", "bipartite_match",
           "target_assign", "detection_output", "ssd_loss", "detection_map", "rpn_target_assign",
           "generate_proposals", "generate_proposal_labels", "polygon_box_transform", "multiclass_nms"]


def _out(helper, dtype="float32", n=1, stop_gradient=True):
    vs = [helper.create_variable_for_type_inference(dtype=dtype, stop_gradient=stop_gradient) for _ in range(n)]
    return vs if n > 1 else vs[0]


def prior_box(input, image, min_sizes, max_sizes=None, aspect_ratios=(1.0,), variance=(0.1, 0.1, 0.2, 0.2),
              flip=False, clip=False, steps=(0.0, 0.0), offset=0.5, name=None, min_max_aspect_ratios_order=False):
    helper = LayerHelper("prior_box", **locals())
    box, var = _out(helper, n=2)
    as_list = lambda v: list(v) if isinstance(v, (list, tuple)) else [v]  # noqa: E731
    helper.append_op(type="prior_box", inputs={"Input": input, "Image": image},
                     outputs={"Boxes": box, "Variances": var},
                     attrs={"min_sizes": as_list(min_sizes), "max_sizes": as_list(max_sizes or []),
                            "aspect_ratios": as_list(aspect_ratios), "variances": list(variance), "flip": flip,
                            "clip": clip, "step_w": steps[0], "step_h": steps[1], "offset": offset,
                            "min_max_aspect_ratios_order": min_max_aspect_ratios_order})
    return box, var


def anchor_generator(input, anchor_sizes=None, aspect_ratios=None, variance=(0.1, 0.1, 0.2, 0.2), stride=None,
                     offset=0.5, name=None):
    helper = LayerHelper("anchor_generator", **locals())
    anc, var = _out(helper, n=2)
    helper.append_op(type="anchor_generator", inputs={"Input": input}, outputs={"Anchors": anc, "Variances": var},
                     attrs={"anchor_sizes": list(anchor_sizes or [64, 128, 256, 512]),
                            "aspect_ratios": list(aspect_ratios or [0.5, 1.0, 2.0]), "variances": list(variance),
                            "stride": list(stride or [16.0, 16.0]), "offset": offset})
    return anc, var


def box_coder(prior_box, prior_box_var, target_box, code_type="encode_center_size", box_normalized=True, name=None):
    helper = LayerHelper("box_coder", **locals())
    out = _out(helper, stop_gradient=False)
    ins = {"PriorBox": prior_box, "TargetBox": target_box}
    if prior_box_var is not None:
        ins["PriorBoxVar"] = prior_box_var
    helper.append_op(type="box_coder", inputs=ins, outputs={"OutputBox": out},
                     attrs={"code_type": code_type, "box_normalized": box_normalized})
    return out


def iou_similarity(x, y, name=None):
    helper = LayerHelper("iou_similarity", **locals())
    out = _out(helper)
    helper.append_op(type="iou_similarity", inputs={"X": x, "Y": y}, outputs={"Out": out})
    return out


def bipartite_match(dist_matrix, match_type=None, dist_threshold=None, name=None):
    helper = LayerHelper("bipartite_match", **locals())
    idx = _out(helper, "int32")
    dist = _out(helper)
    helper.append_op(type="bipartite_match", inputs={"DistMat": dist_matrix},
                     outputs={"ColToRowMatchIndices": idx, "ColToRowMatchDist": dist},
                     attrs={"match_type": match_type or "bipartite",
                            "dist_threshold": 0.5 if dist_threshold is None else dist_threshold})
    return idx, dist


def target_assign(input, matched_indices, negative_indices=None, mismatch_value=None, name=None):
    helper = LayerHelper("target_assign", **locals())
    out, w = _out(helper), _out(helper)
    ins = {"X": input, "MatchIndices": matched_indices}
    if negative_indices is not None:
        ins["NegIndices"] = negative_indices
    helper.append_op(type="target_assign", inputs=ins, outputs={"Out": out, "OutWeight": w},
                     attrs={"mismatch_value": mismatch_value or 0})
    return out, w


def multiclass_nms(bboxes, scores, score_threshold, nms_top_k, keep_top_k, nms_threshold=0.3, normalized=True,
                   nms_eta=1.0, background_label=0, name=None):
    helper = LayerHelper("multiclass_nms", **locals())
    out = _out(helper)
    helper.append_op(type="multiclass_nms", inputs={"BBoxes": bboxes, "Scores": scores}, outputs={"Out": out},
                     attrs={"background_label": background_label, "score_threshold": score_threshold,
                            "nms_top_k": nms_top_k, "nms_threshold": nms_threshold, "nms_eta": nms_eta,
                            "keep_top_k": keep_top_k, "normalized": normalized})
    return out


def detection_output(loc, scores, prior_box, prior_box_var, background_label=0, nms_threshold=0.3, nms_top_k=400,
                     keep_top_k=200, score_threshold=0.01, nms_eta=1.0):
    from .nn import softmax, transpose

    decoded = box_coder(prior_box, prior_box_var, loc, code_type="decode_center_size")
    probs = transpose(softmax(scores), perm=[0, 2, 1])
    return multiclass_nms(decoded, probs, score_threshold, nms_top_k, keep_top_k, nms_threshold, True, nms_eta,
                          background_label)


def polygon_box_transform(input, name=None):
    helper = LayerHelper("polygon_box_transform", **locals())
    out = _out(helper)
    helper.append_op(type="polygon_box_transform", inputs={"Input": input}, outputs={"Output": out})
    return out


def detection_map(detect_res, label, class_num, background_label=0, overlap_threshold=0.3, evaluate_difficult=True,
                  has_state=None, input_states=None, out_states=None, ap_version="integral"):
    helper = LayerHelper("detection_map", **locals())
    m = _out(helper)
    pc, tp, fp = _out(helper, "int32"), _out(helper), _out(helper)
    helper.append_op(type="detection_map", inputs={"DetectRes": detect_res, "Label": label},
                     outputs={"MAP": m, "AccumPosCount": pc, "AccumTruePos": tp, "AccumFalsePos": fp},
                     attrs={"class_num": class_num, "background_label": background_label,
                            "overlap_threshold": overlap_threshold, "evaluate_difficult": evaluate_difficult,
                            "ap_type": ap_version})
    return m


def rpn_target_assign(loc, scores, anchor_box, gt_box, rpn_batch_size_per_im=256, fg_fraction=0.25,
                      rpn_positive_overlap=0.7, rpn_negative_overlap=0.3):
    from .nn import gather, reshape

    helper = LayerHelper("rpn_target_assign", **locals())
    iou = iou_similarity(anchor_box, gt_box)
    li, si = _out(helper, "int32"), _out(helper, "int32")
    tl = _out(helper, "int64")
    helper.append_op(type="rpn_target_assign", inputs={"DistMat": iou},
                     outputs={"LocationIndex": li, "ScoreIndex": si, "TargetLabel": tl},
                     attrs={"rpn_batch_size_per_im": rpn_batch_size_per_im, "fg_fraction": fg_fraction,
                            "rpn_positive_overlap": rpn_positive_overlap,
                            "rpn_negative_overlap": rpn_negative_overlap})
    pred_scores = gather(reshape(scores, [-1, 1]), si)
    pred_loc = gather(reshape(loc, [-1, 4]), li)
    tgt_bbox = gather(reshape(anchor_box, [-1, 4]), li)
    return pred_scores, pred_loc, tl, tgt_bbox


def generate_proposals(scores, bbox_deltas, im_info, anchors, variances, pre_nms_top_n=6000, post_nms_top_n=1000,
                       nms_thresh=0.5, min_size=0.1, eta=1.0, name=None):
    helper = LayerHelper("generate_proposals", **locals())
    rois, probs = _out(helper), _out(helper)
    helper.append_op(type="generate_proposals",
                     inputs={"Scores": scores, "BboxDeltas": bbox_deltas, "ImInfo": im_info, "Anchors": anchors,
                             "Variances": variances},
                     outputs={"RpnRois": rois, "RpnRoiProbs": probs},
                     attrs={"pre_nms_topN": pre_nms_top_n, "post_nms_topN": post_nms_top_n,
                            "nms_thresh": nms_thresh, "min_size": min_size, "eta": eta})
    return rois, probs


def generate_proposal_labels(rpn_rois, gt_classes, gt_boxes, im_scales, batch_size_per_im=256, fg_fraction=0.25,
                             fg_thresh=0.25, bg_thresh_hi=0.5, bg_thresh_lo=0.0,
                             bbox_reg_weights=(0.1, 0.1, 0.2, 0.2), class_nums=None):
    helper = LayerHelper("generate_proposal_labels", **locals())
    outs = [_out(helper) for _ in range(5)]
    outs[1] = _out(helper, "int32")
    helper.append_op(type="generate_proposal_labels",
                     inputs={"RpnRois": rpn_rois, "GtClasses": gt_classes, "GtBoxes": gt_boxes,
                             "ImScales": im_scales},
                     outputs=dict(zip(["Rois", "LabelsInt32", "BboxTargets", "BboxInsideWeights",
                                       "BboxOutsideWeights"], outs)),
                     attrs={"batch_size_per_im": batch_size_per_im, "fg_fraction": fg_fraction,
                            "fg_thresh": fg_thresh, "bg_thresh_hi": bg_thresh_hi, "bg_thresh_lo": bg_thresh_lo,
                            "bbox_reg_weights": list(bbox_reg_weights), "class_nums": class_nums or 81})
    return tuple(outs)


def multi_box_head(inputs, image, base_size, num_classes, aspect_ratios, min_ratio=None, max_ratio=None,
                   min_sizes=None, max_sizes=None, steps=None, step_w=None, step_h=None, offset=0.5,
                   variance=(0.1, 0.1, 0.2, 0.2), flip=True, clip=False, kernel_size=1, pad=0, stride=1, name=None,
                   min_max_aspect_ratios_order=False):
    """SSD heads: per feature map a prior_box + 3x3 conv for locations and confidences."""
    from .nn import conv2d, flatten, reshape, transpose
    from .tensor import concat

    n = len(inputs)
    if min_sizes is None:
        step = int((max_ratio - min_ratio) / (n - 2)) if n > 2 else 0
        min_sizes, max_sizes = [], []
        for r in range(min_ratio, max_ratio + 1, max(step, 1)):
            min_sizes.append(base_size * r / 100.0)
            max_sizes.append(base_size * (r + step) / 100.0)
        min_sizes = [base_size * 0.10] + min_sizes
        max_sizes = [base_size * 0.20] + max_sizes
    locs, confs, boxes, vars_ = [], [], [], []
    for i, x in enumerate(inputs):
        ms = min_sizes[i] if isinstance(min_sizes[i], (list, tuple)) else [min_sizes[i]]
        mx = (max_sizes[i] if isinstance(max_sizes[i], (list, tuple)) else [max_sizes[i]]) if max_sizes else []
        ar = aspect_ratios[i] if isinstance(aspect_ratios[i], (list, tuple)) else [aspect_ratios[i]]
        st = steps[i] if steps else (step_w[i] if step_w else 0.0, step_h[i] if step_h else 0.0)
        st = st if isinstance(st, (list, tuple)) else (st, st)
        b, v = prior_box(x, image, ms, mx, ar, variance, flip, clip, st, offset,
                         min_max_aspect_ratios_order=min_max_aspect_ratios_order)
        boxes.append(reshape(b, [-1, 4]))
        vars_.append(reshape(v, [-1, 4]))
        npri = len(ms) * (len(_expand(ar, flip))) + len(mx)
        loc = conv2d(x, npri * 4, kernel_size, stride, pad)
        conf = conv2d(x, npri * num_classes, kernel_size, stride, pad)
        locs.append(flatten(transpose(loc, [0, 2, 3, 1]), 1))
        confs.append(flatten(transpose(conf, [0, 2, 3, 1]), 1))
    mbox_loc = reshape(concat(locs, axis=1), [0, -1, 4])
    mbox_conf = reshape(concat(confs, axis=1), [0, -1, num_classes])
    return mbox_loc, mbox_conf, concat(boxes), concat(vars_)


def _expand(ars, flip):
    out = [1.0]
    for a in ars:
        for b in ([a, 1.0 / a] if flip else [a]):
            if all(abs(b - c) > 1e-6 for c in out):
                out.append(b)
    return out


def ssd_loss(location, confidence, gt_box, gt_label, prior_box, prior_box_var=None, background_label=0,
             overlap_threshold=0.5, neg_pos_ratio=3.0, neg_overlap=0.5, loc_loss_weight=1.0, conf_loss_weight=1.0,
             match_type="per_prediction", mining_type="max_negative", normalize=True, sample_size=None):
    """SSD multibox loss: match priors to ground truth, mine hard negatives, smooth-L1
    location loss + softmax confidence loss (reference layers/detection.py ssd_loss)."""
    from .nn import reduce_sum, reshape, smooth_l1, softmax_with_cross_entropy
    from .tensor import cast

    helper = LayerHelper("ssd_loss", **locals())
    iou = iou_similarity(gt_box, prior_box)
    matched, dist = bipartite_match(iou, match_type, overlap_threshold)
    gt_label_f = cast(gt_label, "float32")
    tgt_label, _ = target_assign(reshape(gt_label_f, [-1, 1, 1]), matched, mismatch_value=background_label)
    conf_flat = reshape(confidence, [-1, confidence.shape[-1]])
    conf_loss = softmax_with_cross_entropy(conf_flat, cast(reshape(tgt_label, [-1, 1]), "int64"))
    conf_loss = reshape(conf_loss, [-1, prior_box.shape[0]] if prior_box.shape[0] > 0 else [0, -1])
    neg, upd = _out(helper, "int32"), _out(helper, "int32")
    helper.append_op(type="mine_hard_examples",
                     inputs={"ClsLoss": conf_loss, "MatchIndices": matched, "MatchDist": dist},
                     outputs={"NegIndices": neg, "UpdatedMatchIndices": upd},
                     attrs={"neg_pos_ratio": neg_pos_ratio, "neg_dist_threshold": neg_overlap,
                            "mining_type": mining_type, "sample_size": sample_size or 0})
    enc = box_coder(prior_box, prior_box_var, gt_box, code_type="encode_center_size")
    tgt_bbox, tgt_w = target_assign(enc, upd, mismatch_value=background_label)
    tgt_label2, tgt_cw = target_assign(reshape(gt_label_f, [-1, 1, 1]), upd, neg, mismatch_value=background_label)
    conf_loss2 = softmax_with_cross_entropy(conf_flat, cast(reshape(tgt_label2, [-1, 1]), "int64"))
    conf_loss2 = conf_loss2 * reshape(tgt_cw, [-1, 1])
    loc_loss = smooth_l1(reshape(location, [-1, 4]), reshape(tgt_bbox, [-1, 4]), reshape(tgt_w, [-1, 1]))
    loss = conf_loss_weight * reduce_sum(conf_loss2) + loc_loss_weight * reduce_sum(loc_loss)
    if normalize:
        loss = loss / (reduce_sum(tgt_w) + 1e-6)
    return loss
