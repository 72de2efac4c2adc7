"""Detection operators (SSD / Faster-RCNN building blocks).

Parity: paddle/fluid/operators/detection/{prior_box, anchor_generator, box_coder,
iou_similarity, bipartite_match, target_assign, mine_hard_examples,
multiclass_nms, polygon_box_transform, rpn_target_assign, generate_proposals,
generate_proposal_labels}_op.* (SURVEY §2.7 "Detection").  Conventions kept:
pixel boxes use the +1 width convention when ``box_normalized`` is false
(box_coder_op.h:45-66), anchors are Detectron-style (anchor_generator_op.h:
base_w = round(sqrt(stride^2 / ar)), centre w*stride + offset*(stride-1)),
polygon_box_transform outputs (w - x, h - y) on even / odd channels.

Dense geometry (priors, anchors, coders, IoU matrices) is vectorised on the
device; the inherently sequential parts (greedy bipartite matching, NMS,
sampling) run per image with small host loops over already-reduced candidates.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..framework.op_kernel_type import LibraryType, register_op_kernel
from ..framework.registry import register_op
from ..ops import oplib as _oplib


def _expand_ars(ars, flip):
    out = [1.0]
    for a in ars:
        for b in ([a, 1.0 / a] if flip else [a]):
            if all(abs(b - c) > 1e-6 for c in out):
                out.append(b)
    return out


@register_op("prior_box", ["Input", "Image"], ["Boxes", "Variances"],
             {"min_sizes": [], "max_sizes": [], "aspect_ratios": [], "variances": [0.1, 0.1, 0.2, 0.2],
              "flip": True, "clip": True, "step_w": 0.0, "step_h": 0.0, "offset": 0.5,
              "min_max_aspect_ratios_order": False}, grad=None)
def prior_box(ctx):
    feat, img = ctx.input("Input"), ctx.input("Image")
    H, W = feat.shape[2], feat.shape[3]
    IH, IW = img.shape[2], img.shape[3]
    mins, maxs = list(ctx.attr("min_sizes")), list(ctx.attr("max_sizes"))
    ars = _expand_ars(ctx.attr("aspect_ratios"), ctx.attr("flip"))
    sw = ctx.attr("step_w") or IW / W
    sh = ctx.attr("step_h") or IH / H
    off = ctx.attr("offset")
    sizes = []
    for k, m in enumerate(mins):
        if ctx.attr("min_max_aspect_ratios_order"):
            sizes.append((m, m))
            if maxs:
                s = math.sqrt(m * maxs[k])
                sizes.append((s, s))
            sizes += [(m * math.sqrt(a), m / math.sqrt(a)) for a in ars if abs(a - 1.0) > 1e-6]
        else:
            sizes += [(m * math.sqrt(a), m / math.sqrt(a)) for a in ars]
            if maxs:
                s = math.sqrt(m * maxs[k])
                sizes.append((s, s))
    r = _oplib.prior_box_op(feat, H, W, IH, IW, sizes, ctx.attr("variances"), sw, sh, off, ctx.attr("clip"))
    if r is not None:  # GenPriorBox counterpart (detect.hip)
        ctx.set_output("Boxes", r[0].to(feat.dtype))
        ctx.set_output("Variances", r[1].to(feat.dtype))
        return
    dev = feat.device
    bw = torch.tensor([s[0] for s in sizes], device=dev)
    bh = torch.tensor([s[1] for s in sizes], device=dev)
    cx = ((torch.arange(W, device=dev) + off) * sw).view(1, W, 1)
    cy = ((torch.arange(H, device=dev) + off) * sh).view(H, 1, 1)
    boxes = torch.stack([((cx - bw / 2) / IW).expand(H, W, -1), ((cy - bh / 2) / IH).expand(H, W, -1),
                         ((cx + bw / 2) / IW).expand(H, W, -1), ((cy + bh / 2) / IH).expand(H, W, -1)], -1)
    if ctx.attr("clip"):
        boxes = boxes.clamp(0.0, 1.0)
    var = torch.tensor(ctx.attr("variances"), device=dev, dtype=boxes.dtype).expand_as(boxes).contiguous()
    ctx.set_output("Boxes", boxes.to(feat.dtype))
    ctx.set_output("Variances", var.to(feat.dtype))


@register_op("anchor_generator", ["Input"], ["Anchors", "Variances"],
             {"anchor_sizes": [], "aspect_ratios": [], "variances": [0.1, 0.1, 0.2, 0.2], "stride": [16.0, 16.0],
              "offset": 0.5}, grad=None)
def anchor_generator(ctx):
    feat = ctx.input("Input")
    H, W = feat.shape[2], feat.shape[3]
    sw, sh = ctx.attr("stride")
    off = ctx.attr("offset")
    ws, hs = [], []
    for ar in ctx.attr("aspect_ratios"):
        for size in ctx.attr("anchor_sizes"):
            base_w = round(math.sqrt(sw * sh / ar))
            base_h = round(base_w * ar)
            ws.append(size / sw * base_w)
            hs.append(size / sh * base_h)
    r = _oplib.anchor_generator_op(feat, H, W, ws, hs, ctx.attr("variances"), sw, sh, off)
    if r is not None:  # GenAnchors counterpart (detect.hip)
        ctx.set_output("Anchors", r[0].to(feat.dtype))
        ctx.set_output("Variances", r[1].to(feat.dtype))
        return
    dev = feat.device
    aw, ah = torch.tensor(ws, device=dev), torch.tensor(hs, device=dev)
    xc = (torch.arange(W, device=dev) * sw + off * (sw - 1)).view(1, W, 1)
    yc = (torch.arange(H, device=dev) * sh + off * (sh - 1)).view(H, 1, 1)
    anchors = torch.stack([(xc - 0.5 * (aw - 1)).expand(H, W, -1), (yc - 0.5 * (ah - 1)).expand(H, W, -1),
                           (xc + 0.5 * (aw - 1)).expand(H, W, -1), (yc + 0.5 * (ah - 1)).expand(H, W, -1)], -1)
    ctx.set_output("Anchors", anchors.to(feat.dtype))
    ctx.set_output("Variances", torch.tensor(ctx.attr("variances"), device=dev, dtype=feat.dtype)
                   .expand_as(anchors).contiguous())


def _wh(b, normalized):
    one = 0.0 if normalized else 1.0
    return b[..., 2] - b[..., 0] + one, b[..., 3] - b[..., 1] + one


@register_op("box_coder", ["PriorBox", "PriorBoxVar?", "TargetBox"], ["OutputBox"],
             {"code_type": "encode_center_size", "box_normalized": True})
def box_coder(ctx):
    prior, tgt = ctx.input("PriorBox"), ctx.input("TargetBox")
    var = ctx.input("PriorBoxVar") if ctx.has_input("PriorBoxVar") else None
    norm = ctx.attr("box_normalized")
    pw, ph = _wh(prior, norm)
    pcx, pcy = (prior[:, 0] + prior[:, 2]) / 2, (prior[:, 1] + prior[:, 3]) / 2
    if ctx.attr("code_type").lower().startswith("encode"):
        t = tgt.unsqueeze(1)                                 # [N, 1, 4] vs priors [M, 4]
        tw, th = _wh(t, norm)
        tcx, tcy = (t[..., 0] + t[..., 2]) / 2, (t[..., 1] + t[..., 3]) / 2
        out = torch.stack([(tcx - pcx) / pw, (tcy - pcy) / ph, torch.log(torch.abs(tw / pw)),
                           torch.log(torch.abs(th / ph))], -1)
        if var is not None:
            out = out / var
    else:
        d = tgt if tgt.dim() == 3 else tgt.unsqueeze(1)     # [N, M, 4] deltas
        v = var if var is not None else torch.ones_like(prior)
        cx = v[:, 0] * d[..., 0] * pw + pcx
        cy = v[:, 1] * d[..., 1] * ph + pcy
        w = torch.exp(v[:, 2] * d[..., 2]) * pw
        h = torch.exp(v[:, 3] * d[..., 3]) * ph
        one = 0.0 if norm else 1.0
        out = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - one, cy + h / 2 - one], -1)
    ctx.set_output("OutputBox", out)


def _iou_matrix(a, b, normalized=True):
    one = 0.0 if normalized else 1.0
    area_a = (a[:, 2] - a[:, 0] + one) * (a[:, 3] - a[:, 1] + one)
    area_b = (b[:, 2] - b[:, 0] + one) * (b[:, 3] - b[:, 1] + one)
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt + one).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area_a[:, None] + area_b[None, :] - inter).clamp(min=1e-10)


@register_op("iou_similarity", ["X", "Y"], ["Out"], {"box_normalized": True}, grad=None)
def iou_similarity(ctx):
    x, y = ctx.input("X"), ctx.input("Y")
    ctx.set_output("Out", _iou_matrix(x, y, ctx.attr("box_normalized")), ctx.input_lod("X"))


@register_op("bipartite_match", ["DistMat"], ["ColToRowMatchIndices", "ColToRowMatchDist"],
             {"match_type": "bipartite", "dist_threshold": 0.5}, grad=None, no_infer=True)
def bipartite_match(ctx):
    dist = ctx.input("DistMat").detach().float().cpu()
    lod = ctx.input_lod("DistMat")
    off = lod[-1] if lod else [0, dist.shape[0]]
    M = dist.shape[1]
    idx_out = torch.full((len(off) - 1, M), -1, dtype=torch.int32)
    d_out = torch.zeros((len(off) - 1, M), dtype=torch.float32)
    for b in range(len(off) - 1):
        d = dist[off[b]:off[b + 1]].clone()
        if d.numel() == 0:
            continue
        work = d.clone()
        while True:  # greedy global-max bipartite matching
            v, flat = work.reshape(-1).max(0)
            if v <= 0:
                break
            r, c = divmod(int(flat), M)
            idx_out[b, c], d_out[b, c] = r, float(d[r, c])
            work[r, :] = -1
            work[:, c] = -1
        if ctx.attr("match_type") == "per_prediction":
            best_v, best_r = d.max(0)
            sel = (idx_out[b] < 0) & (best_v >= ctx.attr("dist_threshold"))
            idx_out[b][sel] = best_r[sel].int()
            d_out[b][sel] = best_v[sel]
    dev = ctx.input("DistMat").device
    ctx.set_output("ColToRowMatchIndices", idx_out.to(dev))
    ctx.set_output("ColToRowMatchDist", d_out.to(dev))


@register_op("target_assign", ["X", "MatchIndices", "NegIndices?"], ["Out", "OutWeight"], {"mismatch_value": 0},
             grad=None, no_infer=True)
def target_assign(ctx):
    x = ctx.input("X")
    xo = ctx.input_lod("X")[-1] if ctx.input_lod("X") else [0, x.shape[0]]
    mi = ctx.input("MatchIndices").long()
    N, P = mi.shape
    has_neg = ctx.has_input("NegIndices")
    r = _oplib.target_assign_op(x, xo, mi, ctx.input("NegIndices") if has_neg else None,
                                ctx.input_lod("NegIndices")[-1] if has_neg else None, ctx.attr("mismatch_value"))
    if r is not None:  # target_assign kernels (detect.hip)
        ctx.set_output("Out", r[0].to(x.dtype))
        ctx.set_output("OutWeight", r[1].to(x.dtype))
        return
    K = x.shape[-1]
    xs = x.reshape(x.shape[0], -1, K)
    out = torch.full((N, P, K), float(ctx.attr("mismatch_value")), dtype=x.dtype, device=x.device)
    w = torch.zeros(N, P, 1, dtype=x.dtype, device=x.device)
    for b in range(N):
        m = mi[b]
        sel = m >= 0
        rows = xs[xo[b]:xo[b + 1]]
        if sel.any():
            col = torch.nonzero(sel).reshape(-1)
            src = rows[m[sel], col % rows.shape[1]] if rows.shape[1] > 1 else rows[m[sel], 0]
            out[b, sel] = src
            w[b, sel] = 1
    if ctx.has_input("NegIndices"):
        neg = ctx.input("NegIndices").reshape(-1).long()
        no = ctx.input_lod("NegIndices")[-1]
        for b in range(N):
            ids = neg[no[b]:no[b + 1]]
            w[b, ids] = 1
            out[b, ids] = float(ctx.attr("mismatch_value"))
    ctx.set_output("Out", out)
    ctx.set_output("OutWeight", w)


@register_op("mine_hard_examples", ["ClsLoss", "LocLoss?", "MatchIndices", "MatchDist"],
             ["NegIndices", "UpdatedMatchIndices"],
             {"neg_pos_ratio": 1.0, "neg_dist_threshold": 0.5, "sample_size": 0, "mining_type": "max_negative"},
             grad=None, no_infer=True)
def mine_hard_examples(ctx):
    cls = ctx.input("ClsLoss").detach().float().cpu()
    loc = ctx.input("LocLoss").detach().float().cpu() if ctx.has_input("LocLoss") else None
    mi = ctx.input("MatchIndices").long().cpu().clone()
    md = ctx.input("MatchDist").float().cpu()
    N, P = mi.shape
    kind = ctx.attr("mining_type")
    negs, off = [], [0]
    for b in range(N):
        loss = cls[b] + (loc[b] if (loc is not None and kind == "hard_example") else 0)
        if kind == "max_negative":
            cand = torch.nonzero((mi[b] < 0) & (md[b] < ctx.attr("neg_dist_threshold"))).reshape(-1)
            npos = int((mi[b] >= 0).sum())
            k = min(int(npos * ctx.attr("neg_pos_ratio")), len(cand))
        else:
            cand = torch.arange(P)
            k = min(ctx.attr("sample_size"), P)
        order = cand[torch.argsort(loss[cand], descending=True, stable=True)][:k]
        sel = sorted(order.tolist())
        if kind == "hard_example":
            keep = set(sel)
            for p in range(P):
                if mi[b, p] >= 0 and p not in keep:
                    mi[b, p] = -1
            sel = [p for p in sel if mi[b, p] < 0]
        negs += sel
        off.append(len(negs))
    dev = ctx.input("ClsLoss").device
    ctx.set_output("NegIndices", torch.tensor(negs, dtype=torch.int32, device=dev).reshape(-1, 1), [off])
    ctx.set_output("UpdatedMatchIndices", mi.int().to(dev))


def _nms(boxes, scores, thr, top_k, eta=1.0, normalized=True):
    order = torch.argsort(scores, descending=True, stable=True)
    if top_k > -1:
        order = order[:top_k]
    keep = []
    adaptive = thr
    while order.numel():
        i = int(order[0])
        keep.append(i)
        if order.numel() == 1:
            break
        ious = _iou_matrix(boxes[i:i + 1], boxes[order[1:]], normalized)[0]
        order = order[1:][ious <= adaptive]
        if eta < 1 and adaptive > 0.5:
            adaptive *= eta
    return keep


@register_op("multiclass_nms", ["BBoxes", "Scores"], ["Out"],
             {"background_label": 0, "score_threshold": 0.01, "nms_top_k": 400, "nms_threshold": 0.3, "nms_eta": 1.0,
              "keep_top_k": 200, "normalized": True}, grad=None, no_infer=True)
def multiclass_nms(ctx):
    boxes, scores = ctx.input("BBoxes").detach().float(), ctx.input("Scores").detach().float()
    N, C, M = scores.shape
    rows, off = [], [0]
    for b in range(N):
        dets = []
        for c in range(C):
            if c == ctx.attr("background_label"):
                continue
            s = scores[b, c]
            cand = torch.nonzero(s > ctx.attr("score_threshold")).reshape(-1)
            if not cand.numel():
                continue
            keep = _nms(boxes[b, cand], s[cand], ctx.attr("nms_threshold"), ctx.attr("nms_top_k"),
                        ctx.attr("nms_eta"), ctx.attr("normalized"))
            for k in keep:
                i = int(cand[k])
                dets.append([float(c), float(s[i])] + boxes[b, i].tolist())
        dets.sort(key=lambda r: -r[1])
        if ctx.attr("keep_top_k") > -1:
            dets = dets[:ctx.attr("keep_top_k")]
        rows += dets
        off.append(len(rows))
    if not rows:  # the reference emits one row of -1 when nothing survives
        rows, off = [[-1.0] * 6], [0, 1]
    ctx.set_output("Out", torch.tensor(rows, dtype=torch.float32, device=boxes.device), [off])


# ---------------------------------------------------------------- typed GPU kernels (detect.hip)


@register_op_kernel("iou_similarity", "GPU", [torch.float32], library=LibraryType.NATIVE)
def iou_similarity_native(ctx):
    r = _oplib.iou_matrix_op(ctx.input("X"), ctx.input("Y"), ctx.attr("box_normalized"))
    if r is None:
        return iou_similarity(ctx)
    ctx.set_output("Out", r, ctx.input_lod("X"))


@register_op_kernel("box_coder", "GPU", [torch.float32], library=LibraryType.NATIVE)
def box_coder_native(ctx):
    dec = not ctx.attr("code_type").lower().startswith("encode")
    var = ctx.input("PriorBoxVar") if ctx.has_input("PriorBoxVar") else None
    r = _oplib.box_coder_op(dec, ctx.input("PriorBox"), var, ctx.input("TargetBox"), ctx.attr("box_normalized"))
    if r is None:
        return box_coder(ctx)
    ctx.set_output("OutputBox", r)


@register_op_kernel("multiclass_nms", "GPU", [torch.float32], library=LibraryType.NATIVE)
def multiclass_nms_native(ctx):
    """Batched bitmask NMS; adaptive thresholds (nms_eta < 1) stay on the host loop."""
    r = None
    if ctx.attr("nms_eta") >= 1.0:
        r = _oplib.multiclass_nms_op(ctx.input("BBoxes"), ctx.input("Scores"), ctx.attr("background_label"),
                                     ctx.attr("score_threshold"), ctx.attr("nms_top_k"), ctx.attr("nms_threshold"),
                                     ctx.attr("keep_top_k"), ctx.attr("normalized"))
    if r is None:
        return multiclass_nms(ctx)
    ctx.set_output("Out", r[0], [r[1]])


@register_op("polygon_box_transform", ["Input"], ["Output"], {}, grad=None)
def polygon_box_transform(ctx):
    x = ctx.input("Input")
    r = _oplib.polygon_box_transform_op(x)
    if r is not None:  # PolygonBoxTransformKernel counterpart (detect.hip)
        ctx.set_output("Output", r)
        return
    N, C, H, W = x.shape
    gw = torch.arange(W, device=x.device, dtype=x.dtype).view(1, 1, 1, W).expand(N, C, H, W)
    gh = torch.arange(H, device=x.device, dtype=x.dtype).view(1, 1, H, 1).expand(N, C, H, W)
    even = (torch.arange(C, device=x.device) % 2 == 0).view(1, C, 1, 1)
    ctx.set_output("Output", torch.where(even, gw, gh) - x)


def _rng(ctx):
    return np.random.RandomState(ctx.attr("seed") if ctx.attr("fix_seed") else None)


@register_op("rpn_target_assign", ["DistMat"], ["LocationIndex", "ScoreIndex", "TargetLabel"],
             {"rpn_positive_overlap": 0.7, "rpn_negative_overlap": 0.3, "fg_fraction": 0.25,
              "rpn_batch_size_per_im": 256, "fix_seed": False, "seed": 0}, grad=None, no_infer=True)
def rpn_target_assign(ctx):
    dist = ctx.input("DistMat").detach().float().cpu().numpy()  # [anchors*, gt] per image (LoD over anchors)
    lod = ctx.input_lod("DistMat")
    off = lod[-1] if lod else [0, dist.shape[0]]
    rng = _rng(ctx)
    loc, score, lab = [], [], []
    for b in range(len(off) - 1):
        d = dist[off[b]:off[b + 1]]
        A = d.shape[0]
        labels = -np.ones(A, np.int64)
        if d.shape[1]:
            amax = d.max(1)
            labels[amax < ctx.attr("rpn_negative_overlap")] = 0
            gt_best = d.max(0)
            labels[np.nonzero((d == gt_best[None, :]) & (gt_best[None, :] > 0))[0]] = 1
            labels[amax >= ctx.attr("rpn_positive_overlap")] = 1
        else:
            labels[:] = 0
        bs = ctx.attr("rpn_batch_size_per_im")
        fg = np.nonzero(labels == 1)[0]
        nfg = int(ctx.attr("fg_fraction") * bs)
        if len(fg) > nfg:
            labels[rng.choice(fg, len(fg) - nfg, replace=False)] = -1
        fg = np.nonzero(labels == 1)[0]
        bg = np.nonzero(labels == 0)[0]
        nbg = bs - len(fg)
        if len(bg) > nbg:
            labels[rng.choice(bg, len(bg) - nbg, replace=False)] = -1
        bg = np.nonzero(labels == 0)[0]
        loc += (fg + off[b]).tolist()
        score += (np.concatenate([fg, bg]) + off[b]).tolist()
        lab += [1] * len(fg) + [0] * len(bg)
    dev = ctx.input("DistMat").device
    ctx.set_output("LocationIndex", torch.tensor(loc, dtype=torch.int32, device=dev))
    ctx.set_output("ScoreIndex", torch.tensor(score, dtype=torch.int32, device=dev))
    ctx.set_output("TargetLabel", torch.tensor(lab, dtype=torch.int64, device=dev).reshape(-1, 1))


def _decode_clip(anchors, deltas, var, im_h, im_w):
    aw = anchors[:, 2] - anchors[:, 0] + 1
    ah = anchors[:, 3] - anchors[:, 1] + 1
    acx, acy = anchors[:, 0] + 0.5 * aw, anchors[:, 1] + 0.5 * ah
    d = deltas * var if var is not None else deltas
    cx, cy = d[:, 0] * aw + acx, d[:, 1] * ah + acy
    w = torch.exp(d[:, 2].clamp(max=math.log(1000.0 / 16))) * aw
    h = torch.exp(d[:, 3].clamp(max=math.log(1000.0 / 16))) * ah
    b = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - 1, cy + h / 2 - 1], 1)
    b[:, 0::2] = b[:, 0::2].clamp(0, im_w - 1)
    b[:, 1::2] = b[:, 1::2].clamp(0, im_h - 1)
    return b


@register_op("generate_proposals", ["Scores", "BboxDeltas", "ImInfo", "Anchors", "Variances?"],
             ["RpnRois", "RpnRoiProbs"],
             {"pre_nms_topN": 6000, "post_nms_topN": 1000, "nms_thresh": 0.5, "min_size": 0.1, "eta": 1.0},
             grad=None, no_infer=True)
def generate_proposals(ctx):
    sc, dl = ctx.input("Scores").detach().float(), ctx.input("BboxDeltas").detach().float()
    info = ctx.input("ImInfo").detach().float()
    anchors = ctx.input("Anchors").detach().float().reshape(-1, 4)
    var = ctx.input("Variances").detach().float().reshape(-1, 4) if ctx.has_input("Variances") else None
    N, A, H, W = sc.shape
    rois, probs, off = [], [], [0]
    for b in range(N):
        s = sc[b].permute(1, 2, 0).reshape(-1)
        d = dl[b].view(A, 4, H, W).permute(2, 3, 0, 1).reshape(-1, 4)
        order = torch.argsort(s, descending=True, stable=True)
        if ctx.attr("pre_nms_topN") > 0:
            order = order[:ctx.attr("pre_nms_topN")]
        boxes = _decode_clip(anchors[order], d[order], var[order] if var is not None else None, float(info[b, 0]),
                             float(info[b, 1]))
        ms = ctx.attr("min_size") * float(info[b, 2])
        ok = ((boxes[:, 2] - boxes[:, 0] + 1) >= ms) & ((boxes[:, 3] - boxes[:, 1] + 1) >= ms)
        boxes, ss = boxes[ok], s[order][ok]
        keep = _nms(boxes, ss, ctx.attr("nms_thresh"), -1, ctx.attr("eta"), normalized=False)
        keep = keep[:ctx.attr("post_nms_topN")] if ctx.attr("post_nms_topN") > 0 else keep
        rois.append(boxes[keep])
        probs.append(ss[keep].reshape(-1, 1))
        off.append(off[-1] + len(keep))
    ctx.set_output("RpnRois", torch.cat(rois) if rois else sc.new_zeros(0, 4), [off])
    ctx.set_output("RpnRoiProbs", torch.cat(probs) if probs else sc.new_zeros(0, 1), [off])


@register_op("generate_proposal_labels", ["RpnRois", "GtClasses", "GtBoxes", "ImScales"],
             ["Rois", "LabelsInt32", "BboxTargets", "BboxInsideWeights", "BboxOutsideWeights"],
             {"batch_size_per_im": 256, "fg_fraction": 0.25, "fg_thresh": 0.25, "bg_thresh_hi": 0.5,
              "bg_thresh_lo": 0.0, "bbox_reg_weights": [0.1, 0.1, 0.2, 0.2], "class_nums": 81, "fix_seed": False,
              "seed": 0}, grad=None, no_infer=True)
def generate_proposal_labels(ctx):
    rois_all = ctx.input("RpnRois").detach().float().cpu()
    gtc = ctx.input("GtClasses").reshape(-1).long().cpu()
    gtb = ctx.input("GtBoxes").detach().float().cpu()
    scales = ctx.input("ImScales").reshape(-1).float().cpu()
    ro = ctx.input_lod("RpnRois")[-1]
    go = ctx.input_lod("GtBoxes")[-1]
    rng = _rng(ctx)
    C = ctx.attr("class_nums")
    wts = torch.tensor(ctx.attr("bbox_reg_weights"))
    out_r, out_l, out_t, out_iw, off = [], [], [], [], [0]
    for b in range(len(ro) - 1):
        gb = gtb[go[b]:go[b + 1]]
        gc = gtc[go[b]:go[b + 1]]
        r = torch.cat([rois_all[ro[b]:ro[b + 1]] / scales[b], gb])
        ov = _iou_matrix(r, gb, False) if len(gb) else torch.zeros(len(r), 0)
        mx, arg = (ov.max(1) if ov.shape[1] else (torch.zeros(len(r)), torch.zeros(len(r), dtype=torch.long)))
        fg = np.nonzero((mx >= ctx.attr("fg_thresh")).numpy())[0]
        bg = np.nonzero(((mx < ctx.attr("bg_thresh_hi")) & (mx >= ctx.attr("bg_thresh_lo"))).numpy())[0]
        nfg = min(int(ctx.attr("fg_fraction") * ctx.attr("batch_size_per_im")), len(fg))
        fg = rng.choice(fg, nfg, replace=False) if len(fg) > nfg else fg
        nbg = min(ctx.attr("batch_size_per_im") - len(fg), len(bg))
        bg = rng.choice(bg, nbg, replace=False) if len(bg) > nbg else bg
        keep = np.concatenate([fg, bg]).astype(np.int64)
        sel = r[keep]
        labels = torch.cat([gc[arg[fg]] if len(fg) else torch.zeros(0, dtype=torch.long),
                            torch.zeros(len(bg), dtype=torch.long)])
        tgt = torch.zeros(len(keep), 4 * C)
        iw = torch.zeros(len(keep), 4 * C)
        if len(fg):
            g = gb[arg[fg]]
            pw, ph = sel[:len(fg), 2] - sel[:len(fg), 0] + 1, sel[:len(fg), 3] - sel[:len(fg), 1] + 1
            pcx, pcy = sel[:len(fg), 0] + 0.5 * pw, sel[:len(fg), 1] + 0.5 * ph
            gw, gh = g[:, 2] - g[:, 0] + 1, g[:, 3] - g[:, 1] + 1
            gcx, gcy = g[:, 0] + 0.5 * gw, g[:, 1] + 0.5 * gh
            d = torch.stack([(gcx - pcx) / pw, (gcy - pcy) / ph, torch.log(gw / pw), torch.log(gh / ph)], 1) / wts
            for i in range(len(fg)):
                c = int(labels[i])
                tgt[i, 4 * c:4 * c + 4] = d[i]
                iw[i, 4 * c:4 * c + 4] = 1
        out_r.append(sel * scales[b])
        out_l.append(labels)
        out_t.append(tgt)
        out_iw.append(iw)
        off.append(off[-1] + len(keep))
    dev = ctx.input("RpnRois").device
    lod = [off]
    ctx.set_output("Rois", torch.cat(out_r).to(dev), lod)
    ctx.set_output("LabelsInt32", torch.cat(out_l).int().reshape(-1, 1).to(dev), lod)
    ctx.set_output("BboxTargets", torch.cat(out_t).to(dev), lod)
    ctx.set_output("BboxInsideWeights", torch.cat(out_iw).to(dev), lod)
    ctx.set_output("BboxOutsideWeights", torch.cat(out_iw).to(dev), lod)
