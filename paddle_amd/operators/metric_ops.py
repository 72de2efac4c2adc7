"""Metric, sparse-table and fake-quantisation operators.

Parity:
  * auc (auc_op.h: num_thresholds buckets with thresholds i/(n-1), -eps and 1+eps
    at the ends, counts accumulated into TP/FP/TN/FN, trapezoid ROC or PR area),
    precision_recall (per-class TP/FP/TN/FN states -> macro and micro P/R/F1),
    positive_negative_pair (pairwise ranking agreement per query), mean_iou,
    detection_map (VOC-style AP per class, ``integral`` or ``11point``);
  * lookup_sparse_table / extract_rows / split_selected_rows / split_ids /
    merge_ids (the distributed lookup-table plumbing of DistributeTranspiler);
  * fake_quantize_abs_max / fake_quantize_range_abs_max / fake_dequantize_max_abs.
Accumulator ops run on the device where the math is vectorisable (auc counts are
one comparison matrix) and on the host for the per-query / per-image loops.
"""
from __future__ import annotations

import numpy as np
import torch

from ..framework import core
from ..framework.op_kernel_type import LibraryType, register_op_kernel
from ..framework.registry import register_op
from ..ops import oplib as _oplib


@register_op("auc", ["Predict", "Label", "TP?", "FP?", "TN?", "FN?"], ["AUC", "TPOut", "FPOut", "TNOut", "FNOut"],
             {"curve": "ROC", "num_thresholds": 200}, grad=None, no_infer=True)
def auc(ctx):
    p = ctx.input("Predict")
    lab = ctx.input("Label").reshape(-1).bool()
    n = ctx.attr("num_thresholds")
    th = torch.arange(n, dtype=torch.float64, device=p.device) / (n - 1)
    th[0], th[-1] = -1e-7, 1.0 + 1e-7
    score = (p[:, 1] if p.dim() == 2 and p.shape[1] > 1 else p.reshape(-1)).double()
    ge = score.unsqueeze(0) >= th.unsqueeze(1)              # [n, N]
    pos = lab.unsqueeze(0)
    cnt = {"TP": (ge & pos).sum(1), "FN": (~ge & pos).sum(1), "FP": (ge & ~pos).sum(1), "TN": (~ge & ~pos).sum(1)}
    out = {}
    for k, v in cnt.items():
        prev = ctx.input(k) if ctx.has_input(k) else None
        out[k] = v.long() + (prev.long().reshape(-1) if prev is not None and prev.numel() == n else 0)
        ctx.set_output(k + "Out", out[k])
    eps = 1e-6
    tp, fn, fp, tn = (out[k].double() for k in ("TP", "FN", "FP", "TN"))
    tpr = (tp + eps) / (tp + fn + eps)
    fpr = fp / (fp + tn + eps)
    prec = (tp + eps) / (tp + fp + eps)
    if ctx.attr("curve") == "PR":
        a = ((tpr[1:] - tpr[:-1]) * (prec[1:] + prec[:-1]) / 2).sum()
    else:
        a = ((fpr[:-1] - fpr[1:]) * (tpr[:-1] + tpr[1:]) / 2).sum()
    ctx.set_output("AUC", a.reshape(1))


@register_op("precision_recall", ["MaxProbs", "Indices", "Labels", "Weights?", "StatesInfo?"],
             ["BatchMetrics", "AccumMetrics", "AccumStatesInfo"], {"class_number": 2}, grad=None, no_infer=True)
def precision_recall(ctx):
    C = ctx.attr("class_number")
    pred = ctx.input("Indices").reshape(-1).long().cpu()
    lab = ctx.input("Labels").reshape(-1).long().cpu()
    w = ctx.input("Weights").reshape(-1).double().cpu() if ctx.has_input("Weights") else torch.ones(len(pred),
                                                                                                    dtype=torch.float64)
    st = torch.zeros(C, 4, dtype=torch.float64)  # TP, FP, TN, FN
    for c in range(C):
        pc, lc = pred == c, lab == c
        st[c, 0] = (w * (pc & lc)).sum()
        st[c, 1] = (w * (pc & ~lc)).sum()
        st[c, 2] = (w * (~pc & ~lc)).sum()
        st[c, 3] = (w * (~pc & lc)).sum()

    def metrics(s):
        tp, fp, fn = s[:, 0], s[:, 1], s[:, 3]
        p = torch.where(tp + fp > 0, tp / (tp + fp).clamp(min=1e-12), torch.ones_like(tp))
        r = torch.where(tp + fn > 0, tp / (tp + fn).clamp(min=1e-12), torch.ones_like(tp))
        mp, mr = p.mean(), r.mean()
        mf = 2 * mp * mr / (mp + mr) if mp + mr > 0 else torch.tensor(0.0, dtype=torch.float64)
        TP, FP, FN = tp.sum(), fp.sum(), fn.sum()
        up = TP / (TP + FP) if TP + FP > 0 else torch.tensor(1.0, dtype=torch.float64)
        ur = TP / (TP + FN) if TP + FN > 0 else torch.tensor(1.0, dtype=torch.float64)
        uf = 2 * up * ur / (up + ur) if up + ur > 0 else torch.tensor(0.0, dtype=torch.float64)
        return torch.stack([mp, mr, mf, up, ur, uf]).float()

    acc = st + (ctx.input("StatesInfo").double().cpu() if ctx.has_input("StatesInfo") else 0)
    dev = ctx.input("Indices").device
    ctx.set_output("BatchMetrics", metrics(st).to(dev))
    ctx.set_output("AccumMetrics", metrics(acc).to(dev))
    ctx.set_output("AccumStatesInfo", acc.float().to(dev))


@register_op("positive_negative_pair",
             ["Score", "Label", "QueryID", "AccumulatePositivePair?", "AccumulateNegativePair?",
              "AccumulateNeutralPair?", "Weight?"], ["PositivePair", "NegativePair", "NeutralPair"], {"column": 0},
             grad=None, no_infer=True)
def positive_negative_pair(ctx):
    s = ctx.input("Score")
    col = ctx.attr("column")
    score = (s[:, col] if s.dim() == 2 else s.reshape(-1)).double().cpu().numpy()
    lab = ctx.input("Label").reshape(-1).double().cpu().numpy()
    q = ctx.input("QueryID").reshape(-1).cpu().numpy()
    w = ctx.input("Weight").reshape(-1).double().cpu().numpy() if ctx.has_input("Weight") else np.ones(len(q))
    pos = neg = neu = 0.0
    for qid in np.unique(q):
        ix = np.nonzero(q == qid)[0]
        for a in range(len(ix)):
            for b in range(a + 1, len(ix)):
                i, j = ix[a], ix[b]
                if lab[i] == lab[j]:
                    continue
                ww = (w[i] + w[j]) / 2
                if score[i] == score[j]:
                    neu += ww
                elif (score[i] > score[j]) == (lab[i] > lab[j]):
                    pos += ww
                else:
                    neg += ww
    dev = s.device
    for slot, acc, v in (("PositivePair", "AccumulatePositivePair", pos), ("NegativePair", "AccumulateNegativePair", neg),
                         ("NeutralPair", "AccumulateNeutralPair", neu)):
        base = float(ctx.input(acc).reshape(-1)[0]) if ctx.has_input(acc) else 0.0
        ctx.set_output(slot, torch.tensor([v + base], dtype=torch.float32, device=dev))


@register_op("mean_iou", ["Predictions", "Labels", "InWrongs*?", "InCorrects*?", "InMeanIou*?"],
             ["OutMeanIou", "OutWrong", "OutCorrect"], {"num_classes": 2}, grad=None, no_infer=True)
def mean_iou(ctx):
    C = ctx.attr("num_classes")
    p = ctx.input("Predictions").reshape(-1).long()
    l = ctx.input("Labels").reshape(-1).long()
    hist = _oplib.mean_iou_hist(p, l, C) if p.is_cuda else None
    if hist is not None:
        correct, wrong = hist[0].long(), hist[1].long()
    else:
        correct = torch.bincount(l[p == l], minlength=C)
        wrong = torch.bincount(p[p != l], minlength=C) + torch.bincount(l[p != l], minlength=C)
    for t in ctx.inputs("InWrongs"):
        wrong = wrong + t.reshape(-1).long()
    for t in ctx.inputs("InCorrects"):
        correct = correct + t.reshape(-1).long()
    den = correct + wrong
    valid = den > 0
    iou = (correct.double() / den.clamp(min=1).double())[valid]
    m = iou.mean() if valid.any() else torch.tensor(0.0, dtype=torch.float64)
    for t in ctx.inputs("InMeanIou"):
        m = m + t.reshape(-1)[0].double()
    ctx.set_output("OutMeanIou", m.float().reshape(1))
    ctx.set_output("OutWrong", wrong.int())
    ctx.set_output("OutCorrect", correct.int())


def _iou(a, b):
    ix = max(0.0, min(a[2], b[2]) - max(a[0], b[0]))
    iy = max(0.0, min(a[3], b[3]) - max(a[1], b[1]))
    inter = ix * iy
    ua = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter
    return inter / ua if ua > 0 else 0.0


@register_op("detection_map", ["DetectRes", "Label", "HasState?", "PosCount?", "TruePos?", "FalsePos?"],
             ["AccumPosCount", "AccumTruePos", "AccumFalsePos", "MAP"],
             {"class_num": 1, "background_label": 0, "overlap_threshold": 0.5, "evaluate_difficult": True,
              "ap_type": "integral"}, grad=None, no_infer=True)
def detection_map(ctx):
    det = ctx.input("DetectRes").double().cpu().numpy()
    gt = ctx.input("Label").double().cpu().numpy()
    doff = ctx.input_lod("DetectRes")[-1] if ctx.input_lod("DetectRes") else [0, len(det)]
    goff = ctx.input_lod("Label")[-1] if ctx.input_lod("Label") else [0, len(gt)]
    thr, bg = ctx.attr("overlap_threshold"), ctx.attr("background_label")
    eval_diff = ctx.attr("evaluate_difficult")
    has_diff = gt.shape[1] == 6
    pos_count, records = {}, {}
    for i in range(len(goff) - 1):
        g = gt[goff[i]:goff[i + 1]]
        d = det[doff[i]:doff[i + 1]] if i < len(doff) - 1 else det[:0]
        for row in g:
            c = int(row[0])
            diff = bool(row[1]) if has_diff else False
            if eval_diff or not diff:
                pos_count[c] = pos_count.get(c, 0) + 1
        for c in set(int(x) for x in d[:, 0]) if len(d) else []:
            dc = d[d[:, 0] == c]
            dc = dc[np.argsort(-dc[:, 1], kind="stable")]
            gc = g[g[:, 0] == c]
            used = np.zeros(len(gc), bool)
            for row in dc:
                box = row[2:6]
                best, bj = -1.0, -1
                for j, grow in enumerate(gc):
                    o = _iou(box, grow[-4:])
                    if o > best:
                        best, bj = o, j
                tp = 0
                if best >= thr:
                    diff = bool(gc[bj][1]) if has_diff else False
                    if not eval_diff and diff:
                        continue
                    if not used[bj]:
                        tp, used[bj] = 1, True
                records.setdefault(c, []).append((row[1], tp))
    aps = []
    for c, npos in pos_count.items():
        if c == bg or npos == 0:
            continue
        rec = sorted(records.get(c, []), key=lambda t: -t[0])
        tps = np.cumsum([t for _, t in rec]) if rec else np.zeros(0)
        fps = np.cumsum([1 - t for _, t in rec]) if rec else np.zeros(0)
        recall = tps / npos
        prec = tps / np.maximum(tps + fps, 1e-12)
        if ctx.attr("ap_type") == "11point":
            ap = sum((prec[recall >= t].max() if (recall >= t).any() else 0.0) for t in np.linspace(0, 1, 11)) / 11
        else:
            ap, prev_r = 0.0, 0.0
            for r, p in zip(recall, prec):
                ap += p * (r - prev_r)
                prev_r = r
        aps.append(ap)
    dev = ctx.input("DetectRes").device
    ctx.set_output("MAP", torch.tensor([float(np.mean(aps)) if aps else 0.0], dtype=torch.float32, device=dev))
    cls = sorted(pos_count)
    ctx.set_output("AccumPosCount", torch.tensor([[pos_count[c]] for c in cls] or [[0]], dtype=torch.int32,
                                                 device=dev))
    for slot in ("AccumTruePos", "AccumFalsePos"):
        rows = [[s, t if slot == "AccumTruePos" else 1 - t] for c in sorted(records) for s, t in records[c]]
        ctx.set_output(slot, torch.tensor(rows or [[0.0, 0.0]], dtype=torch.float32, device=dev))


# ---------------------------------------------------------------- sparse tables
@register_op("lookup_sparse_table", ["W", "Ids"], ["Out"],
             {"padding_idx": -1, "auto_grown_table": True, "is_test": False}, grad=None, no_infer=True)
def lookup_sparse_table(ctx):
    table = ctx.input_value("W")
    ids = ctx.input("Ids").reshape(-1).long()
    rows = list(table.rows())
    val = table.get_tensor().tensor
    pos = {r: i for i, r in enumerate(rows)}
    missing = [int(i) for i in ids.tolist() if int(i) not in pos]
    if missing and ctx.attr("auto_grown_table"):
        new = sorted(set(missing))
        g = torch.Generator().manual_seed(len(rows))
        add = (torch.rand(len(new), val.shape[1], generator=g) * 2 - 1).to(val.device, val.dtype)
        for r in new:
            pos[r] = len(rows)
            rows.append(r)
        val = torch.cat([val, add])
        table.set_rows(rows)
        table.get_tensor().set(val)
    idx = torch.tensor([pos.get(int(i), 0) for i in ids.tolist()], device=val.device)
    out = val[idx]
    pad = ctx.attr("padding_idx")
    if pad is not None and pad >= 0:
        out = out.masked_fill((ids == pad).unsqueeze(1), 0)
    ctx.set_output("Out", out)


@register_op("extract_rows", ["X"], ["Out"], {}, grad=None, no_infer=True)
def extract_rows(ctx):
    sr = ctx.input_value("X")
    ctx.set_output("Out", torch.tensor(list(sr.rows()), dtype=torch.int64).reshape(-1, 1))


@register_op("split_selected_rows", ["X"], ["Out*"], {"height_sections": []}, grad=None, no_infer=True)
def split_selected_rows(ctx):
    sr = ctx.input_value("X")
    secs = list(ctx.attr("height_sections"))
    n_out = len(ctx.output_names("Out"))
    if not secs:
        h = sr.height()
        secs = [h // n_out + (1 if i < h % n_out else 0) for i in range(n_out)]
    bounds = np.cumsum([0] + secs)
    val = sr.get_tensor().tensor
    rows = list(sr.rows())
    outs = []
    for k in range(len(secs)):
        sel = [i for i, r in enumerate(rows) if bounds[k] <= r < bounds[k + 1]]
        o = core.SelectedRows([rows[i] - int(bounds[k]) for i in sel], int(secs[k]))
        o.get_tensor().set(val[torch.tensor(sel, dtype=torch.long, device=val.device)] if sel else val[:0])
        outs.append(o)
    ctx.set_outputs("Out", outs)


@register_op("split_ids", ["Ids*"], ["Out*"], {}, grad=None, no_infer=True)
def split_ids(ctx):
    ids = torch.cat([t.reshape(-1) for t in ctx.inputs("Ids")]).long()
    n = len(ctx.output_names("Out"))
    ctx.set_outputs("Out", [torch.unique(ids[ids % n == k]).reshape(-1, 1) for k in range(n)])


@register_op("merge_ids", ["Ids*", "Rows*", "X*"], ["Out*"], {}, grad=None, no_infer=True)
def merge_ids(ctx):
    """Rows[k] (ids held by shard k) with X[k] (their looked-up values) -> for every
    Ids input, its values in the original id order."""
    rows = [r.reshape(-1).long() for r in ctx.inputs("Rows")]
    xs = ctx.inputs("X")
    if not rows:  # 0.14 form: shard k holds ids with id % n == k, in split_ids (sorted unique) order
        ids_all = torch.cat([t.reshape(-1) for t in ctx.inputs("Ids")]).long()
        n = len(xs)
        rows = [torch.unique(ids_all[ids_all % n == k]) for k in range(n)]
    lut = {}
    for r, x in zip(rows, xs):
        for j, i in enumerate(r.tolist()):
            lut[i] = x[j]
    outs = []
    for ids in ctx.inputs("Ids"):
        flat = ids.reshape(-1).tolist()
        outs.append(torch.stack([lut[i] for i in flat]) if flat else xs[0][:0])
    ctx.set_outputs("Out", outs)


# ---------------------------------------------------------------- fake quant
@register_op("fake_quantize_abs_max", ["X"], ["Out", "OutScale"], {"bit_length": 8}, grad=None)
def fake_quantize_abs_max(ctx):
    x = ctx.input("X")
    bins = (1 << (ctx.attr("bit_length") - 1)) - 1
    s = x.detach().abs().max().reshape(1)
    ctx.set_output("Out", torch.round(x / s.clamp(min=1e-30) * bins))
    ctx.set_output("OutScale", s)


@register_op("fake_quantize_range_abs_max", ["X", "InScale", "Iter?"], ["Out", "OutScale", "OutScales?"],
             {"bit_length": 8, "window_size": 10000, "is_test": False}, grad=None)
def fake_quantize_range_abs_max(ctx):
    x = ctx.input("X")
    bins = (1 << (ctx.attr("bit_length") - 1)) - 1
    in_s = ctx.input("InScale").reshape(1)
    if ctx.attr("is_test"):
        s = in_s
    else:
        s = torch.maximum(x.detach().abs().max().reshape(1), in_s)
    ctx.set_output("Out", torch.round(torch.clamp(x, -s, s) / s.clamp(min=1e-30) * bins))
    ctx.set_output("OutScale", s)
    if ctx.has_output("OutScales"):
        ctx.set_output("OutScales", s.expand(ctx.attr("window_size")).clone())


@register_op_kernel("fake_quantize_abs_max", "GPU", [torch.float32], library=LibraryType.NATIVE)
def fake_quantize_abs_max_native(ctx):
    """GPU kernel (seqdet.hip): |x|max reduction + round(x / s * bins) in two passes."""
    r = _oplib.fake_quant_op(ctx.input("X"), ctx.attr("bit_length"))
    if r is None:
        return fake_quantize_abs_max(ctx)
    ctx.set_output("Out", r[0])
    ctx.set_output("OutScale", r[1])


@register_op_kernel("fake_quantize_range_abs_max", "GPU", [torch.float32], library=LibraryType.NATIVE)
def fake_quantize_range_abs_max_native(ctx):
    r = _oplib.fake_quant_op(ctx.input("X"), ctx.attr("bit_length"), ctx.input("InScale").reshape(1),
                             ctx.attr("is_test"), True)
    if r is None:
        return fake_quantize_range_abs_max(ctx)
    ctx.set_output("Out", r[0])
    ctx.set_output("OutScale", r[1])
    if ctx.has_output("OutScales"):
        ctx.set_output("OutScales", r[1].expand(ctx.attr("window_size")).clone())


@register_op("fake_dequantize_max_abs", ["X", "Scale"], ["Out"], {"max_range": 127.0})
def fake_dequantize_max_abs(ctx):
    ctx.set_output("Out", ctx.input("X") * ctx.input("Scale").reshape(1) / ctx.attr("max_range"))
