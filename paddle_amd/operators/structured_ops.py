"""Structured-prediction, sampled-softmax and decoding operators.

Parity (SURVEY §2.7 "Losses / metrics", "Beam search"):
  linear_chain_crf (linear_chain_crf_op.h:140-190: Transition rows 0/1 are the
  start/end weights, rows 2.. the tag->tag matrix; output is -log p(y|x)),
  crf_decoding (Viterbi; with Label, 1 where the path matches), chunk_eval
  (chunk_eval_op.h: IOB / IOE / IOBES / plain segment rules), warpctc, ctc_align,
  edit_distance, nce (nce_op.h:94-132: uniform sampler, b = k / num_classes,
  cost -log(o/(o+b)) / -log(b/(o+b))), hierarchical_sigmoid (SimpleCode tree of
  math/matrix_bit_code.h, pre-activation clipped to [-40, 40], soft-relu
  cross entropy), beam_search / beam_search_decode (beam_search_op.cc:
  per-source top-beam over all prefixes' candidates, finished prefixes carry
  end_id; pruning of fully finished sources; decode backtraces the step arrays).

The CRF forward algorithm runs batched over sequences in log space on the device
(one logsumexp per time step for all sequences); gradients come from autograd.
Decoding / metric ops are host-side integer algorithms, as in the reference.
"""
from __future__ import annotations

import torch

from ..autograd import tape as _tape
import torch.nn.functional as F

from ..framework import core
from ..framework.op_kernel_type import LibraryType, register_op_kernel
from ..framework.registry import register_op
from ..ops import oplib as _oplib
from .rnn_ops import _gather, _pack_index


def _off(ctx, slot):
    lod = ctx.input_lod(slot)
    return lod[-1] if lod else [0, ctx.input(slot).shape[0]]


# ------------------------------------------------------------------------- CRF
def _crf_nll(em, trans, lab, off):
    """Batched -log p(label | emission) per sequence; em [T, D], trans [D+2, D]."""
    idx, mask = _pack_index(off, False, em.device)
    N, L = idx.shape
    D = em.shape[1]
    e = _gather(em, idx, mask)                             # [N, L, D]
    start, end, tr = trans[0], trans[1], trans[2:]
    alpha = start + e[:, 0]
    for t in range(1, L):
        nxt = torch.logsumexp(alpha.unsqueeze(2) + tr.unsqueeze(0), dim=1) + e[:, t]
        alpha = torch.where(mask[:, t:t + 1], nxt, alpha)
    logz = torch.logsumexp(alpha + end, dim=1)
    y = _gather(lab.reshape(-1, 1), idx, mask).reshape(N, L).long()
    lens = mask.sum(1)
    score = start[y[:, 0]] + e[:, 0].gather(1, y[:, :1]).squeeze(1)
    for t in range(1, L):
        s = tr[y[:, t - 1], y[:, t]] + e[:, t].gather(1, y[:, t:t + 1]).squeeze(1)
        score = score + torch.where(mask[:, t], s, torch.zeros_like(s))
    last = y.gather(1, (lens - 1).clamp(min=0).unsqueeze(1)).squeeze(1)
    score = score + end[last]
    return (logz - score).unsqueeze(1), idx, mask


@register_op("linear_chain_crf", ["Emission", "Transition", "Label"],
             ["Alpha~", "EmissionExps~", "TransitionExps~", "LogLikelihood"], {}, share_lod=False)
def linear_chain_crf(ctx):
    em, tr, lab = ctx.input("Emission"), ctx.input("Transition"), ctx.input("Label")
    off = _off(ctx, "Emission")
    if ctx.meta:
        ctx.set_output("LogLikelihood", torch.empty(len(off) - 1 if off else 1, 1, dtype=em.dtype, device="meta"))
        for s, t in (("Alpha", em), ("EmissionExps", em), ("TransitionExps", tr)):
            ctx.set_output(s, torch.empty_like(t))
        return
    nll, _, _ = _crf_nll(em, tr, lab, off)
    ctx.set_output("LogLikelihood", nll)
    mx = em.detach().max(1, keepdim=True)[0]
    ctx.set_output("EmissionExps", torch.exp(em.detach() - mx))
    ctx.set_output("TransitionExps", torch.exp(tr.detach()))
    ctx.set_output("Alpha", torch.softmax(em.detach(), 1))


@register_op("crf_decoding", ["Emission", "Transition", "Label?"], ["ViterbiPath"], {}, grad=None, no_infer=True)
def crf_decoding(ctx):
    em, tr = ctx.input("Emission").detach().float(), ctx.input("Transition").detach().float()
    off = _off(ctx, "Emission")
    start, end, T = tr[0], tr[1], tr[2:]
    path = torch.empty(em.shape[0], 1, dtype=torch.int64, device=em.device)
    for i in range(len(off) - 1):
        s, e = off[i], off[i + 1]
        if e == s:
            continue
        score = start + em[s]
        back = []
        for t in range(s + 1, e):
            cand = score.unsqueeze(1) + T
            score, arg = cand.max(0)
            score = score + em[t]
            back.append(arg)
        best = int((score + end).argmax())
        seq = [best]
        for arg in reversed(back):
            best = int(arg[best])
            seq.append(best)
        path[s:e, 0] = torch.tensor(seq[::-1], dtype=torch.int64, device=em.device)
    if ctx.has_input("Label"):
        path = (path == ctx.input("Label").reshape(-1, 1).long()).long()
    ctx.set_output("ViterbiPath", path, ctx.input_lod("Emission"))


# ------------------------------------------------------------------ chunk_eval
_SCHEMES = {"IOB": (2, 0, 1, -1, -1), "IOE": (2, -1, 0, 1, -1), "IOBES": (4, 0, 1, 2, 3),
            "plain": (1, -1, -1, -1, -1)}


def _segments(labels, n_types, scheme):
    ntag, tb, ti, te, ts = _SCHEMES[scheme]
    other = n_types
    segs, start, inside = set(), 0, False
    tag, typ = -1, other

    def ends(pt, pty, t, ty):
        if pty == other:
            return False
        if ty == other or ty != pty:
            return True
        if pt in (tb, ti):
            return t in (tb, ts)
        return pt in (te, ts)

    def begins(pt, pty, t, ty):
        if pty == other:
            return ty != other
        if ty == other:
            return False
        if ty != pty or t in (tb, ts):
            return True
        if t in (ti, te):
            return pt in (te, ts)
        return False

    for i, lab in enumerate(labels):
        pt, pty = tag, typ
        tag, typ = lab % ntag, lab // ntag
        if inside and ends(pt, pty, tag, typ):
            segs.add((start, i - 1, pty))
            inside = False
        if begins(pt, pty, tag, typ):
            start, inside = i, True
    if inside:
        segs.add((start, len(labels) - 1, typ))
    return segs


@register_op("chunk_eval", ["Inference", "Label"],
             ["Precision", "Recall", "F1-Score", "NumInferChunks", "NumLabelChunks", "NumCorrectChunks"],
             {"num_chunk_types": 1, "chunk_scheme": "IOB", "excluded_chunk_types": []}, grad=None, no_infer=True)
def chunk_eval(ctx):
    inf = ctx.input("Inference").reshape(-1).tolist()
    lab = ctx.input("Label").reshape(-1).tolist()
    off = _off(ctx, "Label")
    n, scheme = ctx.attr("num_chunk_types"), ctx.attr("chunk_scheme")
    excl = set(ctx.attr("excluded_chunk_types") or [])
    ni = nl = nc = 0
    for i in range(len(off) - 1):
        a = {s for s in _segments(inf[off[i]:off[i + 1]], n, scheme) if s[2] not in excl}
        b = {s for s in _segments(lab[off[i]:off[i + 1]], n, scheme) if s[2] not in excl}
        ni, nl, nc = ni + len(a), nl + len(b), nc + len(a & b)
    p = nc / ni if ni else 0.0
    r = nc / nl if nl else 0.0
    f1 = 2 * p * r / (p + r) if nc else 0.0
    dev = ctx.input("Label").device
    for s, v, dt in (("Precision", p, torch.float32), ("Recall", r, torch.float32), ("F1-Score", f1, torch.float32),
                     ("NumInferChunks", ni, torch.int64), ("NumLabelChunks", nl, torch.int64),
                     ("NumCorrectChunks", nc, torch.int64)):
        ctx.set_output(s, torch.tensor([v], dtype=dt, device=dev))


# ------------------------------------------------------------------------- CTC
@register_op("warpctc", ["Logits", "Label"], ["WarpCTCGrad~", "Loss"], {"blank": 0, "norm_by_times": False},
             share_lod=False)
def warpctc(ctx):
    """CTC loss (warpctc_op.h).  As in the reference, Loss is the plain -log p(l|x)
    and ``norm_by_times`` scales only the gradient by 1/T (UnpaddingLoDTensorFunctor
    with norm_by_times); impossible alignments give 0 (zero_infinity).  GPU:
    native alpha/beta lattice + fused softmax gradient (seqdet.hip)."""
    x, lab = ctx.input("Logits"), ctx.input("Label")
    xo, lo = _off(ctx, "Logits"), _off(ctx, "Label")
    N = len(xo) - 1
    if ctx.meta:
        ctx.set_output("Loss", torch.empty(N, 1, dtype=x.dtype, device="meta"))
        ctx.set_output("WarpCTCGrad", torch.empty_like(x))
        return
    blank, norm = ctx.attr("blank"), ctx.attr("norm_by_times")
    idx, mask = _pack_index(xo, False, x.device)
    logp = torch.log_softmax(_gather(x.float(), idx, mask), -1).transpose(0, 1)      # [L, N, C]
    xl = torch.tensor([xo[i + 1] - xo[i] for i in range(N)], device=x.device)
    ll = torch.tensor([lo[i + 1] - lo[i] for i in range(N)], device=x.device)
    tgt = lab.reshape(-1).long()
    loss = F.ctc_loss(logp, tgt, xl, ll, blank=blank, reduction="none", zero_infinity=True)
    if norm:
        loss = _tape.apply(_GradScale, loss, 1.0 / xl.clamp(min=1).to(loss.dtype))
    ctx.set_output("Loss", loss.unsqueeze(1).to(x.dtype))
    ctx.set_output("WarpCTCGrad", torch.zeros_like(x))


@register_op_kernel("warpctc", "GPU", [torch.float32, torch.bfloat16], library=LibraryType.NATIVE)
def warpctc_native(ctx):
    """GPU kernel: alpha / beta lattices + fused softmax gradient (seqdet.hip)."""
    x, lab = ctx.input("Logits"), ctx.input("Label")
    loss = _oplib.ctc_loss_op(x, lab, _off(ctx, "Logits"), _off(ctx, "Label"), ctx.attr("blank"),
                              ctx.attr("norm_by_times"))
    if loss is None:
        return warpctc(ctx)
    ctx.set_output("Loss", loss)
    ctx.set_output("WarpCTCGrad", torch.zeros_like(x))


class _GradScale(torch.autograd.Function):
    """Identity forward; backward multiplies the incoming gradient by ``w``."""

    @staticmethod
    def forward(ctx, v, w):
        ctx.save_for_backward(w)
        return v.clone()

    @staticmethod
    def backward(ctx, g):
        (w,) = ctx.saved_tensors
        return g * w, None


@register_op("ctc_align", ["Input"], ["Output"], {"blank": 0, "merge_repeated": True}, grad=None, no_infer=True)
def ctc_align(ctx):
    off = _off(ctx, "Input")
    blank, merge = ctx.attr("blank"), ctx.attr("merge_repeated")
    xin = ctx.input("Input")
    r = _oplib.ctc_align_op(xin, off, blank, merge) if xin.is_cuda else None
    if r is not None:
        ctx.set_output("Output", r[0], [r[1]])
        return
    x = xin.reshape(-1).tolist()
    out, new_off = [], [0]
    for i in range(len(off) - 1):
        prev = None
        for v in x[off[i]:off[i + 1]]:
            if v != blank and not (merge and v == prev):
                out.append(v)
            prev = v
        new_off.append(len(out))
    if not out:  # the reference emits a single -1 when everything was removed
        out, new_off = [-1], [0, 1]
    t = torch.tensor(out, dtype=torch.int64, device=ctx.input("Input").device).reshape(-1, 1)
    ctx.set_output("Output", t, [new_off])


def _levenshtein(a, b):
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


@register_op("edit_distance", ["Hyps", "Refs"], ["SequenceNum", "Out"], {"normalized": False}, grad=None,
             no_infer=True)
def edit_distance(ctx):
    ho, ro = _off(ctx, "Hyps"), _off(ctx, "Refs")
    hyp = ctx.input("Hyps")
    d = _oplib.edit_distance_op(hyp, ctx.input("Refs"), ho, ro, ctx.attr("normalized")) if hyp.is_cuda else None
    if d is not None:
        ctx.set_output("Out", d)
        ctx.set_output("SequenceNum", torch.tensor([len(ho) - 1], dtype=torch.int64, device=hyp.device))
        return
    h, r = hyp.reshape(-1).tolist(), ctx.input("Refs").reshape(-1).tolist()
    out = []
    for i in range(len(ho) - 1):
        a, b = h[ho[i]:ho[i + 1]], r[ro[i]:ro[i + 1]]
        d = float(_levenshtein(a, b))
        if ctx.attr("normalized"):
            d /= max(len(b), 1)
        out.append(d)
    dev = ctx.input("Hyps").device
    ctx.set_output("Out", torch.tensor(out, dtype=torch.float32, device=dev).reshape(-1, 1))
    ctx.set_output("SequenceNum", torch.tensor([len(out)], dtype=torch.int64, device=dev))


# -------------------------------------------------------------- sampled losses
@register_op("nce", ["Input", "Label", "Weight", "Bias?", "SampleWeight?"], ["Cost", "SampleLogits~", "SampleLabels~"],
             {"num_total_classes": 2, "num_neg_samples": 10, "custom_neg_classes": [], "seed": 0, "is_sparse": False},
             share_lod=False)
def nce(ctx):
    x, lab, W = ctx.input("Input"), ctx.input("Label").long(), ctx.input("Weight")
    N = x.shape[0]
    nt = lab.reshape(N, -1).shape[1]
    k = ctx.attr("num_neg_samples")
    C = ctx.attr("num_total_classes")
    if ctx.meta:
        ctx.set_output("Cost", torch.empty(N, 1, dtype=x.dtype, device="meta"))
        ctx.set_output("SampleLogits", torch.empty(N, nt + k, dtype=x.dtype, device="meta"))
        ctx.set_output("SampleLabels", torch.empty(N, nt + k, dtype=torch.int64, device="meta"))
        return
    custom = ctx.attr("custom_neg_classes") or []
    if custom:
        neg = torch.tensor(custom, dtype=torch.int64, device=x.device).reshape(1, -1).expand(N, -1)
    else:
        g = torch.Generator(device="cpu").manual_seed(ctx.attr("seed") or 0)
        neg = torch.randint(0, C, (N, k), generator=g).to(x.device)
    labels = torch.cat([lab.reshape(N, nt), neg], 1)
    logits = (x.unsqueeze(1) * W[labels]).sum(-1)
    if ctx.has_input("Bias"):
        logits = logits + ctx.input("Bias").reshape(-1)[labels]
    o = torch.sigmoid(logits)
    b = float(k) / C
    cost = torch.cat([-torch.log(o[:, :nt] / (o[:, :nt] + b)), -torch.log(b / (o[:, nt:] + b))], 1).sum(1, keepdim=True)
    if ctx.has_input("SampleWeight"):
        cost = cost * ctx.input("SampleWeight").reshape(N, 1)
    ctx.set_output("Cost", cost)
    ctx.set_output("SampleLogits", o.detach())
    ctx.set_output("SampleLabels", labels)


def _hs_codes(label, num_classes):
    """SimpleCode (matrix_bit_code.h:67-79): c = label + num_classes; node index of
    bit j = (c >> (j+1)) - 1, branch bit = (c >> j) & 1, length = floor(log2 c)."""
    c = label.reshape(-1).long() + num_classes
    L = int(num_classes - 1).bit_length()
    j = torch.arange(L, device=label.device)
    idx = (c.unsqueeze(1) >> (j + 1)) - 1
    bit = ((c.unsqueeze(1) >> j) & 1).float()
    length = torch.floor(torch.log2(c.float())).long()
    valid = j.unsqueeze(0) < length.unsqueeze(1)
    return idx.clamp(min=0), bit, valid


@register_op("hierarchical_sigmoid", ["X", "W", "Label", "Bias?"], ["Out", "PreOut~"], {"num_classes": 2},
             share_lod=False)
def hierarchical_sigmoid(ctx):
    x, W, lab = ctx.input("X"), ctx.input("W"), ctx.input("Label")
    C = ctx.attr("num_classes")
    L = int(C - 1).bit_length()
    if ctx.meta:
        ctx.set_output("Out", torch.empty(x.shape[0], 1, dtype=x.dtype, device="meta"))
        ctx.set_output("PreOut", torch.empty(x.shape[0], L, dtype=x.dtype, device="meta"))
        return
    idx, bit, valid = _hs_codes(lab, C)
    pre = (x.unsqueeze(1) * W[idx]).sum(-1)
    if ctx.has_input("Bias"):
        pre = pre + ctx.input("Bias").reshape(-1)[idx]
    pre = pre.clamp(-40.0, 40.0) * valid
    out = (F.softplus(pre) * valid - bit * pre).sum(1, keepdim=True)
    ctx.set_output("Out", out)
    ctx.set_output("PreOut", pre.detach())


# ------------------------------------------------------------------ beam search
@register_op("beam_search", ["pre_ids", "pre_scores?", "ids", "scores"], ["selected_ids", "selected_scores"],
             {"level": 0, "beam_size": 1, "end_id": 0}, grad=None, no_infer=True)
def beam_search(ctx):
    pre_ids = ctx.input("pre_ids").reshape(-1).tolist()
    ps = ctx.input("pre_scores")
    pre_scores = ps.reshape(-1).tolist() if ps is not None else [0.0] * len(pre_ids)
    ids_t, sc_t = ctx.input("ids"), ctx.input("scores")
    lod = ctx.input_lod("ids")
    level = ctx.attr("level")
    beam, end = ctx.attr("beam_size"), ctx.attr("end_id")
    # absolute (row) offsets of the source level (framework::ToAbsOffset)
    if lod:
        absl = [list(l) for l in lod]
        for lv in range(len(lod) - 2, -1, -1):
            absl[lv] = [absl[lv + 1][x] for x in lod[lv]]
        high = absl[level]
    else:
        high = [0, len(pre_ids)]
    ids = ids_t.reshape(len(pre_ids), -1).tolist()
    scores = sc_t.reshape(len(pre_ids), -1).tolist()
    per_prefix = [[] for _ in pre_ids]
    for s in range(len(high) - 1):
        items = []
        for off in range(high[s], high[s + 1]):
            if pre_ids[off] == end:
                items.append((pre_scores[off], off, end))
            else:
                items += [(scores[off][d], off, ids[off][d]) for d in range(len(ids[off]))]
        items.sort(key=lambda t: -t[0])
        for sc, off, i in items[:beam]:
            per_prefix[off].append((i, sc))
        # prune sources whose every branch already ended
        if all(pre_ids[off] == end and all(i == end for i, _ in per_prefix[off]) for off in range(high[s], high[s + 1])):
            for off in range(high[s], high[s + 1]):
                per_prefix[off] = []
    out_ids, out_sc, low = [], [], [0]
    for lst in per_prefix:
        for i, sc in sorted(lst, key=lambda t: -t[1]):
            out_ids.append(i)
            out_sc.append(sc)
        low.append(len(out_ids))
    dev = ids_t.device
    new_lod = [high, low]
    ctx.set_output("selected_ids", torch.tensor(out_ids, dtype=torch.int64, device=dev).reshape(-1, 1), new_lod)
    ctx.set_output("selected_scores", torch.tensor(out_sc, dtype=torch.float32, device=dev).reshape(-1, 1), new_lod)


@register_op("beam_search_decode", ["Ids", "Scores"], ["SentenceIds", "SentenceScores"],
             {"beam_size": 1, "end_id": 0}, grad=None, no_infer=True)
def beam_search_decode(ctx):
    step_ids, step_scores = ctx.input_value("Ids"), ctx.input_value("Scores")
    end = ctx.attr("end_id")
    steps = len(step_ids)
    src_num = len(step_ids[0].lod()[0]) - 1
    sents = [[] for _ in range(src_num)]   # per source: list of [word_ids, scores] built backwards
    prefix = [[] for _ in range(src_num)]  # per source: candidate row each sentence continues from
    for t in range(steps - 1, -1, -1):
        ids = step_ids[t].tensor.reshape(-1).tolist()
        scs = step_scores[t].tensor.reshape(-1).tolist()
        src_lod, sent_lod = step_ids[t].lod()[0], step_ids[t].lod()[1]
        for s in range(src_num):
            ps, pe = src_lod[s], src_lod[s + 1]
            if not prefix[s]:  # finished (pruned) at this step, or the last step: start sentences here
                for p in range(ps, pe):
                    for c in range(sent_lod[p], sent_lod[p + 1]):
                        prefix[s].append(p)
                        sents[s].append([[ids[c]], [scs[c]]])
            else:
                for k, c in enumerate(prefix[s]):
                    w, sc = sents[s][k]
                    if ids[c] != end or not w:
                        w.append(ids[c])
                        sc.append(scs[c])
                    # the prefix row c of this step is candidate row c of the previous step
                    p = ps
                    while sent_lod[p + 1] <= c:
                        p += 1
                    prefix[s][k] = p
    out_ids, out_sc, src_off, sent_off = [], [], [0], [0]
    for s in range(src_num):
        ordered = sorted(sents[s], key=lambda ws: -ws[1][0])  # built backwards: [0] is the final score
        for w, sc in ordered:
            out_ids += w[::-1]
            out_sc += sc[::-1]
            sent_off.append(len(out_ids))
        src_off.append(src_off[-1] + len(ordered))
    dev = step_ids[0].tensor.device
    lod = [src_off, sent_off]
    ctx.set_output("SentenceIds", torch.tensor(out_ids, dtype=torch.int64, device=dev), lod)
    ctx.set_output("SentenceScores", torch.tensor(out_sc, dtype=torch.float32, device=dev), lod)
