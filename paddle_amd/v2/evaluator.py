"""v2 evaluators (reference python/paddle/v2/evaluator.py over
trainer_config_helpers/evaluators.py:170-800, computed by the legacy C++
Evaluator classes, paddle/legacy/gserver/evaluators/Evaluator.cpp).

Each evaluator registers the Fluid variables it needs; the v2 trainer fetches them
every batch and hands the values to the evaluator object, which keeps the
reference's pass-level statistics (start / eval / finish):

  classification_error  mean error, weighted by batch size
  auc                   "last-column-auc": positive-class probability binned into
                        2^24 - 1 bins, trapezoid area over the pass (Evaluator.cpp:459-503)
  precision_recall      per-class TP / FP / FN; one ``positive_label`` or the
                        macro / micro averages (Evaluator.cpp:600-760)
  pnpair                positive-negative pair ratio per query id (Evaluator.cpp:760-873)
  chunk                 chunk_eval counts -> precision / recall / F1 over the pass
  ctc_error             edit-distance sum / reference length over the pass
  sum / column_sum      sum of a layer (per column) over the pass (Evaluator.cpp:180-330)
  value_printer, maxid_printer, classification_error_printer
                        print per batch (NotGetableEvaluator: no value)

``EndIteration.metrics`` carry the batch value, ``EndPass.metrics`` /
``TestResult.metrics`` the pass value; an evaluator with several outputs (e.g.
precision_recall) reports ``name.key`` entries as the reference's getNames does.
"""
from __future__ import annotations

import numpy as np

from .. import fluid
from ._core import STATE, guard


class Evaluator:
    """Base: ``fetch`` is the list of Fluid variables read every batch."""

    def __init__(self, name, fetch):
        self.name, self.fetch = name, list(fetch)
        self.start()

    def start(self):
        pass

    def eval(self, values, batch_size):  # values: numpy arrays in fetch order
        raise NotImplementedError

    def values(self) -> dict:  # pass-level (or since start()) results
        return {}


def _register(ev):
    STATE.setdefault("evaluators", []).append(ev)
    return ev


def evaluators():
    return list(STATE.get("evaluators", []))


class _Mean(Evaluator):
    def start(self):
        self.total, self.n = 0.0, 0

    def eval(self, values, bs):
        v = float(np.asarray(values[0]).ravel()[0])
        self.total += v * bs
        self.n += bs
        return {self.name: v}

    def values(self):
        return {self.name: self.total / max(self.n, 1)}


def classification_error(input, label, name=None, top_k=1, **kw):
    with guard():
        acc = fluid.layers.accuracy(input=input, label=label, k=top_k)
        err = fluid.layers.scale(acc, scale=-1.0, bias=1.0)
    return _register(_Mean(name or "classification_error_evaluator", [err]))


class _Auc(Evaluator):
    BINS = (1 << 24) - 1

    def start(self):
        self.pos = np.zeros(self.BINS + 1)
        self.neg = np.zeros(self.BINS + 1)

    def _add(self, prob, label, w):
        b = np.minimum((prob * self.BINS).astype(np.int64), self.BINS)
        np.add.at(self.neg, b[label == 0], w[label == 0])
        np.add.at(self.pos, b[label != 0], w[label != 0])

    @staticmethod
    def _area(pos, neg):
        # bins from the highest score down; trapezoids of the (neg, pos) ROC curve
        tp = np.cumsum(pos[::-1])
        fp = np.cumsum(neg[::-1])
        tp0 = np.concatenate([[0.0], tp[:-1]])
        fp0 = np.concatenate([[0.0], fp[:-1]])
        auc = float(np.sum((fp - fp0) * (tp + tp0) / 2.0))
        return auc / tp[-1] / fp[-1] if tp[-1] > 0 and fp[-1] > 0 else 0.0

    def eval(self, values, bs):
        out = np.asarray(values[0], dtype=np.float64)
        prob = out.reshape(out.shape[0], -1)[:, -1]  # last column: the positive class
        label = np.asarray(values[1]).reshape(-1).astype(np.int64)
        w = np.asarray(values[2], np.float64).reshape(-1) if len(values) > 2 else np.ones_like(prob)
        self._add(prob, label, w)
        return {self.name: self._area(self.pos, self.neg)}

    def values(self):
        return {self.name: self._area(self.pos, self.neg)}


def auc(input, label, name=None, weight=None):
    return _register(_Auc(name or "auc_evaluator", [input, label] + ([weight] if weight is not None else [])))


class _PrecisionRecall(Evaluator):
    def __init__(self, name, fetch, positive_label):
        self.positive_label = -1 if positive_label is None else int(positive_label)
        super().__init__(name, fetch)

    def start(self):
        self.stats = None  # [dim, 3]: TP, FP, FN

    def eval(self, values, bs):
        out = np.asarray(values[0])
        out = out.reshape(out.shape[0], -1)
        label = np.asarray(values[1]).reshape(-1).astype(np.int64)
        w = np.asarray(values[2], np.float64).reshape(-1) if len(values) > 2 else np.ones(len(label))
        dim = out.shape[1]
        if self.stats is None:
            self.stats = np.zeros((dim, 3))
        pred = out.argmax(1)
        hit = pred == label
        np.add.at(self.stats[:, 0], label[hit], w[hit])
        np.add.at(self.stats[:, 1], pred[~hit], w[~hit])
        np.add.at(self.stats[:, 2], label[~hit], w[~hit])
        return self.values()

    @staticmethod
    def _p(tp, fp):
        return tp / (tp + fp) if tp + fp > 0 else 0.0

    @staticmethod
    def _f1(p, r):
        return 2 * p * r / (p + r) if p + r > 0 else 0.0

    def values(self):
        if self.stats is None:
            return {}
        s = self.stats
        n = self.name
        if self.positive_label != -1:
            tp, fp, fn = s[self.positive_label]
            p, r = self._p(tp, fp), self._p(tp, fn)
            return {f"{n}.precision": p, f"{n}.recal": r, f"{n}.F1-score": self._f1(p, r)}
        mp = float(np.mean([self._p(tp, fp) for tp, fp, _ in s]))
        mr = float(np.mean([self._p(tp, fn) for tp, _, fn in s]))
        tp, fp, fn = s.sum(0)
        return {f"{n}.macro-average-precision": mp, f"{n}.macro-average-recall": mr,
                f"{n}.macro-average-F1-score": self._f1(mp, mr),
                f"{n}.micro-average-precision": self._p(tp, fp)}


def precision_recall(input, label, positive_label=None, weight=None, name=None):
    fetch = [input, label] + ([weight] if weight is not None else [])
    return _register(_PrecisionRecall(name or "precision_recall_evaluator", fetch, positive_label))


class _Pnpair(Evaluator):
    def start(self):
        self.rows = []

    def eval(self, values, bs):
        out = np.asarray(values[0], np.float64)
        score = out.reshape(out.shape[0], -1)[:, -1]
        label = np.asarray(values[1]).reshape(-1)
        qid = np.asarray(values[2]).reshape(-1)
        w = np.asarray(values[3], np.float64).reshape(-1) if len(values) > 3 else np.ones(len(score))
        self.rows.append(np.stack([score, label.astype(np.float64), qid.astype(np.float64), w], 1))
        return {self.name: self._ratio(self.rows[-1])}

    @staticmethod
    def _ratio(rows):
        """pos / neg pair weights over pairs of one query with different labels
        (pair weight = mean of the two sample weights; ties count half to each)."""
        pos = neg = 0.0
        for q in np.unique(rows[:, 2]):
            r = rows[rows[:, 2] == q]
            for i in range(len(r)):
                for j in range(i + 1, len(r)):
                    if r[i, 1] == r[j, 1]:
                        continue
                    hi, lo = (r[i], r[j]) if r[i, 1] > r[j, 1] else (r[j], r[i])
                    w = (hi[3] + lo[3]) / 2.0
                    if hi[0] > lo[0]:
                        pos += w
                    elif hi[0] < lo[0]:
                        neg += w
                    else:
                        pos += w / 2
                        neg += w / 2
        return pos / neg if neg > 0 else 0.0

    def values(self):
        return {self.name: self._ratio(np.concatenate(self.rows)) if self.rows else 0.0}


def pnpair(input, label, query_id, weight=None, name=None):
    fetch = [input, label, query_id] + ([weight] if weight is not None else [])
    return _register(_Pnpair(name or "pnpair_evaluator", fetch))


class _Chunk(Evaluator):
    def start(self):
        self.n_infer = self.n_label = self.n_correct = 0

    def _prf(self, ni, nl, nc):
        p = nc / ni if ni else 0.0
        r = nc / nl if nl else 0.0
        return {f"{self.name}.precision": p, f"{self.name}.recall": r,
                f"{self.name}.F1-score": 2 * p * r / (p + r) if nc else 0.0}

    def eval(self, values, bs):
        ni, nl, nc = (int(np.asarray(v).ravel()[0]) for v in values)
        self.n_infer += ni
        self.n_label += nl
        self.n_correct += nc
        return self._prf(ni, nl, nc)

    def values(self):
        return self._prf(self.n_infer, self.n_label, self.n_correct)


def chunk(input, label, chunk_scheme, num_chunk_types, name=None, excluded_chunk_types=None):
    with guard():
        res = fluid.layers.chunk_eval(input=input, label=label, chunk_scheme=chunk_scheme,
                                      num_chunk_types=num_chunk_types, excluded_chunk_types=excluded_chunk_types)
    # (precision, recall, f1, num_infer, num_label, num_correct)
    return _register(_Chunk(name or "chunk_evaluator", list(res[3:6])))


class _CtcError(Evaluator):
    def start(self):
        self.dist = 0.0
        self.seqs = 0

    def eval(self, values, bs):
        d = np.asarray(values[0], np.float64).reshape(-1)
        n = int(np.asarray(values[1]).ravel()[0])
        self.dist += float(d.sum())
        self.seqs += n
        return {self.name: float(d.sum()) / max(n, 1)}

    def values(self):
        return {self.name: self.dist / max(self.seqs, 1)}


def ctc_error(input, label, name=None):
    """Normalised edit distance between the decoded ``input`` and ``label``
    sequences (the reference's CTCErrorEvaluator), averaged over sequences."""
    with guard():
        dist, seq_num = fluid.layers.edit_distance(input=input, label=label, normalized=True)
    return _register(_CtcError(name or "ctc_error_evaluator", [dist, seq_num]))


class _Sum(Evaluator):
    def __init__(self, name, fetch, per_column):
        self.per_column = per_column
        super().__init__(name, fetch)

    def start(self):
        self.acc = None

    def eval(self, values, bs):
        v = np.asarray(values[0], np.float64)
        v = v.reshape(v.shape[0], -1)
        s = v.sum(0) if self.per_column else np.array([v.sum()])
        self.acc = s if self.acc is None else self.acc + s
        return self._out(s)

    def _out(self, s):
        if self.per_column:
            return {f"{self.name}.{i}": float(x) for i, x in enumerate(s)}
        return {self.name: float(s[0])}

    def values(self):
        return self._out(self.acc) if self.acc is not None else {}


def sum(input, name=None, weight=None):  # noqa: A001  (the reference's evaluator name)
    return _register(_Sum(name or "sum_evaluator", [input], False))


def column_sum(input, name=None, weight=None):
    return _register(_Sum(name or "column_sum_evaluator", [input], True))


class _Printer(Evaluator):
    def __init__(self, name, fetch, fmt):
        self.fmt = fmt
        super().__init__(name, fetch)

    def eval(self, values, bs):
        print(self.fmt(self.name, values), flush=True)
        return {}


def value_printer(input, name=None):
    return _register(_Printer(name or "value_printer_evaluator", [input],
                              lambda n, v: f"{n}: value=\n{np.asarray(v[0])}"))


def maxid_printer(input, num_results=1, name=None):
    def fmt(n, v):
        a = np.asarray(v[0])
        a = a.reshape(a.shape[0], -1)
        ids = np.argsort(-a, axis=1)[:, :num_results]
        return f"{n}: max ids=\n{ids}"

    return _register(_Printer(name or "maxid_printer_evaluator", [input], fmt))


def classification_error_printer(input, label, name=None):
    def fmt(n, v):
        a = np.asarray(v[0])
        wrong = a.reshape(a.shape[0], -1).argmax(1) != np.asarray(v[1]).reshape(-1)
        return f"{n}: error samples={np.nonzero(wrong)[0].tolist()}"

    return _register(_Printer(name or "classification_error_printer_evaluator", [input, label], fmt))


class _Metrics:
    def __init__(self, metrics):
        self.metrics = dict(metrics)
