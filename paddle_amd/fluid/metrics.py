"""Host-side streaming metrics (API of python/paddle/fluid/metrics.py, written from
its documented behaviour).

Every metric declares its accumulator fields in ``_STATE`` (name -> zero value);
``reset`` restores them and ``get_config`` snapshots them, so the base class never
has to guess which instance attributes are state.  Updates are vectorised numpy.
"""
from __future__ import annotations

import copy

import numpy as np

__all__ = ["MetricBase", "CompositeMetric", "Precision", "Recall", "Accuracy", "ChunkEvaluator", "EditDistance",
           "DetectionMAP", "Auc"]


def _scalar(x):
    """First element of a number / array / 1-element tensor as a Python number."""
    return np.asarray(x).reshape(-1)[0].item()


def _check_number_or_array(x, what):
    if not isinstance(x, (int, float, np.integer, np.floating, np.ndarray)):
        raise ValueError(f"{what} must be a number or a numpy array, got {type(x).__name__}")


class MetricBase:
    """Base of all metrics: ``update`` accumulates a mini-batch, ``eval`` reports."""

    _STATE: dict = {}

    def __init__(self, name):
        self._name = self.__class__.__name__ if name is None else str(name)
        self.reset()

    def __str__(self):
        return self._name

    def reset(self):
        for field, zero in self._STATE.items():
            setattr(self, field, copy.copy(zero))

    def get_config(self):
        return {"name": self._name,
                "states": {f: copy.deepcopy(getattr(self, f)) for f in self._STATE}}

    def update(self, preds, labels):
        raise NotImplementedError(f"{type(self).__name__}.update")

    def eval(self):
        raise NotImplementedError(f"{type(self).__name__}.eval")


class CompositeMetric(MetricBase):
    """Several metrics fed the same (preds, labels)."""

    def __init__(self, name=None):
        super().__init__(name)
        self._metrics = []

    def add_metric(self, metric):
        if not isinstance(metric, MetricBase):
            raise ValueError(f"add_metric expects a MetricBase, got {type(metric).__name__}")
        self._metrics.append(metric)

    def update(self, preds, labels):
        for m in self._metrics:
            m.update(preds, labels)

    def eval(self):
        return [m.eval() for m in self._metrics]


def _binary(preds, labels):
    return np.rint(np.asarray(preds)).astype(np.int64).ravel(), np.asarray(labels).astype(np.int64).ravel()


class Precision(MetricBase):
    """Binary precision tp / (tp + fp); predictions are rounded to 0/1."""

    _STATE = {"tp": 0, "fp": 0}

    def __init__(self, name=None):
        super().__init__(name)

    def update(self, preds, labels):
        p, l = _binary(preds, labels)
        pos = p == 1
        self.tp += int(np.count_nonzero(pos & (l == 1)))
        self.fp += int(np.count_nonzero(pos & (l != 1)))

    def eval(self):
        n = self.tp + self.fp
        return self.tp / n if n else 0.0


class Recall(MetricBase):
    """Binary recall tp / (tp + fn); predictions are rounded to 0/1."""

    _STATE = {"tp": 0, "fn": 0}

    def __init__(self, name=None):
        super().__init__(name)

    def update(self, preds, labels):
        p, l = _binary(preds, labels)
        actual = l == 1
        self.tp += int(np.count_nonzero(actual & (p == 1)))
        self.fn += int(np.count_nonzero(actual & (p != 1)))

    def eval(self):
        n = self.tp + self.fn
        return self.tp / n if n else 0.0


class Accuracy(MetricBase):
    """Weighted running mean of per-batch accuracies."""

    _STATE = {"value": 0.0, "weight": 0.0}

    def __init__(self, name=None):
        super().__init__(name)

    def update(self, value, weight):
        _check_number_or_array(value, "Accuracy value")
        self.value += float(_scalar(value)) * weight
        self.weight += weight

    def eval(self):
        if not self.weight:
            raise ValueError("Accuracy.eval() called before any update")
        return self.value / self.weight


class ChunkEvaluator(MetricBase):
    """Chunk precision / recall / F1 from the chunk_eval op's three counters."""

    _STATE = {"num_infer_chunks": 0, "num_label_chunks": 0, "num_correct_chunks": 0}

    def __init__(self, name=None):
        super().__init__(name)

    def update(self, num_infer_chunks, num_label_chunks, num_correct_chunks):
        self.num_infer_chunks += int(_scalar(num_infer_chunks))
        self.num_label_chunks += int(_scalar(num_label_chunks))
        self.num_correct_chunks += int(_scalar(num_correct_chunks))

    def eval(self):
        c = float(self.num_correct_chunks)
        prec = c / self.num_infer_chunks if self.num_infer_chunks else 0.0
        rec = c / self.num_label_chunks if self.num_label_chunks else 0.0
        f1 = 2.0 * prec * rec / (prec + rec) if c else 0.0
        return prec, rec, f1


class EditDistance(MetricBase):
    """Mean edit distance per sequence and the fraction of sequences with any error."""

    _STATE = {"total_distance": 0.0, "seq_num": 0, "instance_error": 0}

    def __init__(self, name):
        super().__init__(name)

    def update(self, distances, seq_num):
        d = np.asarray(distances).ravel()
        n = int(seq_num)
        self.seq_num += n
        self.instance_error += n - int(np.count_nonzero(d == 0))
        self.total_distance += float(d.sum())

    def eval(self):
        if not self.seq_num:
            raise ValueError("EditDistance.eval() called before any update")
        return self.total_distance / self.seq_num, self.instance_error / float(self.seq_num)


class DetectionMAP(MetricBase):
    """Weighted running mean of per-batch mAP values (detection_map op outputs)."""

    _STATE = {"value": 0.0, "weight": 0.0}

    def __init__(self, name=None):
        super().__init__(name)

    def update(self, value, weight):
        self.value += float(_scalar(value)) * weight
        self.weight += weight

    def eval(self):
        if not self.weight:
            raise ValueError("DetectionMAP.eval() called before any update")
        return self.value / self.weight


class Auc(MetricBase):
    """Streaming ROC AUC over ``num_thresholds + 1`` score bins."""

    def __init__(self, name, curve="ROC", num_thresholds=4095):
        self._curve = curve
        self._num_thresholds = num_thresholds
        super().__init__(name=name)

    def reset(self):
        self._stat_pos = np.zeros(self._num_thresholds + 1, dtype=np.float64)
        self._stat_neg = np.zeros(self._num_thresholds + 1, dtype=np.float64)

    def get_config(self):
        return {"name": self._name, "states": {"stat_pos": self._stat_pos.copy(), "stat_neg": self._stat_neg.copy()}}

    def update(self, preds, labels):
        p = np.asarray(preds)
        score = p[:, 1] if p.ndim > 1 else p.ravel()
        bins = (score * self._num_thresholds).astype(np.int64)
        if bins.size and (bins.max() > self._num_thresholds or bins.min() < 0):
            raise ValueError("Auc expects probabilities in [0, 1]")
        pos = np.asarray(labels).ravel().astype(bool)
        self._stat_pos += np.bincount(bins[pos], minlength=self._num_thresholds + 1)
        self._stat_neg += np.bincount(bins[~pos], minlength=self._num_thresholds + 1)

    def eval(self):
        # sweep thresholds from high to low: cumulative TP / FP counts trace the ROC
        tp = np.concatenate([[0.0], np.cumsum(self._stat_pos[::-1])])
        fp = np.concatenate([[0.0], np.cumsum(self._stat_neg[::-1])])
        if tp[-1] <= 0 or fp[-1] <= 0:
            return 0.0
        area = np.sum((fp[1:] - fp[:-1]) * (tp[1:] + tp[:-1]) / 2.0)
        return float(area / tp[-1] / fp[-1])
