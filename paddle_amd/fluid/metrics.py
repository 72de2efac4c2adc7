"""Host-side streaming metrics (python/paddle/fluid/metrics.py)."""
from __future__ import annotations

import copy

import numpy as np

__all__ = ["MetricBase", "CompositeMetric", "Precision", "Recall", "Accuracy", "ChunkEvaluator", "EditDistance",
           "DetectionMAP", "Auc"]


def _is_numpy_(var):
    return isinstance(var, (np.ndarray, np.generic))


def _is_number_(var):
    return isinstance(var, (int, float, np.integer, np.floating)) or (isinstance(var, np.ndarray) and var.shape == (1,))


def _is_number_or_matrix_(var):
    return _is_number_(var) or isinstance(var, np.ndarray)


class MetricBase:
    def __init__(self, name):
        self._name = str(name) if name is not None else self.__class__.__name__

    def __str__(self):
        return self._name

    def reset(self):
        states = {a: v for a, v in self.__dict__.items() if not a.startswith("_")}
        for attr, value in states.items():
            if isinstance(value, int):
                setattr(self, attr, 0)
            elif isinstance(value, float):
                setattr(self, attr, 0.0)
            elif isinstance(value, (np.ndarray, np.generic)):
                setattr(self, attr, np.zeros_like(value))
            else:
                setattr(self, attr, None)

    def get_config(self):
        states = {a: v for a, v in self.__dict__.items() if not a.startswith("_")}
        config = {}
        config.update({"name": self._name, "states": copy.deepcopy(states)})
        return config

    def update(self, preds, labels):
        raise NotImplementedError()

    def eval(self):
        raise NotImplementedError()


class CompositeMetric(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self._metrics = []

    def add_metric(self, metric):
        if not isinstance(metric, MetricBase):
            raise ValueError("SubMetric should be inherit from MetricBase.")
        self._metrics.append(metric)

    def update(self, preds, labels):
        for m in self._metrics:
            m.update(preds, labels)

    def eval(self):
        return [m.eval() for m in self._metrics]


class Precision(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self.tp = 0
        self.fp = 0

    def update(self, preds, labels):
        preds = np.rint(np.asarray(preds)).astype("int32").reshape(-1)
        labels = np.asarray(labels).reshape(-1)
        for p, l in zip(preds, labels):
            if p == 1:
                if p == l:
                    self.tp += 1
                else:
                    self.fp += 1

    def eval(self):
        ap = self.tp + self.fp
        return float(self.tp) / ap if ap != 0 else 0.0


class Recall(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self.tp = 0
        self.fn = 0

    def update(self, preds, labels):
        preds = np.rint(np.asarray(preds)).astype("int32").reshape(-1)
        labels = np.asarray(labels).reshape(-1)
        for p, l in zip(preds, labels):
            if l == 1:
                if p == l:
                    self.tp += 1
                else:
                    self.fn += 1

    def eval(self):
        recall = self.tp + self.fn
        return float(self.tp) / recall if recall != 0 else 0.0


class Accuracy(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self.value = 0.0
        self.weight = 0.0

    def update(self, value, weight):
        if not _is_number_or_matrix_(value):
            raise ValueError("The 'value' must be a number(int, float) or a numpy ndarray.")
        self.value += float(np.asarray(value).reshape(-1)[0]) * weight
        self.weight += weight

    def eval(self):
        if self.weight == 0:
            raise ValueError("There is no data in Accuracy Metrics.")
        return self.value / self.weight


class ChunkEvaluator(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self.num_infer_chunks = 0
        self.num_label_chunks = 0
        self.num_correct_chunks = 0

    def update(self, num_infer_chunks, num_label_chunks, num_correct_chunks):
        self.num_infer_chunks += int(np.asarray(num_infer_chunks).reshape(-1)[0])
        self.num_label_chunks += int(np.asarray(num_label_chunks).reshape(-1)[0])
        self.num_correct_chunks += int(np.asarray(num_correct_chunks).reshape(-1)[0])

    def eval(self):
        precision = float(self.num_correct_chunks) / self.num_infer_chunks if self.num_infer_chunks else 0
        recall = float(self.num_correct_chunks) / self.num_label_chunks if self.num_label_chunks else 0
        f1 = float(2 * precision * recall) / (precision + recall) if self.num_correct_chunks else 0
        return precision, recall, f1


class EditDistance(MetricBase):
    def __init__(self, name):
        super().__init__(name)
        self.total_distance = 0.0
        self.seq_num = 0
        self.instance_error = 0

    def update(self, distances, seq_num):
        distances = np.asarray(distances)
        seq_right_count = np.sum(distances == 0)
        total_distance = np.sum(distances)
        self.seq_num += int(seq_num)
        self.instance_error += int(seq_num) - int(seq_right_count)
        self.total_distance += float(total_distance)

    def eval(self):
        if self.seq_num == 0:
            raise ValueError("There is no data in EditDistance Metric.")
        return self.total_distance / self.seq_num, self.instance_error / float(self.seq_num)


class DetectionMAP(MetricBase):
    def __init__(self, name=None):
        super().__init__(name)
        self.value = 0.0
        self.weight = 0.0

    def update(self, value, weight):
        self.value += float(np.asarray(value).reshape(-1)[0]) * weight
        self.weight += weight

    def eval(self):
        if self.weight == 0:
            raise ValueError("There is no data in DetectionMAP Metrics.")
        return self.value / self.weight


class Auc(MetricBase):
    def __init__(self, name, curve="ROC", num_thresholds=4095):
        super().__init__(name=name)
        self._curve = curve
        self._num_thresholds = num_thresholds
        self._stat_pos = [0] * (num_thresholds + 1)
        self._stat_neg = [0] * (num_thresholds + 1)

    def update(self, preds, labels):
        preds = np.asarray(preds)
        labels = np.asarray(labels).reshape(-1)
        for i, lbl in enumerate(labels):
            value = preds[i, 1] if preds.ndim > 1 else preds[i]
            bin_idx = int(value * self._num_thresholds)
            assert bin_idx <= self._num_thresholds
            if lbl:
                self._stat_pos[bin_idx] += 1.0
            else:
                self._stat_neg[bin_idx] += 1.0

    @staticmethod
    def trapezoid_area(x1, x2, y1, y2):
        return abs(x1 - x2) * (y1 + y2) / 2.0

    def eval(self):
        tot_pos = tot_neg = 0.0
        auc = 0.0
        idx = self._num_thresholds
        while idx >= 0:
            tot_pos_prev, tot_neg_prev = tot_pos, tot_neg
            tot_pos += self._stat_pos[idx]
            tot_neg += self._stat_neg[idx]
            auc += self.trapezoid_area(tot_neg, tot_neg_prev, tot_pos, tot_pos_prev)
            idx -= 1
        return auc / tot_pos / tot_neg if tot_pos > 0.0 and tot_neg > 0.0 else 0.0
