"""paddle.metric: Accuracy, Precision, Recall, Auc (streaming) + ``accuracy``.

Reference parity: fluid/metrics.py (Accuracy, Precision, Recall, Auc,
ChunkEvaluator, EditDistance) and the ``accuracy`` / ``auc`` ops."""
from __future__ import annotations

import numpy as np
import torch


def accuracy(input, label, k=1, correct=None, total=None, name=None):
    topk = input.topk(k, -1).indices
    lab = label.reshape(-1, 1)
    return (topk == lab).any(-1).float().mean()


class Metric:
    def reset(self):
        raise NotImplementedError

    def update(self, *args):
        raise NotImplementedError

    def accumulate(self):
        raise NotImplementedError

    def name(self):
        return self._name

    def compute(self, *args):
        return args


class Accuracy(Metric):
    def __init__(self, topk=(1,), name=None):
        self.topk = tuple(topk) if isinstance(topk, (list, tuple)) else (topk,)
        self._name = name or "acc"
        self.reset()

    def compute(self, pred, label, *args):
        k = max(self.topk)
        idx = pred.topk(k, -1).indices
        return (idx == label.reshape(-1, 1)).float()

    def update(self, correct, *args):
        c = correct.cpu().numpy() if torch.is_tensor(correct) else np.asarray(correct)
        for i, k in enumerate(self.topk):
            self.total[i] += c[:, :k].any(-1).sum()
            self.count[i] += c.shape[0]
        return [float(c[:, :k].any(-1).mean()) for k in self.topk]

    def reset(self):
        self.total = [0.0] * len(self.topk)
        self.count = [0] * len(self.topk)

    def accumulate(self):
        r = [t / max(c, 1) for t, c in zip(self.total, self.count)]
        return r[0] if len(r) == 1 else r


class Precision(Metric):
    def __init__(self, name="precision"):
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = (np.asarray(preds.detach().cpu() if torch.is_tensor(preds) else preds).reshape(-1) > 0.5).astype(int)
        l = np.asarray(labels.detach().cpu() if torch.is_tensor(labels) else labels).reshape(-1).astype(int)
        self.tp += int(((p == 1) & (l == 1)).sum())
        self.fp += int(((p == 1) & (l == 0)).sum())

    def reset(self):
        self.tp = self.fp = 0

    def accumulate(self):
        return self.tp / (self.tp + self.fp) if self.tp + self.fp else 0.0


class Recall(Metric):
    def __init__(self, name="recall"):
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = (np.asarray(preds.detach().cpu() if torch.is_tensor(preds) else preds).reshape(-1) > 0.5).astype(int)
        l = np.asarray(labels.detach().cpu() if torch.is_tensor(labels) else labels).reshape(-1).astype(int)
        self.tp += int(((p == 1) & (l == 1)).sum())
        self.fn += int(((p == 0) & (l == 1)).sum())

    def reset(self):
        self.tp = self.fn = 0

    def accumulate(self):
        return self.tp / (self.tp + self.fn) if self.tp + self.fn else 0.0


class Auc(Metric):
    """Histogram ROC-AUC (the reference auc op's bucketed algorithm, num_thresholds buckets)."""

    def __init__(self, curve="ROC", num_thresholds=4095, name="auc"):
        self._name, self.n = name, num_thresholds
        self.reset()

    def update(self, preds, labels):
        p = np.asarray(preds.detach().cpu() if torch.is_tensor(preds) else preds)
        p = p[:, 1] if p.ndim == 2 and p.shape[1] == 2 else p.reshape(-1)
        l = np.asarray(labels.detach().cpu() if torch.is_tensor(labels) else labels).reshape(-1)
        b = np.clip((p * self.n).astype(int), 0, self.n)
        np.add.at(self.pos, b[l > 0], 1)
        np.add.at(self.neg, b[l <= 0], 1)

    def reset(self):
        self.pos = np.zeros(self.n + 1)
        self.neg = np.zeros(self.n + 1)

    def accumulate(self):
        tp = fp = 0.0
        area = 0.0
        for i in range(self.n, -1, -1):
            ntp, nfp = tp + self.pos[i], fp + self.neg[i]
            area += (nfp - fp) * (tp + ntp) / 2
            tp, fp = ntp, nfp
        return area / (tp * fp) if tp > 0 and fp > 0 else 0.0
