"""fluid.metrics behaviour (reference API: python/paddle/fluid/metrics.py)."""
import numpy as np
import pytest

from paddle_amd.fluid import metrics


def test_precision_recall_and_reset():
    preds = np.array([0.9, 0.2, 0.7, 0.6, 0.1])
    labels = np.array([1, 0, 0, 1, 1])
    p, r = metrics.Precision(), metrics.Recall()
    p.update(preds, labels)
    r.update(preds, labels)
    assert p.eval() == pytest.approx(2 / 3)   # predicted 1: idx 0, 2, 3 -> tp 2, fp 1
    assert r.eval() == pytest.approx(2 / 3)   # actual 1: idx 0, 3, 4 -> tp 2, fn 1
    assert p.get_config() == {"name": "Precision", "states": {"tp": 2, "fp": 1}}
    p.reset()
    assert (p.tp, p.fp, p.eval()) == (0, 0, 0.0)


def test_accuracy_chunk_edit_distance():
    a = metrics.Accuracy()
    a.update(np.array([0.5]), 2)
    a.update(1.0, 2)
    assert a.eval() == pytest.approx(0.75)
    with pytest.raises(ValueError):
        metrics.Accuracy().eval()
    c = metrics.ChunkEvaluator()
    c.update(np.array([4]), np.array([5]), np.array([3]))
    pr, rc, f1 = c.eval()
    assert (pr, rc) == (0.75, 0.6) and f1 == pytest.approx(2 * 0.75 * 0.6 / 1.35)
    e = metrics.EditDistance("ed")
    e.update(np.array([[0.0], [2.0], [1.0]]), 3)
    assert e.eval() == (1.0, pytest.approx(2 / 3))


def test_auc_matches_sklearn():
    sk = pytest.importorskip("sklearn.metrics")
    rng = np.random.default_rng(0)
    labels = rng.integers(0, 2, 4000)
    score = np.clip(labels * 0.3 + rng.random(4000) * 0.7, 0, 1)
    auc = metrics.Auc("auc", num_thresholds=4095)
    for i in range(0, 4000, 500):
        p = np.stack([1 - score[i:i + 500], score[i:i + 500]], 1)
        auc.update(p, labels[i:i + 500])
    # binning to 4096 thresholds changes the exact value by < 1e-3
    assert auc.eval() == pytest.approx(sk.roc_auc_score(labels, score), abs=1e-3)


def test_composite():
    comp = metrics.CompositeMetric()
    comp.add_metric(metrics.Precision())
    comp.add_metric(metrics.Recall())
    comp.update(np.array([1, 1, 0]), np.array([1, 0, 1]))
    assert comp.eval() == [0.5, 0.5]
    with pytest.raises(ValueError):
        comp.add_metric(object())
