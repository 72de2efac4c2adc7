"""v2 evaluators (reference v2/evaluator.py): metric Fluid variables fetched each
iteration and averaged over a pass / test run."""
from .. import fluid
from ._core import STATE, guard


def _register(name, var):
    STATE.setdefault("metrics", []).append((name, var))
    return var


def classification_error(input, label, name=None, top_k=1, **kw):
    with guard():
        acc = fluid.layers.accuracy(input=input, label=label, k=top_k)
        err = fluid.layers.scale(acc, scale=-1.0, bias=1.0)
    return _register(name or "classification_error_evaluator", err)


class _Metrics:
    def __init__(self, metrics):
        self.metrics = dict(metrics)
