"""v2 ``trainer.SGD`` (reference v2/trainer.py:37-250): owns the optimizer step of
the topology, feeds minibatches from a reader (``feeding`` maps data-layer names
to sample fields), fires BeginPass / BeginIteration / EndIteration / EndPass
events with the evaluator metrics, and tests on a program cloned before the
backward pass."""
from __future__ import annotations

import numpy as np

from .. import fluid
from . import event as E
from ._core import STATE, executor, guard, place


class _Eval:
    def __init__(self, metrics):
        self.metrics = metrics


class SGD:
    def __init__(self, cost, parameters, update_equation, extra_layers=None, is_local=True, **kw):
        self.cost, self.parameters = cost, parameters
        self.test_program = STATE["main"].clone(for_test=True)
        with guard():
            update_equation.to_fluid().minimize(cost)
        # the optimizer added accumulators to the startup program: run it again
        # with the trained parameters kept
        snap = parameters.snapshot()
        with fluid.scope_guard(STATE["scope"]):
            executor().run(STATE["startup"])
        parameters.restore(snap)
        self.evaluators = list(STATE.get("evaluators", []))

    def _feeder(self, feeding):
        names = list(STATE["data"])
        if feeding is not None:
            order = sorted(feeding.items(), key=lambda kv: kv[1]) if isinstance(feeding, dict) else \
                [(n, i) for i, n in enumerate(feeding)]
            names = [n for n, _ in order]
        block = STATE["main"].global_block()
        return fluid.DataFeeder(feed_list=[block.var(n) for n in names], place=place(), program=STATE["main"])

    def _run(self, program, feeder, batch):
        """One batch: fetch the cost and every evaluator's variables, feed the values
        to the evaluators (pass statistics) and return (cost, batch metrics)."""
        fetch = [self.cost] + [v for ev in self.evaluators for v in ev.fetch]
        with fluid.scope_guard(STATE["scope"]):
            outs = executor().run(program, feed=feeder.feed(batch), fetch_list=fetch)
        outs = [np.array(o) for o in outs]
        met, i = {}, 1
        for ev in self.evaluators:
            met.update(ev.eval(outs[i:i + len(ev.fetch)], len(batch)))
            i += len(ev.fetch)
        return float(outs[0].ravel()[0]), met

    def _pass_metrics(self):
        out = {}
        for ev in self.evaluators:
            out.update(ev.values())
        return out

    def _start(self):
        for ev in self.evaluators:
            ev.start()

    def train(self, reader, num_passes=1, event_handler=None, feeding=None):
        handler = event_handler or (lambda e: None)
        feeder = self._feeder(feeding)
        for pass_id in range(num_passes):
            handler(E.BeginPass(pass_id))
            self._start()
            for batch_id, batch in enumerate(reader()):
                handler(E.BeginIteration(pass_id, batch_id))
                cost, met = self._run(STATE["main"], feeder, batch)
                handler(E.EndIteration(pass_id, batch_id, cost, _Eval(met)))
            handler(E.EndPass(pass_id, _Eval(self._pass_metrics())))

    def test(self, reader, feeding=None):
        feeder = self._feeder(feeding)
        costs, n = [], 0
        self._start()
        for batch in reader():
            cost, _ = self._run(self.test_program, feeder, batch)
            costs.append(cost * len(batch))
            n += len(batch)
        res = E.TestResult(_Eval(self._pass_metrics()), sum(costs) / max(n, 1))
        self._start()
        return res

    def save_parameter_to_tar(self, f):
        self.parameters.to_tar(f)
