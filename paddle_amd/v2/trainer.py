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
        self.metrics = list(STATE.get("metrics", []))

    def _feeder(self, feeding):
        names = list(STATE["data"])
        if feeding is not None:
            order = sorted(feeding.items(), key=lambda kv: kv[1]) if isinstance(feeding, dict) else \
                [(n, i) for i, n in enumerate(feeding)]
            names = [n for n, _ in order]
        block = STATE["main"].global_block()
        return fluid.DataFeeder(feed_list=[block.var(n) for n in names], place=place(), program=STATE["main"])

    def _run(self, program, feeder, batch):
        fetch = [self.cost] + [v for _, v in self.metrics]
        with fluid.scope_guard(STATE["scope"]):
            outs = executor().run(program, feed=feeder.feed(batch), fetch_list=fetch)
        vals = [float(np.array(o).ravel()[0]) for o in outs]
        return vals[0], {n: v for (n, _), v in zip(self.metrics, vals[1:])}

    def train(self, reader, num_passes=1, event_handler=None, feeding=None):
        handler = event_handler or (lambda e: None)
        feeder = self._feeder(feeding)
        for pass_id in range(num_passes):
            handler(E.BeginPass(pass_id))
            sums, n = {}, 0
            for batch_id, batch in enumerate(reader()):
                handler(E.BeginIteration(pass_id, batch_id))
                cost, met = self._run(STATE["main"], feeder, batch)
                for k, v in met.items():
                    sums[k] = sums.get(k, 0.0) + v
                n += 1
                handler(E.EndIteration(pass_id, batch_id, cost, _Eval(met)))
            handler(E.EndPass(pass_id, _Eval({k: v / max(n, 1) for k, v in sums.items()})))

    def test(self, reader, feeding=None):
        feeder = self._feeder(feeding)
        costs, sums, n = [], {}, 0
        for batch in reader():
            cost, met = self._run(self.test_program, feeder, batch)
            costs.append(cost * len(batch))
            n += len(batch)
            for k, v in met.items():
                sums[k] = sums.get(k, 0.0) + v * len(batch)
        return E.TestResult(_Eval({k: v / max(n, 1) for k, v in sums.items()}), sum(costs) / max(n, 1))

    def save_parameter_to_tar(self, f):
        self.parameters.to_tar(f)
