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


def _server_opt(update_equation):
    """OptimizationConfig (+ per-parameter momentum) of a v2 optimizer for the
    block-sharded parameter servers (distributed/pserver2.py)."""
    from . import optimizer as O

    oc = {"algorithm": "sgd", "learning_rate": float(update_equation.learning_rate)}
    mu = 0.0
    if isinstance(update_equation, O.Adam):
        oc.update(learning_method="adam", adam_beta1=update_equation.b1, adam_beta2=update_equation.b2,
                  adam_epsilon=update_equation.eps)
    elif isinstance(update_equation, O.AdaGrad):
        oc["learning_method"] = "adagrad"
    elif isinstance(update_equation, O.AdaDelta):
        oc.update(learning_method="adadelta", ada_rou=update_equation.rho, ada_epsilon=update_equation.eps)
    elif isinstance(update_equation, O.Momentum):
        oc["learning_method"] = "momentum"
        mu = float(update_equation.momentum)
    else:
        raise ValueError(f"remote training: {type(update_equation).__name__} has no server-side update rule")
    if update_equation.regularization is not None:
        oc["l2weight"] = float(update_equation.regularization.rate)
    return oc, mu


class SGD:
    """``is_local=False`` (with ``pserver_spec="host:port,..."``, ``trainer_id``): the
    update runs on the block-sharded parameter servers (ParameterServer2 protocol,
    distributed/pserver2.py): each batch's gradients go out as ADD_GRADIENT (the
    servers average over the trainers and apply the optimizer once) and the new
    values come back -- the reference's remote updater of ``is_local=False,
    use_etcd=False``."""

    def __init__(self, cost, parameters, update_equation, extra_layers=None, is_local=True, **kw):
        self.cost, self.parameters = cost, parameters
        self.test_program = STATE["main"].clone(for_test=True)
        self._client = None
        if not is_local:
            if not kw.get("pserver_spec"):
                raise ValueError("SGD(is_local=False) needs pserver_spec='host:port,...'")
            with guard():
                self._pg = fluid.backward.append_backward(cost)
        else:
            with guard():
                update_equation.to_fluid().minimize(cost)
        # the optimizer added accumulators to the startup program: run it again
        # with the trained parameters kept
        snap = parameters.snapshot()
        with fluid.scope_guard(STATE["scope"]):
            executor().run(STATE["startup"])
        parameters.restore(snap)
        self.evaluators = list(STATE.get("evaluators", []))
        if not is_local:
            from ..distributed.pserver2 import ParameterClient2

            oc, mu = _server_opt(update_equation)
            self._names = [p.name for p, g in self._pg if g is not None]
            self._grads = [g for p, g in self._pg if g is not None]
            self._client = ParameterClient2(kw["pserver_spec"], trainer_id=int(kw.get("trainer_id", 0)))
            got = self._client.init({n: np.asarray(parameters[n], np.float32) for n in self._names},
                                    param_configs={n: {"momentum": mu} for n in self._names}, opt_config=oc)
            for n, v in got.items():
                parameters[n] = v

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
        remote = self._client is not None and program is STATE["main"]
        if remote:
            fetch = fetch + self._grads
        from ..utils.stat import global_stat

        with fluid.scope_guard(STATE["scope"]), global_stat.timer("forwardBackward"):
            outs = executor().run(program, feed=feeder.feed(batch), fetch_list=fetch)
        outs = [np.array(o) for o in outs]
        if remote:
            grads = outs[len(outs) - len(self._grads):]
            outs = outs[:len(outs) - len(self._grads)]
            with global_stat.timer("sendAndReceiveParameter"):
                new = self._client.add_gradient(dict(zip(self._names, grads)), num_samples=len(batch),
                                                cost=float(outs[0].ravel()[0]))
            for n, v in new.items():
                self.parameters[n] = v
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
