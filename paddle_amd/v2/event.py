"""v2 training events (reference v2/event.py)."""


class WithMetric:
    def __init__(self, evaluator):
        self.evaluator = evaluator

    @property
    def metrics(self):
        return dict(self.evaluator.metrics) if self.evaluator is not None else {}


class TestResult(WithMetric):
    def __init__(self, evaluator, cost):
        super().__init__(evaluator)
        self.cost = cost


class BeginPass:
    def __init__(self, pass_id):
        self.pass_id = pass_id


class EndPass(WithMetric):
    def __init__(self, pass_id, evaluator, gm=None):
        super().__init__(evaluator)
        self.pass_id = pass_id
        self.gm = gm


class BeginIteration:
    def __init__(self, pass_id, batch_id):
        self.pass_id, self.batch_id = pass_id, batch_id


class EndForwardBackward:
    def __init__(self, pass_id, batch_id, gm=None):
        self.pass_id, self.batch_id, self.gm = pass_id, batch_id, gm


class EndIteration(WithMetric):
    def __init__(self, pass_id, batch_id, cost, evaluator, gm=None):
        super().__init__(evaluator)
        self.pass_id, self.batch_id, self.cost, self.gm = pass_id, batch_id, cost, gm
