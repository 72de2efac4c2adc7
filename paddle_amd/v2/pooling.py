"""v2 sequence / image pooling types (reference v2/pooling.py)."""


class BasePool:
    seq = "AVERAGE"
    img = "avg"

    def __init__(self, output_max_index=None, strategy=None, **kw):
        # MaxPooling(output_max_index=True): the layer emits the arg-max index
        self.output_max_index = output_max_index
        self.strategy = strategy


class Max(BasePool):
    seq, img = "MAX", "max"


class Avg(BasePool):
    seq, img = "AVERAGE", "avg"


class Sum(BasePool):
    seq, img = "SUM", "avg"


class SquareRootN(BasePool):
    seq, img = "SQRT", "avg"
