"""v2 sequence / image pooling types (reference v2/pooling.py)."""


class BasePool:
    seq = "AVERAGE"
    img = "avg"

    def __init__(self):
        pass


class Max(BasePool):
    seq, img = "MAX", "max"


class Avg(BasePool):
    seq, img = "AVERAGE", "avg"


class Sum(BasePool):
    seq, img = "SUM", "avg"


class SquareRootN(BasePool):
    seq, img = "SQRT", "avg"
