"""v2 activations (reference v2/activation.py): names of the Fluid act attribute."""


class BaseActivation:
    name = None

    def __init__(self):
        pass


def _act(n):
    return type(n.title().replace("_", ""), (BaseActivation,), {"name": n})


Relu = _act("relu")
Tanh = _act("tanh")
Sigmoid = _act("sigmoid")
Softmax = _act("softmax")
Exp = _act("exp")
Abs = _act("abs")
Square = _act("square")
BRelu = _act("brelu")
SoftRelu = _act("soft_relu")
STanh = _act("stanh")
SequenceSoftmax = _act("sequence_softmax")
Log = _act("log")
Sqrt = _act("sqrt")
Reciprocal = _act("reciprocal")


class Linear(BaseActivation):
    name = None


Identity = Linear


def act_name(act):
    if act is None:
        return None
    return act.name if isinstance(act, BaseActivation) or isinstance(act, type) else act
