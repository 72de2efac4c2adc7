"""v2 parameter / extra-layer attributes (reference v2/attr.py ->
trainer_config_helpers/attrs.py), mapped onto fluid.ParamAttr."""
from .. import fluid


class Param:
    def __init__(self, name=None, initial_std=None, initial_mean=0.0, l2_rate=None, learning_rate=1.0,
                 is_static=False, initial_max=None, initial_min=None, **kw):
        self.name, self.initial_std, self.initial_mean = name, initial_std, initial_mean
        self.l2_rate, self.learning_rate, self.is_static = l2_rate, learning_rate, is_static
        self.initial_max, self.initial_min = initial_max, initial_min

    def to_fluid(self):
        init = None
        if self.initial_max is not None and self.initial_min is not None:  # uniform [min, max] (strategy 1)
            init = fluid.initializer.Uniform(low=self.initial_min, high=self.initial_max)
        elif self.initial_std is not None:
            init = fluid.initializer.Normal(loc=self.initial_mean, scale=self.initial_std)
        reg = fluid.regularizer.L2Decay(self.l2_rate) if self.l2_rate else None
        return fluid.ParamAttr(name=self.name, initializer=init, regularizer=reg, learning_rate=self.learning_rate,
                               trainable=not self.is_static)


class Extra:
    def __init__(self, drop_rate=None, **kw):
        self.drop_rate = drop_rate


ParamAttr = Param
ExtraAttr = ExtraLayerAttribute = Extra
ParameterAttribute = Param


def to_fluid(a):
    if a is None or a is True:
        return None
    if a is False:
        return False
    if isinstance(a, (list, tuple)):  # one attribute per input
        return [to_fluid(x) for x in a]
    return a.to_fluid() if isinstance(a, Param) else a
