"""ParamAttr / WeightNormParamAttr (python/paddle/fluid/param_attr.py)."""
from __future__ import annotations

from .initializer import ConstantInitializer, Initializer, XavierInitializer


class ParamAttr:
    def __init__(self, name=None, initializer=None, learning_rate=1.0, regularizer=None, trainable=True,
                 gradient_clip=None, do_model_average=False):
        self.name = name
        self.initializer = initializer
        self.learning_rate = learning_rate
        self.regularizer = regularizer
        self.trainable = trainable
        self.gradient_clip = gradient_clip
        self.model_average = do_model_average

    def _set_default_initializer(self, initializer):
        if initializer is None:
            raise ValueError("initializer should not be None")
        if self.initializer is None:
            self.initializer = initializer

    def _set_default_param_initializer(self):
        self._set_default_initializer(XavierInitializer())

    def _set_default_bias_initializer(self):
        self._set_default_initializer(ConstantInitializer(0.0))

    @staticmethod
    def _to_attr(arg):
        if arg is None:
            return ParamAttr()
        if isinstance(arg, (list, tuple)):
            return [ParamAttr._to_attr(a) for a in arg]
        if isinstance(arg, ParamAttr):
            return arg
        if isinstance(arg, str):
            return ParamAttr(name=arg)
        if isinstance(arg, Initializer):
            return ParamAttr(initializer=arg)
        if isinstance(arg, bool):
            return ParamAttr._to_attr(None) if arg else False
        if type(arg).__name__ == "ParameterAttribute":
            # the v1 DSL's attribute (trainer_config_helpers): name / std / mean / lr
            from .initializer import NormalInitializer

            init = None
            if getattr(arg, "initial_std", None) is not None or getattr(arg, "initial_mean", None) is not None:
                init = NormalInitializer(loc=float(arg.initial_mean or 0.0), scale=float(arg.initial_std or 0.0))
            lr = getattr(arg, "learning_rate", None)
            return ParamAttr(name=arg.name, initializer=init, learning_rate=1.0 if lr is None else float(lr))
        raise TypeError(f"{type(arg)} cast to ParamAttr")

    def _to_kwargs(self, with_initializer=False):
        kw = {"name": self.name, "optimize_attr": {"learning_rate": self.learning_rate},
              "regularizer": self.regularizer, "trainable": self.trainable,
              "gradient_clip_attr": self.gradient_clip, "do_model_average": self.model_average}
        if with_initializer:
            kw["initializer"] = self.initializer
        return kw


class WeightNormParamAttr(ParamAttr):
    params_with_weight_norm = []

    def __init__(self, dim=None, **kwargs):
        super().__init__(**kwargs)
        self.dim = dim
