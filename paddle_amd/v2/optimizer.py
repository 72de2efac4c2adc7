"""v2 optimizers and regularisation (reference v2/optimizer.py), each lowered to the
Fluid optimizer of the same update rule."""
from .. import fluid


class L2Regularization:
    def __init__(self, rate):
        self.rate = rate


class ModelAverage:
    def __init__(self, average_window, max_average_window=None):
        self.average_window, self.max_average_window = average_window, max_average_window


class Optimizer:
    def __init__(self, learning_rate=1e-3, regularization=None, model_average=None, gradient_clipping_threshold=None,
                 **kw):
        self.learning_rate, self.regularization = learning_rate, regularization
        self.clip = gradient_clipping_threshold

    def _reg(self):
        return fluid.regularizer.L2Decay(self.regularization.rate) if self.regularization else None

    def to_fluid(self):
        raise NotImplementedError


class Momentum(Optimizer):
    def __init__(self, momentum=None, sparse=False, **kw):
        super().__init__(**kw)
        self.momentum = momentum or 0.0

    def to_fluid(self):
        if self.momentum == 0.0:
            return fluid.optimizer.SGD(self.learning_rate, regularization=self._reg())
        return fluid.optimizer.Momentum(self.learning_rate, self.momentum, regularization=self._reg())


class Adam(Optimizer):
    def __init__(self, beta1=0.9, beta2=0.999, epsilon=1e-8, **kw):
        super().__init__(**kw)
        self.b1, self.b2, self.eps = beta1, beta2, epsilon

    def to_fluid(self):
        return fluid.optimizer.Adam(self.learning_rate, self.b1, self.b2, self.eps, regularization=self._reg())


class Adamax(Adam):
    def to_fluid(self):
        return fluid.optimizer.Adamax(self.learning_rate, self.b1, self.b2, self.eps, regularization=self._reg())


class AdaGrad(Optimizer):
    def to_fluid(self):
        return fluid.optimizer.Adagrad(self.learning_rate, regularization=self._reg())


class DecayedAdaGrad(Optimizer):
    def __init__(self, rho=0.95, epsilon=1e-6, **kw):
        super().__init__(**kw)
        self.rho, self.eps = rho, epsilon

    def to_fluid(self):
        return fluid.optimizer.DecayedAdagrad(self.learning_rate, decay=self.rho, epsilon=self.eps,
                                              regularization=self._reg())


class AdaDelta(Optimizer):
    def __init__(self, rho=0.95, epsilon=1e-6, **kw):
        super().__init__(**kw)
        self.rho, self.eps = rho, epsilon

    def to_fluid(self):
        return fluid.optimizer.Adadelta(self.learning_rate, epsilon=self.eps, rho=self.rho,
                                        regularization=self._reg())


class RMSProp(Optimizer):
    def __init__(self, rho=0.95, epsilon=1e-6, **kw):
        super().__init__(**kw)
        self.rho, self.eps = rho, epsilon

    def to_fluid(self):
        return fluid.optimizer.RMSProp(self.learning_rate, rho=self.rho, epsilon=self.eps,
                                       regularization=self._reg())
