"""``paddle.optimizer.lr`` learning-rate schedulers.

Reference parity: fluid ``layers/learning_rate_scheduler.py`` (noam_decay,
exponential_decay, natural_exp_decay, inverse_time_decay, polynomial_decay,
piecewise_decay, append_LARS) builds these as ops in the program; in DyGraph they
are host-side objects stepped once per iteration/epoch (Paddle 2.x semantics:
``last_epoch`` starts at -1 and the constructor performs the first ``step()``).
"""
from __future__ import annotations

import math


class LRScheduler:
    def __init__(self, learning_rate=0.1, last_epoch=-1, verbose=False):
        self.base_lr = float(learning_rate)
        self.last_lr = float(learning_rate)
        self.last_epoch = last_epoch
        self.verbose = verbose
        self.step()

    def __call__(self):
        return self.last_lr

    def get_lr(self):
        raise NotImplementedError

    def step(self, epoch=None):
        self.last_epoch = self.last_epoch + 1 if epoch is None else epoch
        self.last_lr = float(self.get_lr())

    def state_dict(self):
        return {k: v for k, v in self.__dict__.items() if isinstance(v, (int, float, bool, str, list))}

    def set_state_dict(self, sd):
        for k, v in sd.items():
            setattr(self, k, v)

    set_dict = set_state_dict


class NoamDecay(LRScheduler):
    def __init__(self, d_model, warmup_steps, learning_rate=1.0, last_epoch=-1, verbose=False):
        self.d_model, self.warmup_steps = d_model, warmup_steps
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        e = max(self.last_epoch, 1)
        return self.base_lr * self.d_model ** -0.5 * min(e ** -0.5, e * self.warmup_steps ** -1.5)


class PiecewiseDecay(LRScheduler):
    def __init__(self, boundaries, values, last_epoch=-1, verbose=False):
        self.boundaries, self.values = list(boundaries), list(values)
        super().__init__(values[0], last_epoch, verbose)

    def get_lr(self):
        for b, v in zip(self.boundaries, self.values):
            if self.last_epoch < b:
                return v
        return self.values[len(self.boundaries)]


class NaturalExpDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * math.exp(-self.gamma * self.last_epoch)


class InverseTimeDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr / (1 + self.gamma * self.last_epoch)


class PolynomialDecay(LRScheduler):
    def __init__(self, learning_rate, decay_steps, end_lr=0.0001, power=1.0, cycle=False, last_epoch=-1,
                 verbose=False):
        self.decay_steps, self.end_lr, self.power, self.cycle = decay_steps, end_lr, power, cycle
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        t, ds = self.last_epoch, self.decay_steps
        if self.cycle:
            ds = ds * max(1, math.ceil(t / ds)) if t > 0 else ds
        else:
            t = min(t, ds)
        return (self.base_lr - self.end_lr) * (1 - t / ds) ** self.power + self.end_lr


class LinearWarmup(LRScheduler):
    def __init__(self, learning_rate, warmup_steps, start_lr, end_lr, last_epoch=-1, verbose=False):
        self.inner = learning_rate if isinstance(learning_rate, LRScheduler) else None
        self.warmup_steps, self.start_lr, self.end_lr = warmup_steps, start_lr, end_lr
        super().__init__(end_lr if self.inner else learning_rate, last_epoch, verbose)

    def get_lr(self):
        if self.last_epoch < self.warmup_steps:
            return self.start_lr + (self.end_lr - self.start_lr) * self.last_epoch / self.warmup_steps
        if self.inner is not None:
            self.inner.step(self.last_epoch - self.warmup_steps)
            return self.inner()
        return self.base_lr


class ExponentialDecay(LRScheduler):
    def __init__(self, learning_rate, gamma, last_epoch=-1, verbose=False):
        self.gamma = gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * self.gamma ** self.last_epoch


class MultiStepDecay(LRScheduler):
    def __init__(self, learning_rate, milestones, gamma=0.1, last_epoch=-1, verbose=False):
        self.milestones, self.gamma = list(milestones), gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * self.gamma ** sum(1 for m in self.milestones if self.last_epoch >= m)


class StepDecay(LRScheduler):
    def __init__(self, learning_rate, step_size, gamma=0.1, last_epoch=-1, verbose=False):
        self.step_size, self.gamma = step_size, gamma
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * self.gamma ** (self.last_epoch // self.step_size)


class LambdaDecay(LRScheduler):
    def __init__(self, learning_rate, lr_lambda, last_epoch=-1, verbose=False):
        self.lr_lambda = lr_lambda
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.base_lr * self.lr_lambda(self.last_epoch)


class MultiplicativeDecay(LRScheduler):
    def __init__(self, learning_rate, lr_lambda, last_epoch=-1, verbose=False):
        self.lr_lambda = lr_lambda
        self._cur = float(learning_rate)
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        if self.last_epoch > 0:
            self._cur *= self.lr_lambda(self.last_epoch)
        return self._cur


class CosineAnnealingDecay(LRScheduler):
    def __init__(self, learning_rate, T_max, eta_min=0, last_epoch=-1, verbose=False):
        self.T_max, self.eta_min = T_max, eta_min
        super().__init__(learning_rate, last_epoch, verbose)

    def get_lr(self):
        return self.eta_min + (self.base_lr - self.eta_min) * (1 + math.cos(math.pi * self.last_epoch / self.T_max)) / 2


class OneCycleLR(LRScheduler):
    def __init__(self, max_learning_rate, total_steps, divide_factor=25.0, end_learning_rate=0.0001,
                 phase_pct=0.3, anneal_strategy="cos", three_phase=False, last_epoch=-1, verbose=False):
        self.max_lr, self.total = max_learning_rate, total_steps
        self.init_lr = max_learning_rate / divide_factor
        self.end_lr, self.pct, self.anneal = end_learning_rate, phase_pct, anneal_strategy
        super().__init__(self.init_lr, last_epoch, verbose)

    def _interp(self, a, b, t):
        if self.anneal == "cos":
            return b + (a - b) * (1 + math.cos(math.pi * t)) / 2
        return a + (b - a) * t

    def get_lr(self):
        up = self.pct * self.total
        t = self.last_epoch
        if t <= up:
            return self._interp(self.init_lr, self.max_lr, t / max(up, 1))
        return self._interp(self.max_lr, self.end_lr, (t - up) / max(self.total - up, 1))


class CyclicLR(LRScheduler):
    def __init__(self, base_learning_rate, max_learning_rate, step_size_up, step_size_down=None, mode="triangular",
                 exp_gamma=1.0, scale_fn=None, scale_mode="cycle", last_epoch=-1, verbose=False):
        self.max_lr, self.up = max_learning_rate, step_size_up
        self.down = step_size_down or step_size_up
        self.mode, self.gamma = mode, exp_gamma
        super().__init__(base_learning_rate, last_epoch, verbose)

    def get_lr(self):
        cyc = self.up + self.down
        c = self.last_epoch // cyc
        x = self.last_epoch - c * cyc
        frac = x / self.up if x < self.up else 1 - (x - self.up) / self.down
        amp = self.max_lr - self.base_lr
        if self.mode == "triangular2":
            amp /= 2 ** c
        elif self.mode == "exp_range":
            amp *= self.gamma ** self.last_epoch
        return self.base_lr + amp * frac


class ReduceOnPlateau(LRScheduler):
    def __init__(self, learning_rate, mode="min", factor=0.1, patience=10, threshold=1e-4, threshold_mode="rel",
                 cooldown=0, min_lr=0, epsilon=1e-8, verbose=False):
        self.mode, self.factor, self.patience = mode, factor, patience
        self.threshold, self.threshold_mode, self.cooldown = threshold, threshold_mode, cooldown
        self.min_lr, self.epsilon = min_lr, epsilon
        self.best = None
        self.num_bad, self.cooldown_counter = 0, 0
        self.base_lr = self.last_lr = float(learning_rate)
        self.last_epoch = 0
        self.verbose = verbose

    def _better(self, a, b):
        if b is None:
            return True
        t = self.threshold
        if self.mode == "min":
            return a < (b * (1 - t) if self.threshold_mode == "rel" else b - t)
        return a > (b * (1 + t) if self.threshold_mode == "rel" else b + t)

    def step(self, metrics=None, epoch=None):
        if metrics is None:
            return
        m = float(metrics)
        self.last_epoch += 1
        if self._better(m, self.best):
            self.best, self.num_bad = m, 0
        else:
            self.num_bad += 1
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.num_bad = 0
        if self.num_bad > self.patience:
            new = max(self.last_lr * self.factor, self.min_lr)
            if self.last_lr - new > self.epsilon:
                self.last_lr = new
            self.cooldown_counter = self.cooldown
            self.num_bad = 0
