"""Static-graph optimizers (python/paddle/fluid/optimizer.py:38-1119).

``minimize`` = append_backward + gradient clip + regularization + one optimizer op
per parameter (role Optimize, op_role_var=[param, grad]).  Accumulators (moments,
beta powers) are persistable vars initialised in the startup program, so
``save_persistables`` checkpoints optimizer state exactly like the reference.
"""
from __future__ import annotations

from collections import defaultdict

from ..framework import core
from . import unique_name
from .backward import append_backward
from .clip import append_gradient_clip_ops, error_clip_callback
from .framework import Variable, default_main_program, default_startup_program, program_guard
from .initializer import ConstantInitializer
from .layer_helper import LayerHelper
from .regularizer import append_regularization_ops


class Optimizer:
    def __init__(self, learning_rate, regularization=None, LARS_weight_decay=0.0, name=None):
        if not isinstance(learning_rate, (float, int, Variable)):
            raise TypeError("learning rate should be float or Variable")
        self._name = name
        self.regularization = regularization
        self._learning_rate = learning_rate
        self._dtype = None
        self._learning_rate_map = {}
        self._accumulators = defaultdict(lambda: dict())
        self.helper = None
        self._LARS_weight_decay = LARS_weight_decay

    def _create_global_learning_rate(self):
        prog = default_main_program()
        lr = self._global_learning_rate(prog)
        if lr is not None:
            return
        if isinstance(self._learning_rate, Variable):
            self._learning_rate_map[prog] = self._learning_rate
            return
        name = unique_name.generate("learning_rate")
        helper = LayerHelper("global_learning_rate")
        v = helper.create_global_variable(name=name, persistable=True, shape=[1], dtype=self._dtype or
                                          core.VT.FP32)
        helper.set_variable_initializer(v, ConstantInitializer(float(self._learning_rate)))
        self._learning_rate_map[prog] = v

    def _global_learning_rate(self, program=None):
        if program is None:
            program = default_main_program()
        return self._learning_rate_map.get(program, None)

    def _append_optimize_op(self, block, param_and_grad):
        raise NotImplementedError()

    def _create_param_lr(self, param_and_grad):
        param = param_and_grad[0]
        plr = param.optimize_attr.get("learning_rate", 1.0) if hasattr(param, "optimize_attr") else 1.0
        glr = self._global_learning_rate()
        if plr == 1.0:
            return glr
        helper = LayerHelper("param_lr")
        out = helper.create_variable_for_type_inference(glr.dtype)
        helper.append_op(type="scale", inputs={"X": [glr]}, outputs={"Out": [out]}, attrs={"scale": float(plr)})
        return out

    def _create_accumulators(self, block, parameters):
        pass

    def _finish_update(self, block, parameters_and_grads):
        pass

    def _add_accumulator(self, name, param, dtype=None, fill_value=0.0, shape=None):
        if name in self._accumulators and param.name in self._accumulators[name]:
            raise Exception(f"Accumulator {name} already exists for parameter {param.name}")
        if shape is None:
            shape = param.shape
        helper = LayerHelper(self.__class__.__name__)
        var = helper.create_global_variable(name=unique_name.generate(param.name + "_" + name), persistable=True,
                                            dtype=dtype or param.dtype, type=param.type, shape=shape)
        helper.set_variable_initializer(var, ConstantInitializer(float(fill_value)))
        self._accumulators[name][param.name] = var
        return var

    def _get_accumulator(self, name, param):
        return self._accumulators[name][param.name]

    def _create_optimization_pass(self, parameters_and_grads, loss, startup_program=None):
        prog = loss.block.program
        self._dtype = loss.dtype
        optimize_ops = []
        with program_guard(prog, startup_program or default_startup_program()):
            global_block = prog.global_block()
            self.helper = LayerHelper(self.__class__.__name__)
            self._create_accumulators(global_block, [p[0] for p in parameters_and_grads if p[0].trainable])
            self._create_global_learning_rate()
            for param_and_grad in parameters_and_grads:
                if param_and_grad[1] is None:
                    continue
                with prog.optimized_guard(param_and_grad):
                    if param_and_grad[0].trainable:
                        optimize_ops.append(self._append_optimize_op(global_block, param_and_grad))
            with prog.optimized_guard([]):
                self._finish_update(global_block, parameters_and_grads)
        prog._version += 1
        return optimize_ops

    def backward(self, loss, startup_program=None, parameter_list=None, no_grad_set=None, callbacks=None):
        cbs = list(callbacks or []) + [error_clip_callback]
        return append_backward(loss, parameter_list, no_grad_set, cbs)

    def apply_gradients(self, params_grads):
        params_grads = sorted(params_grads, key=lambda x: x[0].name)
        params_grads = append_gradient_clip_ops(params_grads)
        params_grads = append_regularization_ops(params_grads, self.regularization)
        return params_grads

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        params_grads = self.backward(loss, startup_program, parameter_list, no_grad_set)
        params_grads = self.apply_gradients(params_grads)
        optimize_ops = self._create_optimization_pass(params_grads, loss, startup_program)
        return optimize_ops, params_grads


class SGDOptimizer(Optimizer):
    def __init__(self, learning_rate, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self.type = "sgd"

    def _append_optimize_op(self, block, pg):
        return block.append_op(type=self.type, inputs={"Param": pg[0], "Grad": pg[1],
                                                       "LearningRate": self._create_param_lr(pg)},
                               outputs={"ParamOut": pg[0]})


class MomentumOptimizer(Optimizer):
    _velocity_acc_str = "velocity"

    def __init__(self, learning_rate, momentum, use_nesterov=False, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self.type = "momentum"
        self._momentum, self._use_nesterov = momentum, bool(use_nesterov)

    def _create_accumulators(self, block, parameters):
        for p in parameters:
            self._add_accumulator(self._velocity_acc_str, p)

    def _append_optimize_op(self, block, pg):
        v = self._get_accumulator(self._velocity_acc_str, pg[0])
        return block.append_op(type=self.type, inputs={"Param": pg[0], "Grad": pg[1], "Velocity": v,
                                                       "LearningRate": self._create_param_lr(pg)},
                               outputs={"ParamOut": pg[0], "VelocityOut": v},
                               attrs={"mu": self._momentum, "use_nesterov": self._use_nesterov})


class LarsMomentumOptimizer(MomentumOptimizer):
    def __init__(self, learning_rate, momentum, lars_coeff=0.001, lars_weight_decay=0.0005, **kwargs):
        super().__init__(learning_rate, momentum, **kwargs)
        self.type = "lars_momentum"
        self._lars_coeff, self._lars_wd = lars_coeff, lars_weight_decay

    def _append_optimize_op(self, block, pg):
        v = self._get_accumulator(self._velocity_acc_str, pg[0])
        return block.append_op(type=self.type, inputs={"Param": pg[0], "Grad": pg[1], "Velocity": v,
                                                       "LearningRate": self._create_param_lr(pg)},
                               outputs={"ParamOut": pg[0], "VelocityOut": v},
                               attrs={"mu": self._momentum, "lars_coeff": self._lars_coeff,
                                      "lars_weight_decay": self._lars_wd})


class AdagradOptimizer(Optimizer):
    _moment_acc_str = "moment"

    def __init__(self, learning_rate, epsilon=1.0e-6, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self.type = "adagrad"
        self._epsilon = epsilon

    def _create_accumulators(self, block, parameters):
        for p in parameters:
            self._add_accumulator(self._moment_acc_str, p)

    def _append_optimize_op(self, block, pg):
        m = self._get_accumulator(self._moment_acc_str, pg[0])
        return block.append_op(type=self.type, inputs={"Param": pg[0], "Grad": pg[1], "Moment": m,
                                                       "LearningRate": self._create_param_lr(pg)},
                               outputs={"ParamOut": pg[0], "MomentOut": m}, attrs={"epsilon": self._epsilon})


class AdamOptimizer(Optimizer):
    _moment1_acc_str = "moment1"
    _moment2_acc_str = "moment2"
    _beta1_pow_acc_str = "beta1_pow_acc"
    _beta2_pow_acc_str = "beta2_pow_acc"

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, lazy_mode=False, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self.type = "adam"
        self._beta1, self._beta2, self._epsilon, self._lazy_mode = beta1, beta2, epsilon, lazy_mode

    def _create_accumulators(self, block, parameters):
        for p in parameters:
            self._add_accumulator(self._moment1_acc_str, p)
            self._add_accumulator(self._moment2_acc_str, p)
            self._add_accumulator(self._beta1_pow_acc_str, p, fill_value=self._beta1, shape=[1])
            self._add_accumulator(self._beta2_pow_acc_str, p, fill_value=self._beta2, shape=[1])

    def _append_optimize_op(self, block, pg):
        p = pg[0]
        m1 = self._get_accumulator(self._moment1_acc_str, p)
        m2 = self._get_accumulator(self._moment2_acc_str, p)
        b1 = self._get_accumulator(self._beta1_pow_acc_str, p)
        b2 = self._get_accumulator(self._beta2_pow_acc_str, p)
        return block.append_op(type=self.type,
                               inputs={"Param": p, "Grad": pg[1], "LearningRate": self._create_param_lr(pg),
                                       "Moment1": m1, "Moment2": m2, "Beta1Pow": b1, "Beta2Pow": b2},
                               outputs={"ParamOut": p, "Moment1Out": m1, "Moment2Out": m2},
                               attrs={"beta1": self._beta1, "beta2": self._beta2, "epsilon": self._epsilon,
                                      "lazy_mode": self._lazy_mode})

    def _finish_update(self, block, parameters_and_grads):
        for p, g in parameters_and_grads:
            if g is None or not p.trainable:
                continue
            with p.block.program.optimized_guard([p, g]):
                b1 = self._get_accumulator(self._beta1_pow_acc_str, p)
                b2 = self._get_accumulator(self._beta2_pow_acc_str, p)
                block.append_op(type="scale", inputs={"X": b1}, outputs={"Out": b1}, attrs={"scale": self._beta1})
                block.append_op(type="scale", inputs={"X": b2}, outputs={"Out": b2}, attrs={"scale": self._beta2})


class AdamaxOptimizer(Optimizer):
    _moment_acc_str = "moment"
    _inf_norm_acc_str = "inf_norm"
    _beta1_pow_acc_str = "beta1_pow_acc"

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self.type = "adamax"
        self._beta1, self._beta2, self._epsilon = beta1, beta2, epsilon

    def _create_accumulators(self, block, parameters):
        for p in parameters:
            self._add_accumulator(self._moment_acc_str, p)
            self._add_accumulator(self._inf_norm_acc_str, p)
            self._add_accumulator(self._beta1_pow_acc_str, p, fill_value=self._beta1, shape=[1])

    def _append_optimize_op(self, block, pg):
        p = pg[0]
        m = self._get_accumulator(self._moment_acc_str, p)
        u = self._get_accumulator(self._inf_norm_acc_str, p)
        b1 = self._get_accumulator(self._beta1_pow_acc_str, p)
        return block.append_op(type=self.type, inputs={"Param": p, "Grad": pg[1],
                                                       "LearningRate": self._create_param_lr(pg),
                                                       "Moment": m, "InfNorm": u, "Beta1Pow": b1},
                               outputs={"ParamOut": p, "MomentOut": m, "InfNormOut": u},
                               attrs={"beta1": self._beta1, "beta2": self._beta2, "epsilon": self._epsilon})

    def _finish_update(self, block, parameters_and_grads):
        for p, g in parameters_and_grads:
            if g is None or not p.trainable:
                continue
            b1 = self._get_accumulator(self._beta1_pow_acc_str, p)
            block.append_op(type="scale", inputs={"X": b1}, outputs={"Out": b1}, attrs={"scale": self._beta1})


class DecayedAdagradOptimizer(Optimizer):
    _moment_acc_str = "moment"

    def __init__(self, learning_rate, decay=0.95, epsilon=1.0e-6, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self.type = "decayed_adagrad"
        self._decay, self._epsilon = decay, epsilon

    def _create_accumulators(self, block, parameters):
        for p in parameters:
            self._add_accumulator(self._moment_acc_str, p)

    def _append_optimize_op(self, block, pg):
        m = self._get_accumulator(self._moment_acc_str, pg[0])
        return block.append_op(type=self.type, inputs={"Param": pg[0], "Grad": pg[1], "Moment": m,
                                                       "LearningRate": self._create_param_lr(pg)},
                               outputs={"ParamOut": pg[0], "MomentOut": m},
                               attrs={"epsilon": self._epsilon, "decay": self._decay})


class AdadeltaOptimizer(Optimizer):
    _avg_squared_grad_acc_str = "_avg_squared_grad"
    _avg_squared_update_acc_str = "_avg_squared_update"

    def __init__(self, learning_rate, epsilon=1.0e-6, rho=0.95, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self.type = "adadelta"
        self._epsilon, self._rho = epsilon, rho

    def _create_accumulators(self, block, parameters):
        for p in parameters:
            self._add_accumulator(self._avg_squared_grad_acc_str, p)
            self._add_accumulator(self._avg_squared_update_acc_str, p)

    def _append_optimize_op(self, block, pg):
        g = self._get_accumulator(self._avg_squared_grad_acc_str, pg[0])
        u = self._get_accumulator(self._avg_squared_update_acc_str, pg[0])
        return block.append_op(type=self.type, inputs={"Param": pg[0], "Grad": pg[1], "AvgSquaredGrad": g,
                                                       "AvgSquaredUpdate": u},
                               outputs={"ParamOut": pg[0], "AvgSquaredGradOut": g, "AvgSquaredUpdateOut": u},
                               attrs={"epsilon": self._epsilon, "rho": self._rho})


class RMSPropOptimizer(Optimizer):
    _momentum_acc_str = "momentum"
    _mean_square_acc_str = "mean_square"
    _mean_grad_acc_str = "mean_grad"

    def __init__(self, learning_rate, rho=0.95, epsilon=1.0e-6, momentum=0.0, centered=False, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self.type = "rmsprop"
        self._rho, self._epsilon, self._momentum, self._centered = rho, epsilon, momentum, centered

    def _create_accumulators(self, block, parameters):
        for p in parameters:
            self._add_accumulator(self._momentum_acc_str, p)
            self._add_accumulator(self._mean_square_acc_str, p)
            self._add_accumulator(self._mean_grad_acc_str, p)

    def _append_optimize_op(self, block, pg):
        mo = self._get_accumulator(self._momentum_acc_str, pg[0])
        ms = self._get_accumulator(self._mean_square_acc_str, pg[0])
        mg = self._get_accumulator(self._mean_grad_acc_str, pg[0])
        return block.append_op(type=self.type, inputs={"Param": pg[0], "Grad": pg[1], "Moment": mo,
                                                       "MeanSquare": ms, "MeanGrad": mg,
                                                       "LearningRate": self._create_param_lr(pg)},
                               outputs={"ParamOut": pg[0], "MomentOut": mo, "MeanSquareOut": ms,
                                        "MeanGradOut": mg},
                               attrs={"epsilon": self._epsilon, "decay": self._rho, "momentum": self._momentum,
                                      "centered": self._centered})


class FtrlOptimizer(Optimizer):
    _squared_acc_str = "squared"
    _linear_acc_str = "linear"

    def __init__(self, learning_rate, l1=0.0, l2=0.0, lr_power=-0.5, **kwargs):
        super().__init__(learning_rate=learning_rate, **kwargs)
        self.type = "ftrl"
        self._l1, self._l2, self._lr_power = l1, l2, lr_power

    def _create_accumulators(self, block, parameters):
        for p in parameters:
            self._add_accumulator(self._squared_acc_str, p)
            self._add_accumulator(self._linear_acc_str, p)

    def _append_optimize_op(self, block, pg):
        sq = self._get_accumulator(self._squared_acc_str, pg[0])
        li = self._get_accumulator(self._linear_acc_str, pg[0])
        return block.append_op(type=self.type, inputs={"Param": pg[0], "Grad": pg[1], "SquaredAccumulator": sq,
                                                       "LinearAccumulator": li,
                                                       "LearningRate": self._create_param_lr(pg)},
                               outputs={"ParamOut": pg[0], "SquaredAccumOut": sq, "LinearAccumOut": li},
                               attrs={"l1": self._l1, "l2": self._l2, "lr_power": self._lr_power})


class ModelAverage(Optimizer):
    """Accumulates parameter sums during training; ``apply()`` swaps in the averages
    (optimizer.py ModelAverage; average_accumulates op)."""

    def __init__(self, average_window_rate, min_average_window=10000, max_average_window=10000, **kwargs):
        super().__init__(0.0, **kwargs)
        self.average_window = average_window_rate
        self.min_average_window = min_average_window
        self.max_average_window = max_average_window
        self.params_grads = []
        main = default_main_program()
        for p in main.global_block().all_parameters():
            if p.do_model_average is not False:
                self.params_grads.append((p, None))
        for p, _ in self.params_grads:
            self._append_average_accumulate_op(p)

    def _append_average_accumulate_op(self, param):
        block = default_main_program().global_block()
        s1 = self._add_accumulator("sum_1", param)
        s2 = self._add_accumulator("sum_2", param)
        s3 = self._add_accumulator("sum_3", param)
        na = self._add_accumulator("num_accumulates", param, dtype=core.VT.INT64, shape=[1])
        ona = self._add_accumulator("old_num_accumulates", param, dtype=core.VT.INT64, shape=[1])
        nu = self._add_accumulator("num_updates", param, dtype=core.VT.INT64, shape=[1])
        block.append_op(type="average_accumulates",
                        inputs={"param": param, "in_sum_1": s1, "in_sum_2": s2, "in_sum_3": s3,
                                "in_num_accumulates": na, "in_old_num_accumulates": ona, "in_num_updates": nu},
                        outputs={"out_sum_1": s1, "out_sum_2": s2, "out_sum_3": s3, "out_num_accumulates": na,
                                 "out_old_num_accumulates": ona, "out_num_updates": nu},
                        attrs={"average_window": self.average_window,
                               "min_average_window": self.min_average_window,
                               "max_average_window": self.max_average_window})

    def apply(self, executor, need_restore=True):
        import contextlib
        import torch

        scope = core.global_scope()

        @contextlib.contextmanager
        def _ctx():
            backups = {}
            for p, _ in self.params_grads:
                pv = scope.find_var(p.name).get_tensor()
                s = [scope.find_var(self._get_accumulator(k, p).name).get_tensor().tensor
                     for k in ("sum_1", "sum_2", "sum_3")]
                n = [int(scope.find_var(self._get_accumulator(k, p).name).get_tensor().tensor.reshape(-1)[0])
                     for k in ("num_accumulates", "old_num_accumulates")]
                backups[p.name] = pv.tensor.clone()
                tot = max(1, n[0] + n[1])
                pv.set_tensor(((s[0] + s[1] + s[2]) / tot).to(pv.tensor.dtype))
            try:
                yield
            finally:
                if need_restore:
                    for p, _ in self.params_grads:
                        scope.find_var(p.name).get_tensor().set_tensor(backups[p.name])

        return _ctx()

    def restore(self, executor):
        pass


SGD = SGDOptimizer
Momentum = MomentumOptimizer
Adagrad = AdagradOptimizer
Adam = AdamOptimizer
Adamax = AdamaxOptimizer
DecayedAdagrad = DecayedAdagradOptimizer
Adadelta = AdadeltaOptimizer
RMSProp = RMSPropOptimizer
Ftrl = FtrlOptimizer
LarsMomentum = LarsMomentumOptimizer
