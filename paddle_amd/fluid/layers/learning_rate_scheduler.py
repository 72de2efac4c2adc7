"""Learning-rate schedules as graph ops on a global step counter
(python/paddle/fluid/layers/learning_rate_scheduler.py)."""
from __future__ import annotations

import math

from ..framework import default_main_program
from . import control_flow, nn, ops, tensor

__all__ = ["exponential_decay", "natural_exp_decay", "inverse_time_decay", "polynomial_decay",
           "piecewise_decay", "noam_decay", "append_LARS", "cosine_decay", "linear_lr_warmup"]


def _decay_step_counter(begin=0):
    with default_main_program()._lr_schedule_guard():
        c = tensor._global_step_counter("@LR_DECAY_COUNTER@", begin=begin, step=1)
        return tensor.cast(c, "float32")


def noam_decay(d_model, warmup_steps):
    with default_main_program()._lr_schedule_guard():
        step = _decay_step_counter(1)
        a = nn.pow(step, -0.5)
        b = nn.scale(step, scale=warmup_steps ** -1.5)
        return nn.scale(nn.elementwise_min(a, b), scale=d_model ** -0.5)


def exponential_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    with default_main_program()._lr_schedule_guard():
        step = _decay_step_counter()
        div = nn.scale(step, scale=1.0 / decay_steps)
        if staircase:
            div = ops.floor(div)
        rate = tensor.fill_constant([1], "float32", decay_rate)
        return nn.scale(nn.elementwise_pow(rate, div), scale=float(learning_rate))


def natural_exp_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    with default_main_program()._lr_schedule_guard():
        step = _decay_step_counter()
        div = nn.scale(step, scale=1.0 / decay_steps)
        if staircase:
            div = ops.floor(div)
        return nn.scale(ops.exp(nn.scale(div, scale=-decay_rate)), scale=float(learning_rate))


def inverse_time_decay(learning_rate, decay_steps, decay_rate, staircase=False):
    with default_main_program()._lr_schedule_guard():
        step = _decay_step_counter()
        div = nn.scale(step, scale=1.0 / decay_steps)
        if staircase:
            div = ops.floor(div)
        den = nn.scale(div, scale=decay_rate, bias=1.0)
        return nn.elementwise_div(tensor.fill_constant([1], "float32", learning_rate), den)


def polynomial_decay(learning_rate, decay_steps, end_learning_rate=0.0001, power=1.0, cycle=False):
    with default_main_program()._lr_schedule_guard():
        step = _decay_step_counter()
        ds = tensor.fill_constant([1], "float32", float(decay_steps))
        if cycle:
            div = ops.ceil(nn.scale(step, scale=1.0 / decay_steps))
            one = tensor.fill_constant([1], "float32", 1.0)
            div = nn.elementwise_max(div, one)
            ds = nn.scale(div, scale=float(decay_steps))
        else:
            step = nn.elementwise_min(step, ds)
        frac = nn.scale(nn.elementwise_div(step, ds), scale=-1.0, bias=1.0)
        return nn.scale(nn.pow(frac, power), scale=float(learning_rate - end_learning_rate),
                        bias=float(end_learning_rate))


def piecewise_decay(boundaries, values):
    with default_main_program()._lr_schedule_guard():
        if len(values) - len(boundaries) != 1:
            raise ValueError("len(values) - len(boundaries) should be 1")
        step = _decay_step_counter()
        lr = tensor.create_global_var(shape=[1], value=0.0, dtype="float32", persistable=True,
                                      name="learning_rate")
        with control_flow.Switch() as sw:
            for i in range(len(boundaries)):
                bv = tensor.fill_constant([1], "float32", float(boundaries[i]), force_cpu=True)
                with sw.case(control_flow.less_than(step, bv)):
                    tensor.assign(tensor.fill_constant([1], "float32", float(values[i])), lr)
            with sw.default():
                tensor.assign(tensor.fill_constant([1], "float32", float(values[-1])), lr)
        return lr


def cosine_decay(learning_rate, step_each_epoch, epochs):
    with default_main_program()._lr_schedule_guard():
        step = _decay_step_counter()
        epoch = ops.floor(nn.scale(step, scale=1.0 / step_each_epoch))
        c = ops.cos(nn.scale(epoch, scale=math.pi / epochs))
        return nn.scale(nn.scale(c, bias=1.0), scale=learning_rate * 0.5)


def linear_lr_warmup(learning_rate, warmup_steps, start_lr, end_lr):
    with default_main_program()._lr_schedule_guard():
        step = _decay_step_counter()
        ws = tensor.fill_constant([1], "float32", float(warmup_steps))
        frac = nn.elementwise_min(nn.elementwise_div(step, ws), tensor.fill_constant([1], "float32", 1.0))
        warm = nn.scale(frac, scale=end_lr - start_lr, bias=start_lr)
        if not hasattr(learning_rate, "name"):
            learning_rate = tensor.fill_constant([1], "float32", float(learning_rate))
        is_warm = control_flow.less_than(step, ws)
        w = tensor.cast(is_warm, "float32")
        return nn.elementwise_add(nn.elementwise_mul(w, warm),
                                  nn.elementwise_mul(nn.scale(w, scale=-1.0, bias=1.0), learning_rate))


def append_LARS(params_grads, learning_rate, weight_decay):
    for param, grad in params_grads:
        pn = ops.sqrt(nn.reduce_sum(ops.square(param)))
        gn = ops.sqrt(nn.reduce_sum(ops.square(grad)))
        decayed = nn.elementwise_div(nn.elementwise_mul(learning_rate, pn),
                                     nn.elementwise_add(gn, nn.scale(pn, scale=weight_decay)))
        param.optimize_attr["learning_rate"] = decayed
