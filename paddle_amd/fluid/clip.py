"""Gradient / error clipping (python/paddle/fluid/clip.py)."""
from __future__ import annotations

import copy

from ..framework import registry as R
from . import layers as _layers_mod  # noqa: F401  (ensures layer registry import order)
from .framework import Parameter, default_main_program


class BaseErrorClipAttr:
    def _append_clip_op(self, block, grad_name):
        raise NotImplementedError()


class ErrorClipByValue(BaseErrorClipAttr):
    def __init__(self, max, min=None):
        max = float(max)
        min = -max if min is None else float(min)
        self.max, self.min = max, min

    def _append_clip_op(self, block, grad_name):
        block.append_op(type="clip", inputs={"X": [grad_name]}, outputs={"Out": [grad_name]},
                        attrs={"min": self.min, "max": self.max})


def error_clip_callback(block, context):
    op = block.ops[-1]
    for grad_n in [n for n in op.output_arg_names if n.endswith(R.GRAD_SUFFIX)]:
        fwd = block._find_var_recursive(grad_n[:-len(R.GRAD_SUFFIX)])
        ec = getattr(fwd, "error_clip", None) if fwd is not None else None
        if ec is not None:
            ec._append_clip_op(block, grad_n)


class BaseGradientClipAttr:
    def _process_context(self, context, param, grad):
        raise NotImplementedError()

    def _create_operators(self, param, grad):
        raise NotImplementedError()


class NullGradientClipAttr(BaseGradientClipAttr):
    def _process_context(self, context, param, grad):
        pass

    def _create_operators(self, param, grad):
        return param, grad


class GradientClipByValue(BaseGradientClipAttr):
    def __init__(self, max, min=None):
        max = float(max)
        self.max, self.min = max, (-max if min is None else float(min))

    def _process_context(self, context, param, grad):
        pass

    def _create_operators(self, param, grad):
        from .layers import nn

        return param, nn.clip(x=grad, min=self.min, max=self.max)


class GradientClipByNorm(BaseGradientClipAttr):
    def __init__(self, clip_norm):
        self.clip_norm = clip_norm

    def _process_context(self, context, param, grad):
        pass

    def _create_operators(self, param, grad):
        from .layers import nn

        return param, nn.clip_by_norm(x=grad, max_norm=self.clip_norm)


class GradientClipByGlobalNorm(BaseGradientClipAttr):
    def __init__(self, clip_norm, group_name="default_group"):
        self.clip_norm = float(clip_norm)
        self.group_name = group_name

    def _process_context(self, context, param, grad):
        from .layers import nn

        if self.group_name not in context:
            context[self.group_name] = []
            context[self.group_name + "_clip_value"] = self.clip_norm
        local = nn.reduce_sum(input=nn.pow(x=grad, factor=2.0))
        context[self.group_name].append(local)
        self.context = context

    def _create_operators(self, param, grad):
        from .layers import nn, tensor

        scale_var = self.group_name + "_scale"
        if scale_var not in self.context:
            gn = nn.sqrt(x=nn.sums(input=self.context[self.group_name]))
            cv = tensor.fill_constant(shape=[1], dtype="float32", value=self.clip_norm)
            self.context[scale_var] = nn.elementwise_div(x=cv, y=nn.elementwise_max(x=cv, y=gn))
        new_grad = nn.elementwise_mul(x=grad, y=self.context[scale_var])
        return param, new_grad


def set_gradient_clip(clip, param_list=None, program=None):
    if program is None:
        program = default_main_program()
    if param_list is None:
        param_list = program.global_block().all_parameters()
    if all(isinstance(e, str) for e in param_list):
        param_list = [program.global_block().var(e) for e in param_list]
    for p in param_list:
        p.gradient_clip_attr = copy.deepcopy(clip)


def append_gradient_clip_ops(param_grads):
    context = dict()
    for p, g in param_grads:
        if g is None:
            continue
        with p.block.program.optimized_guard([p, g]):
            clip_attr = getattr(p, "gradient_clip_attr", None) or NullGradientClipAttr()
            clip_attr._process_context(context=context, param=p, grad=g)
    res = []
    for p, g in param_grads:
        if g is None:
            res.append((p, g))
            continue
        with p.block.program.optimized_guard([p, g]):
            clip_attr = getattr(p, "gradient_clip_attr", None) or NullGradientClipAttr()
            res.append(clip_attr._create_operators(param=p, grad=g))
    return res


ClipByValue = GradientClipByValue
ClipByNorm = GradientClipByNorm
ClipByGlobalNorm = GradientClipByGlobalNorm
