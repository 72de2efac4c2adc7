"""Optimizer update operators (one op per parameter, static-graph semantics).

Parity: paddle/fluid/operators/{sgd,momentum,lars_momentum,adam,adamax,adagrad,
decayed_adagrad,adadelta,rmsprop,ftrl,proximal_gd,proximal_adagrad,
average_accumulates}_op.* (SURVEY §2.7 "Optimizers").  Dense fp32 Adam / Momentum
on the HIP device run the fused gfx950 kernels (lr and beta-pow read from device
memory: no host sync); SelectedRows (sparse) gradients update only their rows.
When an output var is its input var (ParamOut == Param, Moment1Out == Moment1, as
the optimizer pass wires them) the update is in place, with no copies.
"""
from __future__ import annotations

import torch

from ..framework import core
from ..framework.op_kernel_type import LibraryType, register_op_kernel
from ..framework.registry import OP_REGISTRY, register_op
from ..ops import oplib as _oplib
from ..ops import optim as fopt


def _grad(ctx):
    return ctx.input_value("Grad")


def _lr(ctx):
    return ctx.input("LearningRate").reshape(-1)[0:1]


def _inplace(ctx, in_slot, out_slot):
    """Out var is the In var (ParamOut == Param, the optimizer pass's wiring): the
    kernel may update the tensor in place, as the reference does (adam_op.h:223-321)."""
    op = ctx.op
    if op is None:
        return False
    try:
        i, o = op.input(in_slot), ctx.out_names.get(out_slot) or []
    except Exception:  # noqa: BLE001
        return False
    return len(i) == 1 and len(o) == 1 and i[0] == o[0]


def _buf(ctx, t, in_slot, out_slot):
    """The update target: ``t`` itself when updating in place, else a copy."""
    if t is None:
        return None
    return t if _inplace(ctx, in_slot, out_slot) and t.is_contiguous() else t.clone()


def _native(ctx, kind, p, g, states, outs, lr=True, in_slots=None, **h):
    """Run the fused optim_ext.hip update -- in place on every tensor whose Out var
    is its In var (``in_slots`` names the state inputs), on copies otherwise."""
    if not p.is_cuda:
        return False
    p2 = _buf(ctx, p, "Param", "ParamOut")
    in_slots = list(in_slots or [None] * len(states))
    s2 = [None if s is None else (_buf(ctx, s, si, so) if si and so else s.clone())
          for s, si, so in zip(states, in_slots, outs)]
    lr_t = ctx.input("LearningRate") if lr else None
    if _oplib.opt_update_(kind, p2, g, s2, lr_t, **h) is None:
        return False
    ctx.set_output("ParamOut", p2)
    for name, t in zip(outs, s2):
        if name is not None and t is not None:
            ctx.set_output(name, t)
    return True


@register_op("sgd", ["Param", "Grad", "LearningRate"], ["ParamOut"], {}, grad=None, no_infer=True)
def sgd(ctx):
    p = ctx.input("Param")
    g = _grad(ctx)
    if p.is_cuda:
        out = _buf(ctx, p, "Param", "ParamOut")
        if isinstance(g, core.SelectedRows):
            done = _oplib.sgd_sparse_(out, g.rows(), g.get_tensor().tensor, ctx.input("LearningRate"))
        else:
            done = _oplib.sgd_(out, g.tensor.to(p.dtype), ctx.input("LearningRate"))
        if done is not None:
            ctx.set_output("ParamOut", out)
            return
    lr = _lr(ctx).to(p.dtype)
    out = p.clone()
    if isinstance(g, core.SelectedRows):
        rows = torch.as_tensor(g.rows(), dtype=torch.long, device=p.device)
        out.index_add_(0, rows, -lr * g.get_tensor().tensor.to(p.dtype))
    else:
        out -= lr * g.tensor.to(p.dtype)
    ctx.set_output("ParamOut", out)


@register_op("momentum", ["Param", "Grad", "Velocity", "LearningRate"], ["ParamOut", "VelocityOut"],
             {"mu": 0.9, "use_nesterov": False}, grad=None, no_infer=True)
def momentum(ctx):
    p, v = ctx.input("Param"), ctx.input("Velocity")
    g = _grad(ctx)
    g = g.to_dense() if isinstance(g, core.SelectedRows) else g.tensor
    if p.is_cuda and p.dtype == torch.float32 and p.is_contiguous():
        p2, v2 = _buf(ctx, p, "Param", "ParamOut"), _buf(ctx, v, "Velocity", "VelocityOut")
        fopt.momentum_flat(p2.view(-1), g.contiguous().view(-1), v2.view(-1), lr=0.0,
                           lr_tensor=ctx.input("LearningRate"), mu=ctx.attr("mu"),
                           nesterov=ctx.attr("use_nesterov"))
    else:
        mu = ctx.attr("mu")
        lr = _lr(ctx).to(p.dtype)
        v2 = mu * v + g
        p2 = p - (g + mu * v2) * lr if ctx.attr("use_nesterov") else p - lr * v2
    ctx.set_output("ParamOut", p2)
    ctx.set_output("VelocityOut", v2)


@register_op("lars_momentum", ["Param", "Grad", "Velocity", "LearningRate"], ["ParamOut", "VelocityOut"],
             {"mu": 0.9, "lars_coeff": 0.001, "lars_weight_decay": 0.0005}, grad=None, no_infer=True)
def lars_momentum(ctx):
    p, v, g = ctx.input("Param"), ctx.input("Velocity"), _grad(ctx).tensor
    wd = ctx.attr("lars_weight_decay")
    lr = _lr(ctx)
    pn, gn = p.norm(), g.norm()
    local = lr * ctx.attr("lars_coeff") * pn / (gn + wd * pn + 1e-12)
    v2 = ctx.attr("mu") * v + local * (g + wd * p)
    ctx.set_output("ParamOut", p - v2)
    ctx.set_output("VelocityOut", v2)


@register_op("adam", ["Param", "Grad", "LearningRate", "Moment1", "Moment2", "Beta1Pow", "Beta2Pow"],
             ["ParamOut", "Moment1Out", "Moment2Out"],
             {"beta1": 0.9, "beta2": 0.999, "epsilon": 1e-8, "lazy_mode": False}, grad=None, no_infer=True)
def adam(ctx):
    p, m1, m2 = ctx.input("Param"), ctx.input("Moment1"), ctx.input("Moment2")
    b1, b2, eps = ctx.attr("beta1"), ctx.attr("beta2"), ctx.attr("epsilon")
    g = _grad(ctx)
    p2, m1o, m2o = (_buf(ctx, p, "Param", "ParamOut"), _buf(ctx, m1, "Moment1", "Moment1Out"),
                    _buf(ctx, m2, "Moment2", "Moment2Out"))
    if isinstance(g, core.SelectedRows):
        # sparse Adam: merge duplicate rows, update only touched rows (SparseAdamFunctor)
        rows = torch.as_tensor(g.rows(), dtype=torch.long, device=p.device)
        gv = g.get_tensor().tensor.to(p.dtype)
        uniq, inv = torch.unique(rows, return_inverse=True)
        gm = torch.zeros((uniq.shape[0],) + tuple(gv.shape[1:]), dtype=p.dtype, device=p.device).index_add_(0, inv, gv)
        lr = _lr(ctx).to(p.dtype)
        bp1, bp2 = ctx.input("Beta1Pow").reshape(-1)[0], ctx.input("Beta2Pow").reshape(-1)[0]
        mm = b1 * m1[uniq] + (1 - b1) * gm
        vv = b2 * m2[uniq] + (1 - b2) * gm * gm
        lr_t = lr * torch.sqrt(1 - bp2) / (1 - bp1)
        upd = p[uniq] - lr_t * mm / (torch.sqrt(vv) + eps)
        m1o[uniq], m2o[uniq], p2[uniq] = mm, vv, upd
    else:
        gt = g.tensor
        if p.is_cuda and p.dtype == torch.float32 and p.is_contiguous():
            fopt.adamw_flat(p2.view(-1), gt.contiguous().view(-1), m1o.view(-1), m2o.view(-1), lr=0.0,
                            beta1=b1, beta2=b2, eps=eps, weight_decay=0.0,
                            lr_tensor=ctx.input("LearningRate"), beta1_pow=ctx.input("Beta1Pow"),
                            beta2_pow=ctx.input("Beta2Pow"), lr_t_eps=True)
        else:
            lr = _lr(ctx).to(p.dtype)
            bp1, bp2 = ctx.input("Beta1Pow").reshape(-1)[0], ctx.input("Beta2Pow").reshape(-1)[0]
            m1o = b1 * m1 + (1 - b1) * gt
            m2o = b2 * m2 + (1 - b2) * gt * gt
            lr_t = lr * torch.sqrt(1 - bp2) / (1 - bp1)
            p2 = p - lr_t * m1o / (torch.sqrt(m2o) + eps)
    ctx.set_output("ParamOut", p2)
    ctx.set_output("Moment1Out", m1o)
    ctx.set_output("Moment2Out", m2o)


@register_op("adamax", ["Param", "Grad", "LearningRate", "Moment", "InfNorm", "Beta1Pow"],
             ["ParamOut", "MomentOut", "InfNormOut"], {"beta1": 0.9, "beta2": 0.999, "epsilon": 1e-8},
             grad=None, no_infer=True)
def adamax(ctx):
    p, m, u, g = ctx.input("Param"), ctx.input("Moment"), ctx.input("InfNorm"), _grad(ctx).tensor
    b1, b2, eps = ctx.attr("beta1"), ctx.attr("beta2"), ctx.attr("epsilon")
    lr, bp1 = _lr(ctx), ctx.input("Beta1Pow").reshape(-1)[0]
    m2 = b1 * m + (1 - b1) * g
    u2 = torch.maximum(b2 * u + eps, g.abs())
    ctx.set_output("ParamOut", p - lr / (1 - bp1) * m2 / u2)
    ctx.set_output("MomentOut", m2)
    ctx.set_output("InfNormOut", u2)


@register_op("adagrad", ["Param", "Grad", "Moment", "LearningRate"], ["ParamOut", "MomentOut"],
             {"epsilon": 1e-6}, grad=None, no_infer=True)
def adagrad(ctx):
    p, m = ctx.input("Param"), ctx.input("Moment")
    g = _grad(ctx)
    lr, eps = _lr(ctx), ctx.attr("epsilon")
    if isinstance(g, core.SelectedRows):
        rows = torch.as_tensor(g.rows(), dtype=torch.long, device=p.device)
        gv = g.get_tensor().tensor
        uniq, inv = torch.unique(rows, return_inverse=True)
        gm = torch.zeros((uniq.shape[0],) + tuple(gv.shape[1:]), dtype=p.dtype, device=p.device).index_add_(0, inv, gv)
        m2, p2 = m.clone(), p.clone()
        m2[uniq] = m[uniq] + gm * gm
        p2[uniq] = p[uniq] - lr * gm / (torch.sqrt(m2[uniq]) + eps)
    else:
        g = g.tensor
        p2, m2 = _buf(ctx, p, "Param", "ParamOut"), _buf(ctx, m, "Moment", "MomentOut")
        if p.is_cuda and _oplib.adagrad_(p2, g, m2, ctx.input("LearningRate"), eps) is not None:
            ctx.set_output("ParamOut", p2)
            ctx.set_output("MomentOut", m2)
            return
        m2 = m + g * g
        p2 = p - lr * g / (torch.sqrt(m2) + eps)
    ctx.set_output("ParamOut", p2)
    ctx.set_output("MomentOut", m2)


@register_op("decayed_adagrad", ["Param", "Grad", "Moment", "LearningRate"], ["ParamOut", "MomentOut"],
             {"decay": 0.95, "epsilon": 1e-6}, grad=None, no_infer=True)
def decayed_adagrad(ctx):
    p, m, g = ctx.input("Param"), ctx.input("Moment"), _grad(ctx).tensor
    d, eps, lr = ctx.attr("decay"), ctx.attr("epsilon"), _lr(ctx)
    m2 = d * m + (1 - d) * g * g
    ctx.set_output("ParamOut", p - lr * g / (torch.sqrt(m2) + eps))
    ctx.set_output("MomentOut", m2)


@register_op("adadelta", ["Param", "Grad", "AvgSquaredGrad", "AvgSquaredUpdate"],
             ["ParamOut", "AvgSquaredGradOut", "AvgSquaredUpdateOut"], {"rho": 0.95, "epsilon": 1e-6},
             grad=None, no_infer=True)
def adadelta(ctx):
    p, g = ctx.input("Param"), _grad(ctx).tensor
    ag, au = ctx.input("AvgSquaredGrad"), ctx.input("AvgSquaredUpdate")
    rho, eps = ctx.attr("rho"), ctx.attr("epsilon")
    ag2 = rho * ag + (1 - rho) * g * g
    upd = -torch.sqrt((au + eps) / (ag2 + eps)) * g
    au2 = rho * au + (1 - rho) * upd * upd
    ctx.set_output("ParamOut", p + upd)
    ctx.set_output("AvgSquaredGradOut", ag2)
    ctx.set_output("AvgSquaredUpdateOut", au2)


@register_op("rmsprop", ["Param", "MeanSquare", "Grad", "Moment", "LearningRate", "MeanGrad?"],
             ["ParamOut", "MomentOut", "MeanSquareOut", "MeanGradOut?"],
             {"epsilon": 1e-10, "decay": 0.9, "momentum": 0.0, "centered": False}, grad=None, no_infer=True)
def rmsprop(ctx):
    p, ms, mom, g = ctx.input("Param"), ctx.input("MeanSquare"), ctx.input("Moment"), _grad(ctx).tensor
    eps, rho, mu, lr = ctx.attr("epsilon"), ctx.attr("decay"), ctx.attr("momentum"), _lr(ctx)
    mg = ctx.input("MeanGrad") if ctx.attr("centered") else None
    ms2 = rho * ms + (1 - rho) * g * g
    if ctx.attr("centered"):
        mg = ctx.input("MeanGrad")
        mg2 = rho * mg + (1 - rho) * g
        mom2 = mu * mom + lr * g / torch.sqrt(ms2 - mg2 * mg2 + eps)
        ctx.set_output("MeanGradOut", mg2)
    else:
        mom2 = mu * mom + lr * g / torch.sqrt(ms2 + eps)
    ctx.set_output("ParamOut", p - mom2)
    ctx.set_output("MomentOut", mom2)
    ctx.set_output("MeanSquareOut", ms2)


@register_op("ftrl", ["Param", "SquaredAccumulator", "LinearAccumulator", "Grad", "LearningRate"],
             ["ParamOut", "SquaredAccumOut", "LinearAccumOut"], {"l1": 0.0, "l2": 0.0, "lr_power": -0.5},
             grad=None, no_infer=True)
def ftrl(ctx):
    p, sq, lin, g = (ctx.input("Param"), ctx.input("SquaredAccumulator"), ctx.input("LinearAccumulator"),
                     _grad(ctx).tensor)
    l1, l2, lp, lr = ctx.attr("l1"), ctx.attr("l2"), ctx.attr("lr_power"), _lr(ctx)
    nsq = sq + g * g
    if lp == -0.5:
        sigma = (torch.sqrt(nsq) - torch.sqrt(sq)) / lr
        y = torch.sqrt(nsq) / lr + 2 * l2
    else:
        sigma = (nsq.pow(-lp) - sq.pow(-lp)) / lr
        y = nsq.pow(-lp) / lr + 2 * l2
    nlin = lin + g - sigma * p
    pre = torch.clamp(nlin, -l1, l1) - nlin
    ctx.set_output("ParamOut", torch.where(nlin.abs() > l1, pre / y, torch.zeros_like(p)))
    ctx.set_output("SquaredAccumOut", nsq)
    ctx.set_output("LinearAccumOut", nlin)


@register_op("proximal_gd", ["Param", "Grad", "LearningRate"], ["ParamOut"], {"l1": 0.0, "l2": 0.0},
             grad=None, no_infer=True)
def proximal_gd(ctx):
    p, g, lr = ctx.input("Param"), _grad(ctx).tensor, _lr(ctx)
    l1, l2 = ctx.attr("l1"), ctx.attr("l2")
    prox = p - lr * g
    out = torch.sign(prox) * torch.clamp(prox.abs() - lr * l1, min=0) / (1 + lr * l2)
    ctx.set_output("ParamOut", out)


@register_op("proximal_adagrad", ["Param", "Moment", "Grad", "LearningRate"], ["ParamOut", "MomentOut"],
             {"l1": 0.0, "l2": 0.0}, grad=None, no_infer=True)
def proximal_adagrad(ctx):
    p, m, g, lr = ctx.input("Param"), ctx.input("Moment"), _grad(ctx).tensor, _lr(ctx)
    l1, l2 = ctx.attr("l1"), ctx.attr("l2")
    m2 = m + g * g
    lr_t = lr / torch.sqrt(m2)
    prox = p - lr_t * g
    out = torch.sign(prox) * torch.clamp(prox.abs() - lr_t * l1, min=0) / (1 + lr_t * l2)
    ctx.set_output("ParamOut", out)
    ctx.set_output("MomentOut", m2)


@register_op("average_accumulates",
             ["param", "in_sum_1", "in_sum_2", "in_sum_3", "in_num_accumulates", "in_old_num_accumulates",
              "in_num_updates"],
             ["out_sum_1", "out_sum_2", "out_sum_3", "out_num_accumulates", "out_old_num_accumulates",
              "out_num_updates"], {"average_window": 0.0, "max_average_window": 10000, "min_average_window": 10000},
             grad=None, no_infer=True)
def average_accumulates(ctx):
    """ModelAverage accumulation (average_accumulates_op.h)."""
    p = ctx.input("param")
    s1, s2, s3 = ctx.input("in_sum_1"), ctx.input("in_sum_2"), ctx.input("in_sum_3")
    na = int(ctx.input("in_num_accumulates").reshape(-1)[0])
    ona = int(ctx.input("in_old_num_accumulates").reshape(-1)[0])
    nu = int(ctx.input("in_num_updates").reshape(-1)[0])
    nu += 1
    na += 1
    s1 = s1 + p
    k_max = 16384
    if nu % k_max == 0:
        s2 = s2 + s1
        s1 = torch.zeros_like(s1)
    win = ctx.attr("average_window")
    if na >= ctx.attr("min_average_window") and na >= min(ctx.attr("max_average_window"), nu * win):
        s3 = s1 + s2
        s1 = torch.zeros_like(s1)
        s2 = torch.zeros_like(s2)
        ona, na = na, 0
    dev = p.device
    ctx.set_output("out_sum_1", s1)
    ctx.set_output("out_sum_2", s2)
    ctx.set_output("out_sum_3", s3)
    ctx.set_output("out_num_accumulates", torch.tensor([na], dtype=torch.int64, device=dev))
    ctx.set_output("out_old_num_accumulates", torch.tensor([ona], dtype=torch.int64, device=dev))
    ctx.set_output("out_num_updates", torch.tensor([nu], dtype=torch.int64, device=dev))


# ---------------------------------------------------------------- typed GPU kernels
# Dense fp32 updates on the device run one fused optim_ext.hip kernel, registered as
# the NATIVE (GPU, fp32) kernel of the op; a bf16 / fp16 parameter is cast by the
# data transform, sparse gradients and uncovered shapes run the PLAIN kernel.


def _native_opt(op_type, kind, state_slots, out_slots, hyper, lr=True):
    plain = OP_REGISTRY[op_type].kernel

    def kernel(ctx):
        gv = _grad(ctx)
        if not isinstance(gv, core.SelectedRows):
            states = [ctx.input(s) if ctx.has_input(s) and (s != "MeanGrad" or ctx.attr("centered")) else None
                      for s in state_slots]
            if _native(ctx, kind, ctx.input("Param"), gv.tensor, states, out_slots, lr=lr, in_slots=state_slots,
                       **hyper(ctx)):
                return
        plain(ctx)

    kernel.__name__ = f"{op_type}_native_kernel"
    register_op_kernel(op_type, "GPU", [torch.float32], library=LibraryType.NATIVE)(kernel)


_native_opt("adamax", "adamax", ["Moment", "InfNorm"], ["MomentOut", "InfNormOut"],
            lambda c: {"bp1": c.input("Beta1Pow"), "b1": c.attr("beta1"), "b2": c.attr("beta2"),
                       "eps": c.attr("epsilon")})
_native_opt("decayed_adagrad", "decayed_adagrad", ["Moment"], ["MomentOut"],
            lambda c: {"decay": c.attr("decay"), "eps": c.attr("epsilon")})
_native_opt("adadelta", "adadelta", ["AvgSquaredGrad", "AvgSquaredUpdate"],
            ["AvgSquaredGradOut", "AvgSquaredUpdateOut"], lambda c: {"rho": c.attr("rho"), "eps": c.attr("epsilon")},
            lr=False)
_native_opt("rmsprop", "rmsprop", ["MeanSquare", "Moment", "MeanGrad"], ["MeanSquareOut", "MomentOut", "MeanGradOut"],
            lambda c: {"rho": c.attr("decay"), "mu": c.attr("momentum"), "eps": c.attr("epsilon")})
_native_opt("ftrl", "ftrl", ["SquaredAccumulator", "LinearAccumulator"], ["SquaredAccumOut", "LinearAccumOut"],
            lambda c: {"l1": c.attr("l1"), "l2": c.attr("l2"), "lr_power": c.attr("lr_power")})
_native_opt("proximal_gd", "proximal", [], [], lambda c: {"l1": c.attr("l1"), "l2": c.attr("l2")})
_native_opt("proximal_adagrad", "proximal", ["Moment"], ["MomentOut"],
            lambda c: {"l1": c.attr("l1"), "l2": c.attr("l2")})
_native_opt("lars_momentum", "lars", ["Velocity"], ["VelocityOut"],
            lambda c: {"mu": c.attr("mu"), "coeff": c.attr("lars_coeff"), "wd": c.attr("lars_weight_decay")})
