"""``paddle.optimizer`` (DyGraph): SGD, Momentum, Adam, AdamW, Adagrad, RMSProp,
Adadelta, Adamax, Lamb.

Reference parity: the fused update ops (paddle/fluid/operators/{sgd,momentum,adam,
adamax,adagrad,adadelta,rmsprop}_op.*) and fluid/optimizer.py's accumulator
naming (``<param>_moment1_0``, ``<param>_beta1_pow_acc_0`` ...) which is what a
``.pdopt`` file holds.

MI355X design: Adam/AdamW/Momentum/SGD on GPU tensors run the gfx950 fused
kernels (one launch per parameter; ``multi_precision`` keeps an fp32 master copy
for bf16/fp16 parameters and writes the low-precision parameter in the same pass);
Adam follows the reference kernel (adam_op.h:80-84): ``lr_t = lr * sqrt(1-b2^t) / (1-b1^t)``,
``p -= lr_t * m / (sqrt(v) + eps)``.  Other
optimizers are short torch expressions.  For whole-model fused/sharded updates
see :class:`paddle_amd.parallel.sharding.FlatShardedOptimizer`.
"""
from __future__ import annotations

import math

import torch

from ..utils import strict as _strict

from ..ops import optim as fused_optim
from .lr import LRScheduler


class L2Decay:
    def __init__(self, coeff=0.0):
        self.coeff = float(coeff)


class L1Decay:
    def __init__(self, coeff=0.0):
        self.coeff = float(coeff)


def _pname(p, i):
    return getattr(p, "name", None) or f"param_{i}"


class Optimizer:
    _accum_names: tuple = ()

    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None, name=None,
                 multi_precision=False):
        if parameters is None:
            raise ValueError("DyGraph optimizers need `parameters=`")
        params = list(parameters)
        self._param_groups = []
        if params and isinstance(params[0], dict):
            for g in params:
                self._param_groups.append(dict(g, params=list(g["params"])))
        else:
            self._param_groups.append({"params": params})
        self._parameter_list = [p for g in self._param_groups for p in g["params"]]
        self._learning_rate = learning_rate
        self._weight_decay = weight_decay
        self._grad_clip = grad_clip
        self._multi_precision = multi_precision
        self._accumulators: dict = {}
        self._master: dict = {}
        self._step_count = 0
        self._names = {id(p): _pname(p, i) for i, p in enumerate(self._parameter_list)}

    # ------------------------------------------------------------------ lr
    def get_lr(self):
        lr = self._learning_rate
        return lr() if isinstance(lr, LRScheduler) else float(lr)

    def set_lr(self, value):
        if isinstance(self._learning_rate, LRScheduler):
            raise RuntimeError("set_lr is not allowed when the learning rate is a scheduler")
        self._learning_rate = float(value)

    def set_lr_scheduler(self, scheduler):
        self._learning_rate = scheduler

    # --------------------------------------------------------------- state
    def _acc(self, name, p, init=0.0, dtype=torch.float32, shape=None):
        d = self._accumulators.setdefault(name, {})
        if id(p) not in d:
            d[id(p)] = torch.full(shape if shape is not None else p.shape, init, dtype=dtype, device=p.device)
        return d[id(p)]

    def _master_of(self, p):
        if not self._multi_precision or p.dtype == torch.float32:
            return None
        if id(p) not in self._master:
            self._master[id(p)] = p.detach().float().clone()
        return self._master[id(p)]

    def state_dict(self):
        sd = {}
        for name, d in self._accumulators.items():
            for p in self._parameter_list:
                if id(p) in d:
                    sd[f"{self._names[id(p)]}_{name}_0"] = d[id(p)]
        for p in self._parameter_list:
            if id(p) in self._master:
                sd[f"{self._names[id(p)]}_fp32_master_0"] = self._master[id(p)]
        if isinstance(self._learning_rate, LRScheduler):
            sd["LR_Scheduler"] = self._learning_rate.state_dict()
        sd["global_step"] = self._step_count
        sd["__param_order__"] = [self._names[id(p)] for p in self._parameter_list]
        return sd

    def set_state_dict(self, sd):
        by_name = {self._names[id(p)]: p for p in self._parameter_list}
        order = sd.get("__param_order__")
        if order is not None and not all(n in by_name for n in order) and len(order) == len(self._parameter_list):
            # same model rebuilt in another process / name scope: match by position
            by_name = dict(zip(order, self._parameter_list))
        for k, v in sd.items():
            if k == "__param_order__":
                continue
            if k == "LR_Scheduler":
                if isinstance(self._learning_rate, LRScheduler):
                    self._learning_rate.set_state_dict(v)
                continue
            if k == "global_step":
                self._step_count = int(v)
                continue
            for pn, p in sorted(by_name.items(), key=lambda kv: -len(kv[0])):
                if k.startswith(pn + "_") and k.endswith("_0"):
                    acc = k[len(pn) + 1:-2]
                    t = torch.as_tensor(v).to(p.device)
                    if acc == "fp32_master":
                        self._master[id(p)] = t.float().clone()
                    else:
                        self._accumulators.setdefault(acc, {})[id(p)] = t.clone()
                    break

    set_dict = set_state_dict

    # ---------------------------------------------------------------- step
    def clear_grad(self, set_to_zero=True):
        from ..ops import accum as _accum

        _accum.discard()  # deferred dW of an abandoned accumulation (ops/accum.py)
        with _strict.region("optimizer:clear_grad"):
            self._clear_grad(set_to_zero)

    def _clear_grad(self, set_to_zero):
        if set_to_zero and self._flat_grad_zero():
            return
        for p in self._parameter_list:
            if p.grad is not None:
                if set_to_zero:
                    p.grad.zero_()
                else:
                    p.grad = None

    def _flat_grad_zero(self):
        """clear_grad(set_to_zero=True) as ONE fill per (device, dtype): on the first
        call the device gradients are re-homed as views of a flat buffer (the
        backward's in-place accumulation keeps them there), later calls zero the
        buffer in one launch instead of one ``zero_`` per parameter.  A gradient the
        user rebinds (or a parameter without one) falls back to the per-tensor loop
        for that call and the layout is rebuilt on the next."""
        ps = [p for p in self._parameter_list if p.grad is not None]
        if not ps:
            return False
        flat = getattr(self, "_pa_flat_grads", None)
        if flat is not None and flat[0] == len(ps) and all(
                p.grad.data_ptr() == ptr and p.grad.shape == p.shape for p, ptr in zip(ps, flat[1])):
            from ..ops import oplib

            for buf in flat[2]:
                oplib.fill_(buf, 0.0)
            return True
        groups = {}
        for p in ps:
            if (p.grad.layout != torch.strided or not p.grad.is_contiguous()
                    or p.grad.dtype not in (torch.float32, torch.bfloat16, torch.float16)):
                return False
            groups.setdefault((p.grad.device, p.grad.dtype), []).append(p)
        bufs, ptrs = [], {}
        from ..ops import oplib

        for (dev, dt), members in groups.items():
            # 256-B aligned slots (the vectorised kernels take 16-B rows)
            sizes = [(m.grad.numel() + 127) // 128 * 128 for m in members]
            buf = torch.empty(sum(sizes), dtype=dt, device=dev)
            oplib.fill_(buf, 0.0)
            off = 0
            for m, n in zip(members, sizes):
                g = buf[off:off + m.grad.numel()].view(m.grad.shape)
                m.grad = g.as_subclass(type(m.grad)) if type(m.grad) is not torch.Tensor else g
                ptrs[id(m)] = m.grad.data_ptr()
                off += n
            bufs.append(buf)
        self._pa_flat_grads = (len(ps), [ptrs[id(p)] for p in ps], bufs)
        return True

    clear_gradients = clear_grad

    def zero_grad(self, set_to_none=False):
        self.clear_grad(set_to_zero=not set_to_none)

    def _decay_coeff(self, group, p):
        wd = group.get("weight_decay", self._weight_decay)
        if wd is None or getattr(p, "no_weight_decay", False):
            return 0.0, None
        if isinstance(wd, L1Decay):
            return wd.coeff, "l1"
        if isinstance(wd, L2Decay):
            return wd.coeff, "l2"
        return float(wd), "l2"

    @torch.no_grad()
    def step(self):
        # framework region: the update's tensor expressions run on the HIP kernels
        with _strict.region("optimizer:step"):
            self._step()

    def _step(self):
        self._step_count += 1
        pg = [(p, p.grad) for p in self._parameter_list if p.grad is not None and p.requires_grad]
        if self._grad_clip is not None:
            pg = self._grad_clip(pg)
        lr = self.get_lr()
        for group in self._param_groups:
            glr = lr * group.get("learning_rate", 1.0)
            for p in group["params"]:
                if p.grad is None or not p.requires_grad:
                    continue
                g = p.grad
                coeff, kind = self._decay_coeff(group, p)
                if kind is not None and coeff and not self._decoupled:
                    g = g + coeff * (torch.sign(p) if kind == "l1" else p)
                self._update(p, g, glr, group, coeff if self._decoupled else 0.0)

    _decoupled = False

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        loss.backward()
        self.step()
        return None, [(p, p.grad) for p in self._parameter_list]

    def _update(self, p, g, lr, group, wd):
        raise NotImplementedError


class SGD(Optimizer):
    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None,
                 multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)

    def _update(self, p, g, lr, group, wd):
        m = self._master_of(p)
        tgt = m if m is not None else p
        tgt.add_(g.to(tgt.dtype), alpha=-lr)
        if m is not None:
            p.copy_(m)


class Momentum(Optimizer):
    def __init__(self, learning_rate=0.001, momentum=0.9, parameters=None, use_nesterov=False, weight_decay=None,
                 grad_clip=None, multi_precision=False, rescale_grad=1.0, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._momentum, self._nesterov, self._rescale = momentum, use_nesterov, rescale_grad
        self._multi = None

    @staticmethod
    def _multi_eligible(p):
        g = p.grad
        return (p.is_cuda and p.is_contiguous() and p.dtype in (torch.float32, torch.bfloat16) and g is not None
                and g.dtype in (torch.float32, torch.bfloat16) and g.shape == p.shape)

    def _step(self):
        # every parameter in one multi-tensor launch (pa_momentum_multi) when the
        # update is plain Momentum (+ L2) on device tensors -- merged_momentum
        import os

        if (self._grad_clip is None and os.environ.get("FLAGS_multi_tensor_momentum", "1") != "0"
                and all(self._multi_eligible(p) for p in self._parameter_list
                        if p.grad is not None and p.requires_grad)
                and all(self._decay_coeff(g, p)[1] != "l1" for g in self._param_groups for p in g["params"])):
            return self._step_multi()
        return super()._step()

    def _step_multi(self):
        self._step_count += 1
        lr = self.get_lr()
        entries = []
        for group in self._param_groups:
            gl = float(group.get("learning_rate", 1.0))
            for p in group["params"]:
                if p.grad is None or not p.requires_grad:
                    continue
                coeff, kind = self._decay_coeff(group, p)
                m = self._master_of(p)
                vel = self._acc("velocity", p)
                tgt = m if m is not None else p
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                entries.append((tgt.detach(), p.detach() if m is not None else None, g, vel,
                                coeff if kind == "l2" else 0.0, gl))
        if self._multi is None:
            self._multi = fused_optim.MomentumMulti()
        self._multi.step(entries, lr=lr, mu=self._momentum, nesterov=self._nesterov, grad_scale=self._rescale)

    def _update(self, p, g, lr, group, wd):
        vel = self._acc("velocity", p)
        m = self._master_of(p)
        tgt = m if m is not None else p
        if (tgt.is_cuda and tgt.dtype in (torch.float32, torch.bfloat16) and tgt.is_contiguous()
                and g.is_contiguous() and g.dtype in (torch.float32, torch.bfloat16)):
            # bf16 parameters (no master copy) update in place in the same pass
            fused_optim.momentum_flat(tgt.view(-1), g.reshape(-1), vel.view(-1), lr=lr, mu=self._momentum,
                                      nesterov=self._nesterov, grad_scale=self._rescale)
        else:
            gg = g.float() * self._rescale
            vel.mul_(self._momentum).add_(gg)
            upd = gg + self._momentum * vel if self._nesterov else vel
            tgt.sub_((lr * upd).to(tgt.dtype))
        if m is not None:
            p.copy_(m)


class Adam(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None,
                 weight_decay=None, grad_clip=None, lazy_mode=False, multi_precision=False, use_multi_tensor=False,
                 name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._beta1, self._beta2, self._epsilon = beta1, beta2, epsilon

    def _adam(self, p, g, lr, wd):
        m1 = self._acc("moment1", p)
        m2 = self._acc("moment2", p)
        b1p = self._acc("beta1_pow_acc", p, 1.0, shape=[1])
        b2p = self._acc("beta2_pow_acc", p, 1.0, shape=[1])
        b1p.mul_(self._beta1)
        b2p.mul_(self._beta2)
        master = self._master_of(p)
        tgt = master if master is not None else p
        pout = p if master is not None else None
        if tgt.dtype == torch.float32 and tgt.is_contiguous() and g.is_contiguous():
            fused_optim.adamw_flat(tgt.view(-1), g.reshape(-1), m1.view(-1), m2.view(-1), lr=lr, beta1=self._beta1,
                                   beta2=self._beta2, eps=self._epsilon, weight_decay=wd, step=self._step_count,
                                   param_out=pout.view(-1) if pout is not None else None,
                                   beta1_pow=b1p, beta2_pow=b2p, lr_t_eps=True)
            return
        gf = g.float()
        if wd:
            tgt.mul_(1 - lr * wd)
        m1.mul_(self._beta1).add_(gf, alpha=1 - self._beta1)
        m2.mul_(self._beta2).addcmul_(gf, gf, value=1 - self._beta2)
        c1, c2 = 1 - float(b1p), 1 - float(b2p)
        upd = lr * math.sqrt(c2) / c1 * m1 / (m2.sqrt() + self._epsilon)
        tgt.sub_(upd.to(tgt.dtype))
        if pout is not None:
            pout.copy_(tgt)

    def _update(self, p, g, lr, group, wd):
        self._adam(p, g, lr, wd)


class AdamW(Adam):
    _decoupled = True

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None,
                 weight_decay=0.01, lr_ratio=None, apply_decay_param_fun=None, grad_clip=None, lazy_mode=False,
                 multi_precision=False, name=None):
        super().__init__(learning_rate, beta1, beta2, epsilon, parameters, weight_decay, grad_clip,
                         multi_precision=multi_precision, name=name)
        self._apply_decay = apply_decay_param_fun
        self._lr_ratio = lr_ratio

    def _update(self, p, g, lr, group, wd):
        if self._apply_decay is not None and not self._apply_decay(self._names[id(p)]):
            wd = 0.0
        if self._lr_ratio is not None:
            lr = lr * self._lr_ratio(p)
        self._adam(p, g, lr, wd)


class Adamax(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps = beta1, beta2, epsilon

    def _update(self, p, g, lr, group, wd):
        m = self._acc("moment", p)
        u = self._acc("inf_norm", p)
        b1p = self._acc("beta1_pow_acc", p, 1.0, shape=[1])
        b1p.mul_(self._b1)
        gf = g.float()
        m.mul_(self._b1).add_(gf, alpha=1 - self._b1)
        torch.maximum(u * self._b2, gf.abs() + self._eps, out=u)
        p.sub_((lr / (1 - float(b1p)) * m / u).to(p.dtype))


class Adagrad(Optimizer):
    def __init__(self, learning_rate, epsilon=1e-6, parameters=None, weight_decay=None, grad_clip=None, name=None,
                 initial_accumulator_value=0.0):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._eps, self._init = epsilon, initial_accumulator_value

    def _update(self, p, g, lr, group, wd):
        m = self._acc("moment", p, self._init)
        gf = g.float()
        m.add_(gf * gf)
        p.sub_((lr * gf / (m.sqrt() + self._eps)).to(p.dtype))


class RMSProp(Optimizer):
    def __init__(self, learning_rate, rho=0.95, epsilon=1e-6, momentum=0.0, centered=False, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._rho, self._eps, self._mom, self._centered = rho, epsilon, momentum, centered

    def _update(self, p, g, lr, group, wd):
        ms = self._acc("mean_square", p)
        mom = self._acc("momentum", p)
        gf = g.float()
        ms.mul_(self._rho).add_(gf * gf, alpha=1 - self._rho)
        if self._centered:
            mg = self._acc("mean_grad", p)
            mg.mul_(self._rho).add_(gf, alpha=1 - self._rho)
            den = (ms - mg * mg + self._eps).sqrt()
        else:
            den = (ms + self._eps).sqrt()
        mom.mul_(self._mom).add_(lr * gf / den)
        p.sub_(mom.to(p.dtype))


class Adadelta(Optimizer):
    def __init__(self, learning_rate=0.001, epsilon=1e-6, rho=0.95, parameters=None, weight_decay=None,
                 grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._eps, self._rho = epsilon, rho

    def _update(self, p, g, lr, group, wd):
        ag = self._acc("_avg_squared_grad", p)
        au = self._acc("_avg_squared_update", p)
        gf = g.float()
        ag.mul_(self._rho).add_(gf * gf, alpha=1 - self._rho)
        upd = -((au + self._eps) / (ag + self._eps)).sqrt() * gf
        au.mul_(self._rho).add_(upd * upd, alpha=1 - self._rho)
        p.add_((lr * upd).to(p.dtype))


class Lamb(Optimizer):
    _decoupled = True

    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6,
                 parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None, multi_precision=False,
                 name=None):
        super().__init__(learning_rate, parameters, lamb_weight_decay, grad_clip, name, multi_precision)
        self._b1, self._b2, self._eps = beta1, beta2, epsilon
        self._exclude = exclude_from_weight_decay_fn

    def _update(self, p, g, lr, group, wd):
        if self._exclude is not None and self._exclude(p):
            wd = 0.0
        m1 = self._acc("moment1", p)
        m2 = self._acc("moment2", p)
        b1p = self._acc("beta1_pow_acc", p, 1.0, shape=[1])
        b2p = self._acc("beta2_pow_acc", p, 1.0, shape=[1])
        b1p.mul_(self._b1)
        b2p.mul_(self._b2)
        gf = g.float()
        m1.mul_(self._b1).add_(gf, alpha=1 - self._b1)
        m2.mul_(self._b2).addcmul_(gf, gf, value=1 - self._b2)
        r = (m1 / (1 - b1p)) / ((m2 / (1 - b2p)).sqrt() + self._eps) + wd * p.float()
        pn, rn = p.float().norm(), r.norm()
        trust = torch.where((pn > 0) & (rn > 0), pn / rn, torch.ones_like(pn))
        p.sub_((lr * trust * r).to(p.dtype))
