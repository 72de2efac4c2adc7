"""paddle.amp: bf16 autocast (MI355X's native MFMA type) and a dynamic loss scaler.

``auto_cast(level="O1")`` runs matmul/conv/attention in bf16 (or fp16) via the
device autocast; ``level="O2"`` with ``decorate`` casts the model's parameters and
keeps fp32 master weights inside the optimizer (``multi_precision``).  bf16 needs
no loss scaling; ``GradScaler`` implements Paddle's dynamic scaling for fp16.
"""
from __future__ import annotations

import contextlib

import torch


@contextlib.contextmanager
def auto_cast(enable=True, custom_white_list=None, custom_black_list=None, level="O1", dtype="bfloat16",
              use_promote=True):
    if not enable:
        yield
        return
    dt = torch.bfloat16 if dtype in ("bfloat16", "bf16") else torch.float16
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    with torch.autocast(dev, dtype=dt if dev == "cuda" else torch.bfloat16):
        yield


amp_guard = auto_cast


def decorate(models, optimizers=None, level="O1", dtype="bfloat16", master_weight=None, save_dtype=None,
             master_grad=False, excluded_layers=None):
    dt = torch.bfloat16 if dtype in ("bfloat16", "bf16") else torch.float16
    single = not isinstance(models, (list, tuple))
    ms = [models] if single else list(models)
    if level == "O2":
        for m in ms:
            for mod in m.modules():
                if isinstance(mod, (torch.nn.BatchNorm1d, torch.nn.BatchNorm2d)) or "BatchNorm" in type(mod).__name__ \
                        or "LayerNorm" in type(mod).__name__:
                    continue
                for p in mod.parameters(recurse=False):
                    p.data = p.data.to(dt)
        if optimizers is not None:
            for o in (optimizers if isinstance(optimizers, (list, tuple)) else [optimizers]):
                o._multi_precision = True if master_weight is None else master_weight
    out_m = ms[0] if single else ms
    if optimizers is None:
        return out_m
    return out_m, optimizers


class GradScaler:
    def __init__(self, enable=True, init_loss_scaling=2.0 ** 15, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=1000, decr_every_n_nan_or_inf=2, use_dynamic_loss_scaling=True):
        self.enable = enable
        self.scale_v = float(init_loss_scaling)
        self.incr_ratio, self.decr_ratio = incr_ratio, decr_ratio
        self.incr_n, self.decr_n = incr_every_n_steps, decr_every_n_nan_or_inf
        self.dynamic = use_dynamic_loss_scaling
        self._good = self._bad = 0
        self._unscaled = False
        self._found_inf = False

    def scale(self, loss):
        return loss * self.scale_v if self.enable else loss

    def unscale_(self, optimizer):
        if not self.enable or self._unscaled:
            return
        # data-parallel wrappers reduce the gradients first: the inf check below then
        # sees the same (averaged) gradients on every rank (HybridParallelOptimizer)
        pre = getattr(optimizer, "_sync_grads_before_unscale", None)
        if pre is not None:
            pre()
        inv = 1.0 / self.scale_v
        # one device flag for every gradient (native isfinite kernel), one host read
        from ..ops import oplib as _oplib

        flags = {}
        found = False
        for p in optimizer._parameter_list:
            if p.grad is not None:
                p.grad.mul_(inv)
                g = p.grad
                if g.is_cuda:
                    bad = flags.setdefault(g.device, torch.zeros(1, dtype=torch.int32, device=g.device))
                    if _oplib.isfinite_op(g, bad):
                        continue
                    bad.add_((~torch.isfinite(g)).any().int())
                else:
                    found = found or not bool(torch.isfinite(g).all())
        self._found_inf = found or any(int(b.item()) > 0 for b in flags.values())
        self._unscaled = True

    def step(self, optimizer):
        if not self.enable:
            return optimizer.step()
        self.unscale_(optimizer)
        if not self._found_inf:
            optimizer.step()

    def update(self):
        if not (self.enable and self.dynamic):
            self._unscaled = False
            return
        if self._found_inf:
            self._bad += 1
            self._good = 0
            if self._bad >= self.decr_n:
                self.scale_v *= self.decr_ratio
                self._bad = 0
        else:
            self._good += 1
            self._bad = 0
            if self._good >= self.incr_n:
                self.scale_v *= self.incr_ratio
                self._good = 0
        self._unscaled = False

    def minimize(self, optimizer, *args, **kwargs):
        self.step(optimizer)
        self.update()

    def get_loss_scaling(self):
        return self.scale_v

    def state_dict(self):
        return {"scale": self.scale_v, "good": self._good, "bad": self._bad}

    def load_state_dict(self, sd):
        self.scale_v, self._good, self._bad = sd["scale"], sd["good"], sd["bad"]


AmpScaler = GradScaler
