"""Gradient clipping (``paddle.nn.ClipGradBy*``).

Reference parity: fluid/clip.py (GradientClipByValue / ByNorm / ByGlobalNorm,
python/paddle/fluid/clip.py) which appends clip ops to the program.  Here they
operate on the DyGraph ``(param, grad)`` list; the global norm is one fused
device reduction (gfx950 ``pa_sumsq`` per gradient, no host sync).
"""
from __future__ import annotations

import torch

from ..ops import optim as fused_optim


class ClipGradBase:
    def __call__(self, params_grads):
        return self._clip(params_grads)


class ClipGradByValue(ClipGradBase):
    def __init__(self, max, min=None):
        self.max = float(max)
        self.min = -self.max if min is None else float(min)

    def _clip(self, pg):
        for _, g in pg:
            if g is not None:
                g.clamp_(self.min, self.max)
        return pg


class ClipGradByNorm(ClipGradBase):
    def __init__(self, clip_norm):
        self.clip_norm = float(clip_norm)

    def _clip(self, pg):
        for _, g in pg:
            if g is not None:
                n = g.float().norm()
                g.mul_(torch.clamp(self.clip_norm / (n + 1e-6), max=1.0).to(g.dtype))
        return pg


class ClipGradByGlobalNorm(ClipGradBase):
    def __init__(self, clip_norm, group_name="default_group", auto_skip_clip=False):
        self.clip_norm = float(clip_norm)

    def global_norm(self, pg):
        gs = [g for _, g in pg if g is not None]
        if not gs:
            return None
        ss = torch.zeros(1, dtype=torch.float32, device=gs[0].device)
        for g in gs:
            fused_optim.sumsq(g.contiguous(), ss)
        return ss.sqrt()

    def _clip(self, pg):
        n = self.global_norm(pg)
        if n is None:
            return pg
        coef = torch.clamp(self.clip_norm / (n + 1e-6), max=1.0)
        for _, g in pg:
            if g is not None:
                g.mul_(coef.to(g.dtype))
        return pg


# fluid 1.x names
GradientClipByValue = ClipGradByValue
GradientClipByNorm = ClipGradByNorm
GradientClipByGlobalNorm = ClipGradByGlobalNorm
