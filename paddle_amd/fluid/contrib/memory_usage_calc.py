"""Estimate a program's memory footprint (contrib/memory_usage_calc.py)."""
from __future__ import annotations

import numpy as np

from ...framework import core


def memory_usage(program, batch_size):
    total = 0.0
    for var in program.global_block().vars.values():
        if var.type != core.VT.LOD_TENSOR or not var.shape:
            continue
        shape = [batch_size if s < 0 else s for s in var.shape]
        total += float(np.prod(shape)) * core.dtype_size(var.dtype)
    unit = "B"
    for u in ("KB", "MB", "GB"):
        if total >= 1024:
            total /= 1024.0
            unit = u
    return total * 0.95, total * 1.05, unit
