"""DistributeTranspiler: parameter-server data parallelism (filled in by the PS milestone)."""
from __future__ import annotations

from .ps_dispatcher import RoundRobin


class DistributeTranspilerConfig:
    slice_var_up = True
    split_method = RoundRobin
    min_block_size = 8192


class DistributeTranspiler:
    def __init__(self, config=None):
        self.config = config or DistributeTranspilerConfig()
