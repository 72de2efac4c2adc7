"""Detection layers (python/paddle/fluid/layers/detection.py) -- see operators/detection_ops.py."""
from __future__ import annotations

__all__ = []
