"""Framework-owned differentiation: ``tape`` (reverse-mode over the fused ops)."""
from . import tape  # noqa: F401
from .tape import recording  # noqa: F401
