"""Runtime utilities: flags, profiler, checkpoint helpers."""
from . import flags, profiler  # noqa: F401
