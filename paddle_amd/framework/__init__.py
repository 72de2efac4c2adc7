"""Static-graph engine core: IR schema, runtime data model, op registry, executor."""
from . import core, proto, registry  # noqa: F401
