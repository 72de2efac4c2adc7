"""fluid.contrib: beam-search decoder helpers and memory usage estimation."""
from . import memory_usage_calc  # noqa: F401
from .memory_usage_calc import memory_usage  # noqa: F401
from . import decoder  # noqa: F401,E402
from .decoder import BeamSearchDecoder, InitState, StateCell, TrainingDecoder  # noqa: F401,E402
