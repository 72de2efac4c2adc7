"""Reader combinators (python/paddle/reader/decorator.py) and paddle.batch."""
from .decorator import (batch, buffered, cache, chain, compose, firstn, map_readers, shuffle,  # noqa: F401
                        xmap_readers, multiprocess_reader, ComposeNotAligned)
