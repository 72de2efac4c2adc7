"""PyDataProvider2 (reference python/paddle/trainer/PyDataProvider2.py): the
``@provider`` decorator turning a generator ``process(settings, filename)`` into a
data provider for the v1 trainer, with input types, an init hook, shuffling and
per-sample format checks.  The input types are the v2 data types (they lower to
Fluid data layers the same way)."""
from __future__ import annotations

from ..v2.data_type import (dense_vector, integer_value, integer_value_sequence,  # noqa: F401
                            dense_vector_sequence)

try:  # optional sparse types of the v2 facade
    from ..v2.data_type import sparse_binary_vector, sparse_float_vector  # noqa: F401
except ImportError:  # pragma: no cover
    pass


class CacheType:
    NO_CACHE = 0
    CACHE_PASS_IN_MEM = 1


class _Settings:
    """The ``settings`` object handed to the init hook and the generator."""

    def __init__(self, input_types, is_train, **kw):
        self.input_types = input_types
        self.is_train = is_train
        for k, v in kw.items():
            setattr(self, k, v)


class DataProvider:
    def __init__(self, generator, input_types, should_shuffle, init_hook, check, cache):
        self.generator = generator
        self.input_types = input_types
        self.should_shuffle = should_shuffle
        self.init_hook = init_hook
        self.check = check
        self.cache = cache
        self._cached = {}
        self._last_types = input_types

    def __call__(self, settings, filename):  # the decorated generator itself
        return self.generator(settings, filename)

    def make_settings(self, args, is_train=True):
        s = _Settings(self.input_types, is_train)
        if self.init_hook is not None:
            self.init_hook(s, **(args or {}))
        self._last_types = s.input_types
        return s

    def _names(self):
        t = self._last_types
        return list(t.keys()) if isinstance(t, dict) else None

    def samples(self, settings, filename):
        """Samples of one file as tuples (dict samples ordered by the input-type keys)."""
        if self.cache == CacheType.CACHE_PASS_IN_MEM and filename in self._cached:
            yield from self._cached[filename]
            return
        names = self._names()
        n = len(settings.input_types) if settings.input_types is not None else None
        keep = [] if self.cache == CacheType.CACHE_PASS_IN_MEM else None
        for item in self.generator(settings, filename):
            if isinstance(item, dict):
                if names is None:
                    raise TypeError("a provider yielding dicts needs dict input_types")
                item = tuple(item[k] for k in names)
            elif not isinstance(item, (tuple, list)):
                item = (item,)
            if self.check and n is not None and len(item) != n:
                raise ValueError(f"sample has {len(item)} fields, input_types declare {n}")
            item = tuple(item)
            if keep is not None:
                keep.append(item)
            yield item
        if keep is not None:
            self._cached[filename] = keep

    def feeding(self, data_layer_names):
        """{data layer name: field index} for the v2 trainer."""
        names = self._names()
        if names is not None:
            return {k: i for i, k in enumerate(names) if k in data_layer_names}
        return {k: i for i, k in enumerate(data_layer_names)}


def provider(input_types=None, should_shuffle=None, pool_size=-1, min_pool_size=-1, can_over_batch_size=True,
             calc_batch_size=None, cache=CacheType.NO_CACHE, check=False, check_fail_continue=False,
             init_hook=None, **kwargs):
    """Decorator: ``@provider(input_types=[dense_vector(784), integer_value(10)])``
    over ``def process(settings, filename): ... yield sample``."""

    def wrap(gen):
        return DataProvider(gen, input_types, True if should_shuffle is None else should_shuffle, init_hook,
                            check, cache)

    return wrap
