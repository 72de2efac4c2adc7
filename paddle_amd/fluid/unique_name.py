"""Unique name generation (python/paddle/fluid/unique_name.py semantics)."""
import collections
import contextlib


class UniqueNameGenerator:
    def __init__(self, prefix=None):
        self.ids = collections.defaultdict(int)
        self.prefix = prefix or ""

    def __call__(self, key):
        tmp = self.ids[key]
        self.ids[key] += 1
        return self.prefix + "_".join([key, str(tmp)])


generator = UniqueNameGenerator()


def generate(key):
    return generator(key)


def switch(new_generator=None):
    global generator
    old = generator
    generator = new_generator or UniqueNameGenerator()
    return old


@contextlib.contextmanager
def guard(new_generator=None):
    if isinstance(new_generator, str):
        new_generator = UniqueNameGenerator(new_generator)
    old = switch(new_generator)
    try:
        yield
    finally:
        switch(old)
