"""Synthetic cifar reader (no network here).  Sample: image: float32[3072], label: int in [0,10)."""
import numpy as np

TRAIN_SIZE = 50000
TEST_SIZE = 10000
_GEN = lambda r: (r.uniform(0, 1, 3072).astype('float32'), int(r.randint(0, 10)))


def _reader(n, seed):
    def r():
        rng = np.random.RandomState(seed)
        for _ in range(n):
            yield _GEN(rng)
    return r


def train(*args, **kwargs):
    return _reader(TRAIN_SIZE, 1)


def test(*args, **kwargs):
    return _reader(TEST_SIZE, 2)


def fetch():
    pass
