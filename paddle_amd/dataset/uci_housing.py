"""Synthetic uci_housing reader (no network here).  Sample: features: float32[13], price: float32[1]."""
import numpy as np

TRAIN_SIZE = 404
TEST_SIZE = 102
_GEN = lambda r: (r.uniform(-1, 1, 13).astype('float32'), r.uniform(0, 50, 1).astype('float32'))


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
