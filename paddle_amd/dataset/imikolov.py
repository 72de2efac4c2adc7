"""Synthetic imikolov reader (no network here).  Sample: 5-gram of word ids."""
import numpy as np

TRAIN_SIZE = 10000
TEST_SIZE = 1000
_GEN = lambda r: tuple(int(x) for x in r.randint(0, 2074, 5))


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
