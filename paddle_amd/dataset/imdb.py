"""Synthetic imdb reader (no network here).  Sample: word ids: list[int] (len 10..100), label: int in {0,1}."""
import numpy as np

TRAIN_SIZE = 25000
TEST_SIZE = 25000
_GEN = lambda r: ([int(x) for x in r.randint(0, 5148, r.randint(10, 100))], int(r.randint(0, 2)))


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
