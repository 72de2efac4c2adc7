"""Synthetic wmt16 reader (no network here).  Sample: (src ids, trg ids, trg next ids)."""
import numpy as np

TRAIN_SIZE = 10000
TEST_SIZE = 1000
_GEN = lambda r: (lambda n: ([int(x) for x in r.randint(3, 10000, n)], [int(x) for x in r.randint(3, 10000, n)], [int(x) for x in r.randint(3, 10000, n)]))(int(r.randint(5, 50)))


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
