"""Synthetic conll05 reader (no network here).  Sample: SRL slots (9 sequences)."""
import numpy as np

TRAIN_SIZE = 5000
TEST_SIZE = 500
_GEN = lambda r: (lambda n: tuple([int(x) for x in r.randint(0, 44068, n)] for _ in range(8)) + ([int(x) for x in r.randint(0, 59, n)],))(int(r.randint(5, 40)))


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
