"""Synthetic movielens reader (no network here).  Sample: user/movie features + score."""
import numpy as np

TRAIN_SIZE = 9000
TEST_SIZE = 1000
_GEN = lambda r: (int(r.randint(1, 6041)), int(r.randint(0, 2)), int(r.randint(0, 7)), int(r.randint(0, 21)), int(r.randint(1, 3953)), [int(r.randint(0, 18))], [int(x) for x in r.randint(0, 5175, 4)], [float(r.randint(1, 6))])


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
