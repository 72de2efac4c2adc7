"""UCI housing (reference python/paddle/dataset/uci_housing.py).  Reads
``DATA_HOME/uci_housing/housing.data`` (whitespace-separated, 14 columns); the 13
features are mean-centred and divided by their range, the first 80 % of rows are
the training set.  Samples: features float32[13], price float32[1].  Without the
file: deterministic synthetic rows."""
from __future__ import annotations

import numpy as np

from . import common

URL = "https://archive.ics.uci.edu/ml/machine-learning-databases/housing/housing.data"
MD5 = "d4accdce7a25600298819f8e28e8d593"
feature_names = ["CRIM", "ZN", "INDUS", "CHAS", "NOX", "RM", "AGE", "DIS", "RAD", "TAX", "PTRATIO", "B", "LSTAT"]
TRAIN_SIZE, TEST_SIZE = 404, 102
_DATA = {}


def load_data(filename, feature_num=14, ratio=0.8):
    raw = np.loadtxt(filename, dtype=np.float64).reshape(-1, feature_num)
    x = raw.copy()
    mx, mn, avg = raw.max(0), raw.min(0), raw.mean(0)
    rng = np.where(mx - mn == 0, 1.0, mx - mn)
    x[:, :-1] = (raw[:, :-1] - avg[:-1]) / rng[:-1]
    off = int(len(x) * ratio)
    _DATA["train"], _DATA["test"] = x[:off].astype("float32"), x[off:].astype("float32")


def _reader(part, n, seed):
    path = common.download(URL, "uci_housing", MD5)
    if path:
        if part not in _DATA:
            load_data(path)

        def reader():
            for row in _DATA[part]:
                yield row[:-1], row[-1:]
        return reader
    common.synthetic_notice("uci_housing", "housing.data")

    def synth():
        rng = np.random.RandomState(seed)
        for _ in range(n):
            yield rng.uniform(-1, 1, 13).astype("float32"), rng.uniform(0, 50, 1).astype("float32")
    return synth


def train():
    return _reader("train", TRAIN_SIZE, 1)


def test():
    return _reader("test", TEST_SIZE, 2)


def fetch():
    return common.download(URL, "uci_housing", MD5)
