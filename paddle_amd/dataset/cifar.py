"""CIFAR-10 / CIFAR-100 (reference python/paddle/dataset/cifar.py).

The reference unpickles the "python" archives; this package never unpickles data
files, so it reads the equivalent BINARY releases from ``DATA_HOME/cifar``:
``cifar-10-binary.tar.gz`` (``data_batch_{1..5}.bin`` / ``test_batch.bin``: 1 label
byte + 3072 pixel bytes per record) and ``cifar-100-binary.tar.gz`` (``train.bin`` /
``test.bin``: coarse + fine label bytes + 3072 pixels; the fine label is used).
Samples: float32[3072] pixels / 255 (CHW order), int label.  Without the archives:
deterministic synthetic samples."""
from __future__ import annotations

import tarfile

import numpy as np

from . import common

URL_PREFIX = "https://www.cs.toronto.edu/~kriz/"
CIFAR10_URL = URL_PREFIX + "cifar-10-binary.tar.gz"
CIFAR100_URL = URL_PREFIX + "cifar-100-binary.tar.gz"


def _records(path, member_filter, label_bytes):
    rec = label_bytes + 3072
    with tarfile.open(path) as tf:
        names = sorted(m.name for m in tf if m.isfile() and member_filter(m.name))
        for name in names:
            raw = np.frombuffer(tf.extractfile(name).read(), dtype=np.uint8)
            if raw.size % rec:
                raise ValueError(f"{name}: size {raw.size} is not a multiple of {rec}")
            raw = raw.reshape(-1, rec)
            labels = raw[:, label_bytes - 1]
            pix = raw[:, label_bytes:].astype("float32") / 255.0
            for x, y in zip(pix, labels):
                yield x, int(y)


def reader_creator(path, member_filter, label_bytes, cycle=False):
    def reader():
        while True:
            for s in _records(path, member_filter, label_bytes):
                yield s
            if not cycle:
                break
    return reader


def _synthetic(n, classes, seed):
    def reader():
        rng = np.random.RandomState(seed)
        for _ in range(n):
            yield rng.uniform(0, 1, 3072).astype("float32"), int(rng.randint(0, classes))
    return reader


def _make(url, flt, label_bytes, n, classes, seed, cycle=False):
    path = common.download(url, "cifar")
    if path:
        return reader_creator(path, flt, label_bytes, cycle)
    common.synthetic_notice("cifar", url.split("/")[-1] + " (binary release; pickled archives are not read)")
    return _synthetic(n, classes, seed)


def train10(cycle=False):
    return _make(CIFAR10_URL, lambda n: "data_batch_" in n and n.endswith(".bin"), 1, 50000, 10, 1, cycle)


def test10(cycle=False):
    return _make(CIFAR10_URL, lambda n: n.endswith("test_batch.bin"), 1, 10000, 10, 2, cycle)


def train100():
    return _make(CIFAR100_URL, lambda n: n.endswith("train.bin"), 2, 50000, 100, 3)


def test100():
    return _make(CIFAR100_URL, lambda n: n.endswith("test.bin"), 2, 10000, 100, 4)


# round-1 names
train, test = train10, test10


def fetch():
    return [common.download(CIFAR10_URL, "cifar"), common.download(CIFAR100_URL, "cifar")]
