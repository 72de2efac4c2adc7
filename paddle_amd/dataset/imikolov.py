"""PTB language-model corpus (reference python/paddle/dataset/imikolov.py).  Reads
``DATA_HOME/imikolov/simple-examples.tgz`` (``./simple-examples/data/ptb.{train,
valid}.txt``).  ``build_dict(min_word_freq)`` counts words over both files (plus
one ``<s>`` / ``<e>`` per line), keeps words seen more than ``min_word_freq``
times, orders them by (-count, word) and appends ``<unk>``.  Readers yield n-gram
id tuples (NGRAM) or (src, trg) id sequences (SEQ).  Without the archive: a
synthetic corpus with the same reader semantics."""
from __future__ import annotations

import collections
import tarfile

import numpy as np

from . import common

URL = "http://www.fit.vutbr.cz/~imikolov/rnnlm/simple-examples.tgz"
MD5 = "30177ea32e27c525793142b6bf2c8e2d"
TRAIN_FILE = "./simple-examples/data/ptb.train.txt"
TEST_FILE = "./simple-examples/data/ptb.valid.txt"


class DataType:
    NGRAM = 1
    SEQ = 2


def _lines(name):
    path = common.download(URL, "imikolov", MD5)
    if path:
        with tarfile.open(path) as tf:
            member = tf.getmember(name) if name in tf.getnames() else tf.getmember(name.lstrip("./"))
            for ln in tf.extractfile(member):
                yield ln.decode("utf-8", "replace")
        return
    common.synthetic_notice("imikolov", "simple-examples.tgz")
    rng = np.random.RandomState(1 if name == TRAIN_FILE else 2)
    vocab = [f"w{i}" for i in range(2000)]
    zipf = 1.0 / np.arange(1, len(vocab) + 1)
    zipf /= zipf.sum()
    for _ in range(4000 if name == TRAIN_FILE else 400):
        yield " ".join(vocab[i] for i in rng.choice(len(vocab), rng.randint(3, 30), p=zipf)) + "\n"


def word_count(lines, word_freq=None):
    word_freq = collections.defaultdict(int) if word_freq is None else word_freq
    for ln in lines:
        for w in ln.strip().split():
            word_freq[w] += 1
        word_freq["<s>"] += 1
        word_freq["<e>"] += 1
    return word_freq


def build_dict(min_word_freq=50):
    freq = word_count(_lines(TEST_FILE), word_count(_lines(TRAIN_FILE)))
    freq.pop("<unk>", None)
    kept = sorted(((w, c) for w, c in freq.items() if c > min_word_freq), key=lambda x: (-x[1], x[0]))
    word_idx = {w: i for i, (w, _) in enumerate(kept)}
    word_idx["<unk>"] = len(kept)
    return word_idx


def reader_creator(filename, word_idx, n, data_type):
    def reader():
        unk = word_idx["<unk>"]
        for ln in _lines(filename):
            if data_type == DataType.NGRAM:
                if n <= 0:
                    raise ValueError("imikolov: n-gram length must be positive")
                ids = [word_idx.get(w, unk) for w in ["<s>"] + ln.strip().split() + ["<e>"]]
                for i in range(n, len(ids) + 1):
                    yield tuple(ids[i - n:i])
            elif data_type == DataType.SEQ:
                ids = [word_idx.get(w, unk) for w in ln.strip().split()]
                src, trg = [word_idx["<s>"]] + ids, ids + [word_idx["<e>"]]
                if n > 0 and len(src) > n:
                    continue
                yield src, trg
            else:
                raise ValueError(f"imikolov: unknown data type {data_type}")
    return reader


def train(word_idx, n, data_type=DataType.NGRAM):
    return reader_creator(TRAIN_FILE, word_idx, n, data_type)


def test(word_idx, n, data_type=DataType.NGRAM):
    return reader_creator(TEST_FILE, word_idx, n, data_type)


def fetch():
    return common.download(URL, "imikolov", MD5)
