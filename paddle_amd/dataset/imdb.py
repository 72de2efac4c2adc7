"""IMDB sentiment (reference python/paddle/dataset/imdb.py).  Reads
``DATA_HOME/imdb/aclImdb_v1.tar.gz``: every ``aclImdb/{train,test}/{pos,neg}/*.txt``
is lower-cased, stripped of punctuation and split on whitespace.  ``word_dict()``
keeps words seen more than 150 times over the training + test files, ordered by
(-count, word), plus ``<unk>``.  Samples: (word ids, label) with label 0 = pos,
1 = neg.  Without the archive: synthetic documents."""
from __future__ import annotations

import collections
import re
import string
import tarfile
import zlib

import numpy as np

from . import common

URL = "http://ai.stanford.edu/%7Eamaas/data/sentiment/aclImdb_v1.tar.gz"
MD5 = "7c2ac02c03563afcf9b574c7e56c153a"
_PUNCT = str.maketrans("", "", string.punctuation)


def tokenize(pattern):
    path = common.download(URL, "imdb", MD5)
    if path:
        with tarfile.open(path) as tf:
            for m in tf:
                if m.isfile() and pattern.match(m.name):
                    text = tf.extractfile(m).read().decode("utf-8", "replace").rstrip("\n\r")
                    yield text.translate(_PUNCT).lower().split()
        return
    common.synthetic_notice("imdb", "aclImdb_v1.tar.gz")
    rng = np.random.RandomState(zlib.crc32(pattern.pattern.encode()))
    for _ in range(200):
        yield [f"w{i}" for i in rng.randint(0, 300, rng.randint(10, 100))]


def build_dict(pattern, cutoff):
    freq = collections.defaultdict(int)
    for doc in tokenize(pattern):
        for w in doc:
            freq[w] += 1
    kept = sorted(((w, c) for w, c in freq.items() if c > cutoff), key=lambda x: (-x[1], x[0]))
    word_idx = {w: i for i, (w, _) in enumerate(kept)}
    word_idx["<unk>"] = len(kept)
    return word_idx


def reader_creator(pos_pattern, neg_pattern, word_idx):
    unk = word_idx["<unk>"]
    data = [([word_idx.get(w, unk) for w in doc], 0) for doc in tokenize(pos_pattern)]
    data += [([word_idx.get(w, unk) for w in doc], 1) for doc in tokenize(neg_pattern)]

    def reader():
        for doc, label in data:
            yield doc, label
    return reader


def train(word_idx):
    return reader_creator(re.compile(r"aclImdb/train/pos/.*\.txt$"), re.compile(r"aclImdb/train/neg/.*\.txt$"),
                          word_idx)


def test(word_idx):
    return reader_creator(re.compile(r"aclImdb/test/pos/.*\.txt$"), re.compile(r"aclImdb/test/neg/.*\.txt$"),
                          word_idx)


def word_dict():
    return build_dict(re.compile(r"aclImdb/((train)|(test))/((pos)|(neg))/.*\.txt$"), 150)


def fetch():
    return common.download(URL, "imdb", MD5)
