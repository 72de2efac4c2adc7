"""WMT14 en-fr (reference python/paddle/dataset/wmt14.py).

Reads the preprocessed ``wmt14.tgz`` from ``DATA_HOME/wmt14``: a tar holding one
``*src.dict`` and one ``*trg.dict`` (one token per line, line number = id) and the
parallel corpora ``*train/train``, ``*test/test``, ``*gen/gen`` (``src \\t trg`` per
line).  Sample: (src ids with <s> / <e>, trg ids with leading <s>, trg ids with
trailing <e>); training pairs with more than 80 ids on either side are dropped.
Without the archive: deterministic synthetic samples of that structure.
"""
from __future__ import annotations

import tarfile

import numpy as np

from . import common

URL_TRAIN = "http://paddlemodels.bj.bcebos.com/wmt/wmt14.tgz"
MD5_TRAIN = "0791583d57d5beb693b9414c5b36798c"
START, END, UNK = "<s>", "<e>", "<unk>"
UNK_IDX = 2
MAX_LEN = 80


def _members(tf, suffix):
    return [m for m in tf.getmembers() if m.isfile() and m.name.endswith(suffix)]


def _read_dict(tf, suffix, dict_size):
    ms = _members(tf, suffix)
    if len(ms) != 1:
        raise ValueError(f"wmt14: expected one *{suffix} in the archive, found {len(ms)}")
    d = {}
    for i, line in enumerate(tf.extractfile(ms[0])):
        if i >= dict_size:
            break
        d[line.strip().decode("utf-8")] = i
    return d


def read_dicts(tar_path, dict_size):
    with tarfile.open(tar_path) as tf:
        return _read_dict(tf, "src.dict", dict_size), _read_dict(tf, "trg.dict", dict_size)


def reader_creator(tar_path, corpus, dict_size):
    def reader():
        src_dict, trg_dict = read_dicts(tar_path, dict_size)
        s_start, s_end = src_dict.get(START, UNK_IDX), src_dict.get(END, UNK_IDX)
        t_start, t_end = trg_dict.get(START, UNK_IDX), trg_dict.get(END, UNK_IDX)
        with tarfile.open(tar_path) as tf:
            for m in _members(tf, corpus):
                for line in tf.extractfile(m):
                    cols = line.rstrip(b"\r\n").split(b"\t")
                    if len(cols) != 2:
                        continue
                    src = [s_start] + [src_dict.get(w, UNK_IDX) for w in cols[0].decode("utf-8").split()] + [s_end]
                    trg = [trg_dict.get(w, UNK_IDX) for w in cols[1].decode("utf-8").split()]
                    if len(src) > MAX_LEN or len(trg) > MAX_LEN:
                        continue
                    yield src, [t_start] + trg, trg + [t_end]
    return reader


def _synthetic(n, seed, dict_size):
    def reader():
        rng = np.random.RandomState(seed)
        for _ in range(n):
            ls, lt = int(rng.randint(3, 40)), int(rng.randint(3, 40))
            src = [0] + [int(x) for x in rng.randint(3, dict_size, ls)] + [1]
            trg = [int(x) for x in rng.randint(3, dict_size, lt)]
            yield src, [0] + trg, trg + [1]
    return reader


def _make(corpus, dict_size, n, seed):
    path = common.download(URL_TRAIN, "wmt14", MD5_TRAIN)
    if path is None:
        common.synthetic_notice("wmt14", "wmt14.tgz")
        return _synthetic(n, seed, dict_size)
    return reader_creator(path, corpus, dict_size)


def train(dict_size=30000):
    return _make("train/train", dict_size, 10000, 1)


def test(dict_size=30000):
    return _make("test/test", dict_size, 1000, 2)


def gen(dict_size=30000):
    return _make("gen/gen", dict_size, 1000, 3)


def get_dict(dict_size=30000, reverse=True):
    """(src, trg) dictionaries; ``reverse``: id -> word."""
    path = common.download(URL_TRAIN, "wmt14", MD5_TRAIN)
    if path is None:
        src = trg = {START: 0, END: 1, UNK: 2}
    else:
        src, trg = read_dicts(path, dict_size)
    if reverse:
        return {v: k for k, v in src.items()}, {v: k for k, v in trg.items()}
    return src, trg


def fetch():
    return common.download(URL_TRAIN, "wmt14", MD5_TRAIN)
