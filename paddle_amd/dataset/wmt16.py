"""WMT16 multimodal en-de (reference python/paddle/dataset/wmt16.py).

Reads ``wmt16.tar.gz`` from ``DATA_HOME/wmt16``: members ``wmt16/train``,
``wmt16/test``, ``wmt16/val`` with ``en \\t de`` tokenised lines.  Dictionaries are
built from the training corpus by descending frequency (ties: first occurrence),
``<s> <e> <unk>`` first, and cached as ``DATA_HOME/wmt16/<lang>_<size>.dict``.
Sample: (src ids with <s> / <e>, trg ids with leading <s>, trg ids with trailing
<e>).  Without the archive: deterministic synthetic samples of that structure.
"""
from __future__ import annotations

import os
import tarfile
from collections import Counter

import numpy as np

from . import common

DATA_URL = "http://cloud.dlnel.org/filepub/?uuid=46a0808e-ddd8-427c-bacd-0dbc6d045fed"
DATA_MD5 = "0c38be43600334966403524a40dcd81e"
TOTAL_EN_WORDS, TOTAL_DE_WORDS = 11250, 19220
START_MARK, END_MARK, UNK_MARK = "<s>", "<e>", "<unk>"


def _lines(tar_path, member):
    with tarfile.open(tar_path) as tf:
        for line in tf.extractfile(member):
            cols = line.rstrip(b"\r\n").split(b"\t")
            if len(cols) == 2:
                yield cols[0].decode("utf-8").split(), cols[1].decode("utf-8").split()


def build_dict(tar_path, dict_size, lang):
    cnt = Counter()
    col = 0 if lang == "en" else 1
    for pair in _lines(tar_path, "wmt16/train"):
        cnt.update(pair[col])
    # Counter keeps first-insertion order; the stable sort breaks count ties by it
    words = [w for w, _ in sorted(cnt.items(), key=lambda kv: -kv[1])][:max(0, dict_size - 3)]
    return [START_MARK, END_MARK, UNK_MARK] + words


def load_dict(tar_path, dict_size, lang, reverse=False):
    path = os.path.join(common.DATA_HOME, "wmt16", f"{lang}_{dict_size}.dict")
    words = None
    if os.path.exists(path):
        with open(path, encoding="utf-8") as f:
            words = [ln.rstrip("\n") for ln in f]
        if len(words) != dict_size:
            words = None
    if words is None:
        words = build_dict(tar_path, dict_size, lang)
        try:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            with open(path, "w", encoding="utf-8") as f:
                f.write("\n".join(words) + "\n")
        except OSError:
            pass
    return {i: w for i, w in enumerate(words)} if reverse else {w: i for i, w in enumerate(words)}


def _sizes(src, trg, src_lang):
    en_de = src_lang == "en"
    return min(src, TOTAL_EN_WORDS if en_de else TOTAL_DE_WORDS), min(trg, TOTAL_DE_WORDS if en_de else TOTAL_EN_WORDS)


def reader_creator(tar_path, member, src_dict_size, trg_dict_size, src_lang):
    def reader():
        trg_lang = "de" if src_lang == "en" else "en"
        sd = load_dict(tar_path, src_dict_size, src_lang)
        td = load_dict(tar_path, trg_dict_size, trg_lang)
        s, e, u = sd[START_MARK], sd[END_MARK], sd[UNK_MARK]
        sc = 0 if src_lang == "en" else 1
        for pair in _lines(tar_path, member):
            src = [s] + [sd.get(w, u) for w in pair[sc]] + [e]
            trg = [td.get(w, u) for w in pair[1 - sc]]
            yield src, [s] + trg, trg + [e]
    return reader


def _synthetic(n, seed, vs, vt):
    def reader():
        rng = np.random.RandomState(seed)
        for _ in range(n):
            src = [0] + [int(x) for x in rng.randint(3, vs, int(rng.randint(3, 30)))] + [1]
            trg = [int(x) for x in rng.randint(3, vt, int(rng.randint(3, 30)))]
            yield src, [0] + trg, trg + [1]
    return reader


def _make(member, src_dict_size, trg_dict_size, src_lang, n, seed):
    if src_lang not in ("en", "de"):
        raise ValueError("wmt16: src_lang must be 'en' or 'de'")
    vs, vt = _sizes(src_dict_size, trg_dict_size, src_lang)
    path = common.download(DATA_URL, "wmt16", DATA_MD5, "wmt16.tar.gz")
    if path is None:
        common.synthetic_notice("wmt16", "wmt16.tar.gz")
        return _synthetic(n, seed, vs, vt)
    return reader_creator(path, member, vs, vt, src_lang)


def train(src_dict_size, trg_dict_size, src_lang="en"):
    return _make("wmt16/train", src_dict_size, trg_dict_size, src_lang, 10000, 1)


def test(src_dict_size, trg_dict_size, src_lang="en"):
    return _make("wmt16/test", src_dict_size, trg_dict_size, src_lang, 1000, 2)


def validation(src_dict_size, trg_dict_size, src_lang="en"):
    return _make("wmt16/val", src_dict_size, trg_dict_size, src_lang, 1000, 3)


def get_dict(lang, dict_size, reverse=False):
    size = min(dict_size, TOTAL_EN_WORDS if lang == "en" else TOTAL_DE_WORDS)
    path = common.download(DATA_URL, "wmt16", DATA_MD5, "wmt16.tar.gz")
    if path is None:
        words = [START_MARK, END_MARK, UNK_MARK]
        return {i: w for i, w in enumerate(words)} if reverse else {w: i for i, w in enumerate(words)}
    return load_dict(path, size, lang, reverse)


def fetch():
    return common.download(DATA_URL, "wmt16", DATA_MD5, "wmt16.tar.gz")
