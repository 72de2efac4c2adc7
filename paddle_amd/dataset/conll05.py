"""CoNLL-2005 semantic role labelling (reference python/paddle/dataset/conll05.py).

Reads from ``DATA_HOME/conll05st``: ``conll05st-tests.tar.gz`` (gzipped
``test.wsj.words`` / ``test.wsj.props`` column files inside), ``wordDict.txt``,
``verbDict.txt``, ``targetDict.txt`` (one entry per line) and the ``emb`` word
vectors.  Each predicate of a sentence yields one sample of nine sequences:
(word ids, ctx_n2, ctx_n1, ctx_0, ctx_p1, ctx_p2, predicate ids, mark, label ids),
the ctx_* being the words around the predicate (``bos`` / ``eos`` past the ends)
repeated over the sentence and ``mark`` flagging that 5-word window.  The props
bracket notation ``(A0*``, ``*``, ``*)``, ``(V*)`` becomes B-/I-/O tags.  The
reference also trains on the test split (the training set is not free).
Without the files: deterministic synthetic samples of that structure.
"""
from __future__ import annotations

import gzip
import io
import tarfile

import numpy as np

from . import common

DATA_URL = "http://paddlemodels.bj.bcebos.com/conll05st/conll05st-tests.tar.gz"
DATA_MD5 = "387719152ae52d60422c016e92a742fc"
WORDDICT_URL = "http://paddlemodels.bj.bcebos.com/conll05st%2FwordDict.txt"
WORDDICT_MD5 = "ea7fb7d4c75cc6254716f0177a506baa"
VERBDICT_URL = "http://paddlemodels.bj.bcebos.com/conll05st%2FverbDict.txt"
VERBDICT_MD5 = "0d2977293bbb6cbefab5b0f97db1e77c"
TRGDICT_URL = "http://paddlemodels.bj.bcebos.com/conll05st%2FtargetDict.txt"
TRGDICT_MD5 = "d8c7f03ceb5fc2e5a0fa7503a4353751"
EMB_URL = "http://paddlemodels.bj.bcebos.com/conll05st%2Femb"
EMB_MD5 = "bf436eb0faa1f6f9103017f8be57cdb7"
WORDS_NAME = "conll05st-release/test.wsj/words/test.wsj.words.gz"
PROPS_NAME = "conll05st-release/test.wsj/props/test.wsj.props.gz"
UNK_IDX = 0


def load_dict(path):
    with open(path, encoding="utf-8") as f:
        return {line.strip(): i for i, line in enumerate(f)}


def load_label_dict(path):
    """B-X / I-X pairs for every tag X in the file (first-seen order), then O."""
    tags = []
    with open(path, encoding="utf-8") as f:
        for line in f:
            line = line.strip()
            if line[:2] in ("B-", "I-") and line[2:] not in tags:
                tags.append(line[2:])
    d = {}
    for t in tags:
        d["B-" + t] = len(d)
        d["I-" + t] = len(d)
    d["O"] = len(d)
    return d


def bracket_to_tags(col):
    """One props column ('(A0*', '*', '*)', '(V*)', ...) -> B-/I-/O tags."""
    out, cur, inside = [], "O", False
    for tok in col:
        if tok == "*":
            out.append("I-" + cur if inside else "O")
        elif tok == "*)":
            out.append("I-" + cur)
            inside = False
        elif "(" in tok:
            cur = tok[1:tok.index("*")]
            out.append("B-" + cur)
            inside = ")" not in tok
        else:
            raise ValueError(f"conll05: unexpected props token {tok!r}")
    return out


def corpus_reader(tar_path, words_name=WORDS_NAME, props_name=PROPS_NAME):
    """(sentence words, predicate, tags) per predicate of every sentence."""
    def reader():
        with tarfile.open(tar_path) as tf:
            words = gzip.GzipFile(fileobj=io.BytesIO(tf.extractfile(words_name).read()))
            props = gzip.GzipFile(fileobj=io.BytesIO(tf.extractfile(props_name).read()))
            sent, rows = [], []
            for wl, pl in zip(words, props):
                w, cols = wl.decode("utf-8").strip(), pl.decode("utf-8").split()
                if cols:
                    sent.append(w)
                    rows.append(cols)
                    continue
                if rows:
                    columns = list(zip(*rows))
                    verbs = [v for v in columns[0] if v != "-"]
                    for i, col in enumerate(columns[1:]):
                        yield list(sent), verbs[i], bracket_to_tags(col)
                sent, rows = [], []
    return reader


def reader_creator(corpus, word_dict, predicate_dict, label_dict):
    def reader():
        for sentence, predicate, tags in corpus():
            n = len(sentence)
            v = tags.index("B-V")
            mark = [0] * n
            ctx = []
            for off, pad in ((-2, "bos"), (-1, "bos"), (0, None), (1, "eos"), (2, "eos")):
                j = v + off
                if 0 <= j < n:
                    mark[j] = 1
                    ctx.append(sentence[j])
                else:
                    ctx.append(pad)
            word_idx = [word_dict.get(w, UNK_IDX) for w in sentence]
            ctx_idx = [[word_dict.get(c, UNK_IDX)] * n for c in ctx]
            yield (word_idx, *ctx_idx, [predicate_dict.get(predicate)] * n, mark,
                   [label_dict.get(t) for t in tags])
    return reader


def _get(url, md5):
    """The cached file under its URL basename (``conll05st%2FwordDict.txt``, as the
    reference saves it) or its plain name (``wordDict.txt``)."""
    return common.download(url, "conll05st", md5) or common.download(url, "conll05st", md5,
                                                                     url.split("%2F")[-1])


def get_dict():
    paths = [_get(u, m) for u, m in
             ((WORDDICT_URL, WORDDICT_MD5), (VERBDICT_URL, VERBDICT_MD5), (TRGDICT_URL, TRGDICT_MD5))]
    if any(p is None for p in paths):
        return None
    return load_dict(paths[0]), load_dict(paths[1]), load_label_dict(paths[2])


def get_embedding():
    return _get(EMB_URL, EMB_MD5)


def _synthetic(n, seed):
    def reader():
        rng = np.random.RandomState(seed)
        for _ in range(n):
            L = int(rng.randint(5, 40))
            v = int(rng.randint(0, L))
            mark = [1 if abs(i - v) <= 2 else 0 for i in range(L)]
            seqs = [[int(x) for x in rng.randint(0, 44068, L)]]
            seqs += [[int(rng.randint(0, 44068))] * L for _ in range(5)]
            seqs += [[int(rng.randint(0, 3162))] * L, mark, [int(x) for x in rng.randint(0, 59, L)]]
            yield tuple(seqs)
    return reader


def test():
    dicts = get_dict()
    data = common.download(DATA_URL, "conll05st", DATA_MD5)
    if dicts is None or data is None:
        common.synthetic_notice("conll05st", "conll05st-tests.tar.gz / dictionaries")
        return _synthetic(5000, 1)
    return reader_creator(corpus_reader(data), *dicts)


train = test  # the reference trains on the (free) test split


def fetch():
    for u, m in ((WORDDICT_URL, WORDDICT_MD5), (VERBDICT_URL, VERBDICT_MD5), (TRGDICT_URL, TRGDICT_MD5),
                 (EMB_URL, EMB_MD5), (DATA_URL, DATA_MD5)):
        _get(u, m)
