"""paddle.dataset parsers on files in the real on-disk formats (reference
python/paddle/dataset/tests/*).  No network: each test writes a miniature file in
the upstream format (IDX gz, housing text, PTB tgz, aclImdb tgz, CIFAR binary
tgz, ml-1m zip) into a temporary DATA_HOME and checks the parsed samples;
without files the modules fall back to synthetic samples of the same shapes."""
import gzip
import io
import struct
import tarfile
import warnings
import zipfile

import numpy as np
import pytest

from paddle_amd.dataset import cifar, common, imdb, imikolov, mnist, movielens, uci_housing


@pytest.fixture
def home(tmp_path, monkeypatch):
    monkeypatch.setattr(common, "DATA_HOME", str(tmp_path))
    monkeypatch.setenv("PADDLE_DATASET_CHECK_MD5", "0")
    return tmp_path


def _tar(path, files):
    with tarfile.open(path, "w:gz") as tf:
        for name, data in files.items():
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            tf.addfile(ti, io.BytesIO(data))


def test_mnist_idx(home):
    d = home / "mnist"
    d.mkdir()
    imgs = np.arange(3 * 784, dtype=np.uint32).reshape(3, 784) % 256
    with gzip.open(d / "train-images-idx3-ubyte.gz", "wb") as f:
        f.write(struct.pack(">IIII", 0x803, 3, 28, 28) + imgs.astype(np.uint8).tobytes())
    with gzip.open(d / "train-labels-idx1-ubyte.gz", "wb") as f:
        f.write(struct.pack(">II", 0x801, 3) + bytes([7, 0, 9]))
    got = list(mnist.train()())
    assert [y for _, y in got] == [7, 0, 9]
    np.testing.assert_allclose(got[1][0], imgs[1].astype(np.float32) / 255 * 2 - 1, rtol=1e-6)


def test_uci_housing_text(home):
    d = home / "uci_housing"
    d.mkdir()
    rows = np.arange(10 * 14, dtype=np.float64).reshape(10, 14) * 0.5
    rows[:, 3] = np.arange(10) % 2
    np.savetxt(d / "housing.data", rows, fmt="%.3f")
    uci_housing._DATA.clear()
    tr, te = list(uci_housing.train()()), list(uci_housing.test()())
    assert len(tr) == 8 and len(te) == 2
    x0, y0 = tr[0]
    assert x0.shape == (13,) and y0.shape == (1,) and y0[0] == pytest.approx(rows[0, 13])
    col = rows[:, 0]
    assert x0[0] == pytest.approx((col[0] - col.mean()) / (col.max() - col.min()), rel=1e-5)
    uci_housing._DATA.clear()


def test_imikolov_ptb(home):
    d = home / "imikolov"
    d.mkdir()
    train_txt = b"the cat sat\nthe dog sat on the mat\n"
    valid_txt = b"the cat\n"
    _tar(d / "simple-examples.tgz", {"./simple-examples/data/ptb.train.txt": train_txt,
                                       "./simple-examples/data/ptb.valid.txt": valid_txt})
    wd = imikolov.build_dict(min_word_freq=0)
    # counts: the 4, <s> 3, <e> 3, sat 2, cat 2, dog/on/mat 1 -> ordered by (-count, word)
    assert [w for w, _ in sorted(wd.items(), key=lambda kv: kv[1])][:5] == ["the", "<e>", "<s>", "cat", "sat"]
    assert wd["<unk>"] == len(wd) - 1
    grams = list(imikolov.train(wd, 3)())
    assert grams[0] == (wd["<s>"], wd["the"], wd["cat"])
    assert len(grams) == (5 - 3 + 1) + (8 - 3 + 1)
    src, trg = next(iter(imikolov.test(wd, 0, imikolov.DataType.SEQ)()))
    assert src == [wd["<s>"], wd["the"], wd["cat"]] and trg == [wd["the"], wd["cat"], wd["<e>"]]


def test_imdb_tokenizer_and_labels(home):
    d = home / "imdb"
    d.mkdir()
    _tar(d / "aclImdb_v1.tar.gz", {
        "aclImdb/train/pos/1_9.txt": b"Great movie, GREAT acting!\n",
        "aclImdb/train/neg/2_1.txt": b"Bad. Boring movie...\n",
        "aclImdb/test/pos/3_8.txt": b"great fun\n",
        "aclImdb/test/neg/4_2.txt": b"boring\n"})
    import re

    wd = imdb.build_dict(re.compile(r"aclImdb/((train)|(test))/((pos)|(neg))/.*\.txt$"), 0)
    assert wd["great"] == 0  # 3 occurrences, most frequent
    got = list(imdb.train(wd)())
    assert [lab for _, lab in got] == [0, 1]
    assert got[0][0] == [wd["great"], wd["movie"], wd["great"], wd["acting"]]


def test_cifar10_binary(home):
    d = home / "cifar"
    d.mkdir()
    rec = lambda lab, v: bytes([lab]) + bytes([v]) * 3072  # noqa: E731
    _tar(d / "cifar-10-binary.tar.gz", {"cifar-10-batches-bin/data_batch_1.bin": rec(3, 255) + rec(5, 0),
                                        "cifar-10-batches-bin/test_batch.bin": rec(1, 51)})
    tr = list(cifar.train10()())
    assert [y for _, y in tr] == [3, 5] and tr[0][0].shape == (3072,) and tr[0][0][0] == 1.0
    te = list(cifar.test10()())
    assert te[0][1] == 1 and te[0][0][0] == pytest.approx(0.2)


def test_movielens_zip(home):
    d = home / "movielens"
    d.mkdir()
    with zipfile.ZipFile(d / "ml-1m.zip", "w") as z:
        z.writestr("ml-1m/movies.dat", "1::Toy Story (1995)::Animation|Comedy\n2::Heat (1995)::Action\n")
        z.writestr("ml-1m/users.dat", "1::F::1::10::48067\n2::M::56::16::70072\n")
        z.writestr("ml-1m/ratings.dat", "".join(f"{1 + i % 2}::{1 + i % 2}::{1 + i % 5}::97830{i}\n"
                                                for i in range(50)))
    movielens._META.clear()
    tr, te = list(movielens.train()()), list(movielens.test()())
    assert len(tr) + len(te) == 50 and len(te) > 0
    s = tr[0]
    assert len(s) == 8 and isinstance(s[5], list) and isinstance(s[7], list)
    cats = movielens.movie_categories()
    assert sorted(cats) == ["Action", "Animation", "Comedy"]
    user = movielens.user_info()[2].value()
    assert user == [2, 0, 6, 16]
    assert movielens.max_movie_id() == 2
    movielens._META.clear()


def test_synthetic_fallback_warns_once(home):
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        common._NOTICED.discard("cifar")
        x, y = next(iter(cifar.train10()()))
        next(iter(cifar.test10()()))
    assert x.shape == (3072,) and 0 <= y < 10
    assert sum("synthetic" in str(m.message) for m in w) == 1
