"""paddle.dataset parsers on files in the real on-disk formats (reference
python/paddle/dataset/tests/*).  No network: each test writes a miniature file in
the upstream format (IDX gz, housing text, PTB tgz, aclImdb tgz, CIFAR binary
tgz, ml-1m zip, WMT14/WMT16 tgz, CoNLL-05 props, 102flowers tgz + .mat) into a
temporary DATA_HOME and checks the parsed samples;
without files the modules fall back to synthetic samples of the same shapes."""
import gzip
import io
import struct
import tarfile
import warnings
import zipfile

import numpy as np
import pytest

from paddle_amd.dataset import (cifar, common, conll05, flowers, imdb, imikolov, mnist, movielens, uci_housing,
                                wmt14, wmt16)


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


def test_wmt14_tgz(home):
    d = home / "wmt14"
    d.mkdir()
    src_dict = b"<s>\n<e>\n<unk>\nle\nchat\nnoir\n"
    trg_dict = b"<s>\n<e>\n<unk>\nthe\ncat\nblack\n"
    train = b"le chat noir\tthe black cat\nle chien\tthe dog\nbroken line\n" + \
        ("x " * 90).encode() + b"\tthe\n"
    _tar(d / "wmt14.tgz", {"wmt14/src.dict": src_dict, "wmt14/trg.dict": trg_dict, "wmt14/train/train": train,
                           "wmt14/test/test": b"chat\tcat\n"})
    got = list(wmt14.train(dict_size=6)())
    assert got[0] == ([0, 3, 4, 5, 1], [0, 3, 5, 4], [3, 5, 4, 1])
    assert got[1] == ([0, 3, 2, 1], [0, 3, 2], [3, 2, 1])  # unknown words -> UNK_IDX 2
    assert len(got) == 2  # the malformed line and the > 80-id pair are dropped
    assert list(wmt14.test(dict_size=6)()) == [([0, 4, 1], [0, 4], [4, 1])]
    src, trg = wmt14.get_dict(6)
    assert src[4] == "chat" and trg[5] == "black"


def test_wmt16_tgz_builds_frequency_dicts(home):
    d = home / "wmt16"
    d.mkdir()
    train = b"a b b c\tx y y y\nb c\tz x\n"
    _tar(d / "wmt16.tar.gz", {"wmt16/train": train, "wmt16/test": b"c a q\ty z\n", "wmt16/val": b"b\tx\n"})
    en = wmt16.get_dict("en", 6)
    assert list(en) == ["<s>", "<e>", "<unk>", "b", "c", "a"]  # by count, ties by first occurrence
    got = list(wmt16.test(6, 6, "en")())
    de = wmt16.get_dict("de", 6)
    assert got == [([0, en["c"], en["a"], 2, 1], [0, de["y"], de["z"]], [de["y"], de["z"], 1])]
    assert (home / "wmt16" / "en_6.dict").exists()
    rev = list(wmt16.validation(6, 6, "de")())  # German source
    assert rev == [([0, de["x"], 1], [0, en["b"]], [en["b"], 1])]


def test_conll05_props_to_samples(home):
    d = home / "conll05st"
    d.mkdir()
    (d / "wordDict.txt").write_text("<unk>\nThe\ncat\nsat\ndown\nbos\neos\n")
    (d / "verbDict.txt").write_text("sit\n")
    (d / "targetDict.txt").write_text("B-A0\nI-A0\nB-V\nI-V\nB-AM\nI-AM\n")
    words = b"The\ncat\nsat\ndown\n\n"
    # column 0: the predicate lemma on its row; column 1: that predicate's arguments
    props = b"-\t(A0*\n-\t*)\nsit\t(V*)\n-\t(AM*)\n\n"
    _tar(d / "conll05st-tests.tar.gz", {conll05.WORDS_NAME: gzip.compress(words),
                                        conll05.PROPS_NAME: gzip.compress(props)})
    wd, vd, ld = conll05.get_dict()
    assert ld == {"B-A0": 0, "I-A0": 1, "B-V": 2, "I-V": 3, "B-AM": 4, "I-AM": 5, "O": 6}
    (s,) = list(conll05.test()())
    word, n2, n1, c0, p1, p2, pred, mark, lab = s
    assert word == [1, 2, 3, 4]
    assert n2 == [wd["The"]] * 4 and n1 == [wd["cat"]] * 4 and c0 == [wd["sat"]] * 4
    assert p1 == [wd["down"]] * 4 and p2 == [wd["eos"]] * 4 and pred == [0] * 4
    assert mark == [1, 1, 1, 1]
    assert lab == [ld["B-A0"], ld["I-A0"], ld["B-V"], ld["B-AM"]]


def test_flowers_tgz_and_mat(home):
    from PIL import Image
    from scipy.io import savemat

    d = home / "flowers"
    d.mkdir()
    files = {}
    for i in (1, 2, 3):
        buf = io.BytesIO()
        Image.fromarray(np.full((240, 300, 3), 40 * i, dtype=np.uint8)).save(buf, format="JPEG", quality=95)
        files[f"jpg/image_{i:05d}.jpg"] = buf.getvalue()
    _tar(d / "102flowers.tgz", files)
    savemat(d / "imagelabels.mat", {"labels": np.array([[5, 17, 102]])})
    savemat(d / "setid.mat", {"trnid": np.array([[2]]), "tstid": np.array([[1, 3]]), "valid": np.array([[3]])})
    tr = list(flowers.train()())
    assert [y for _, y in tr] == [5, 102]
    assert all(x.shape == (3 * 224 * 224,) and x.dtype == np.float32 for x, _ in tr)
    (x, y), = list(flowers.test()())
    assert y == 17
    # a flat grey image: every pixel of channel c is 80 - mean[c] (BGR order)
    img = x.reshape(3, 224, 224)
    for c in range(3):
        assert abs(float(img[c].mean()) - (80 - flowers.MEAN_BGR[c])) < 2.0
