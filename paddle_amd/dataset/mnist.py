"""MNIST (reference python/paddle/dataset/mnist.py).  Reads the IDX files
``train-images-idx3-ubyte.gz`` / ``...labels-idx1-ubyte.gz`` (and t10k-*) from
``DATA_HOME/mnist``; samples: image float32[784] scaled to [-1, 1], int label.
Without the files: deterministic synthetic samples of that shape."""
from __future__ import annotations

import gzip
import struct

import numpy as np

from . import common

URL_PREFIX = "http://yann.lecun.com/exdb/mnist/"
TRAIN_IMAGE_URL = URL_PREFIX + "train-images-idx3-ubyte.gz"
TRAIN_IMAGE_MD5 = "f68b3c2dcbeaaa9fbdd348bbdeb94873"
TRAIN_LABEL_URL = URL_PREFIX + "train-labels-idx1-ubyte.gz"
TRAIN_LABEL_MD5 = "d53e105ee54ea40749a09fcbcd1e9432"
TEST_IMAGE_URL = URL_PREFIX + "t10k-images-idx3-ubyte.gz"
TEST_IMAGE_MD5 = "9fb629c4189551a2d022fa330f9573f3"
TEST_LABEL_URL = URL_PREFIX + "t10k-labels-idx1-ubyte.gz"
TEST_LABEL_MD5 = "ec29112dd5afa0611ce80d1b7f02629c"
TRAIN_SIZE, TEST_SIZE = 60000, 10000


def _idx(path, magic):
    """Array of an IDX file (big-endian header: magic, dims)."""
    with gzip.open(path, "rb") as f:
        data = f.read()
    m, = struct.unpack(">I", data[:4])
    if m != magic:
        raise ValueError(f"{path}: bad IDX magic {m:#x} (expected {magic:#x})")
    nd = magic & 0xFF
    dims = struct.unpack(">" + "I" * nd, data[4:4 + 4 * nd])
    arr = np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd)
    if arr.size != int(np.prod(dims)):
        raise ValueError(f"{path}: {arr.size} bytes for dims {dims}")
    return arr.reshape(dims)


def reader_creator(image_filename, label_filename, buffer_size=100):
    def reader():
        images = _idx(image_filename, 0x803).reshape(-1, 28 * 28)
        labels = _idx(label_filename, 0x801)
        if len(images) != len(labels):
            raise ValueError("mnist: image / label counts differ")
        for s in range(0, len(labels), buffer_size):
            imgs = images[s:s + buffer_size].astype("float32") / 255.0 * 2.0 - 1.0
            for img, lab in zip(imgs, labels[s:s + buffer_size]):
                yield img, int(lab)
    return reader


def _synthetic(n, seed):
    def reader():
        rng = np.random.RandomState(seed)
        for _ in range(n):
            yield rng.uniform(-1, 1, 784).astype("float32"), int(rng.randint(0, 10))
    return reader


def _make(img_url, img_md5, lab_url, lab_md5, n, seed):
    img = common.download(img_url, "mnist", img_md5)
    lab = common.download(lab_url, "mnist", lab_md5)
    if img and lab:
        return reader_creator(img, lab, 100)
    common.synthetic_notice("mnist", "IDX files")
    return _synthetic(n, seed)


def train():
    return _make(TRAIN_IMAGE_URL, TRAIN_IMAGE_MD5, TRAIN_LABEL_URL, TRAIN_LABEL_MD5, TRAIN_SIZE, 1)


def test():
    return _make(TEST_IMAGE_URL, TEST_IMAGE_MD5, TEST_LABEL_URL, TEST_LABEL_MD5, TEST_SIZE, 2)


def fetch():
    return [common.download(u, "mnist") for u in (TRAIN_IMAGE_URL, TRAIN_LABEL_URL, TEST_IMAGE_URL, TEST_LABEL_URL)]
