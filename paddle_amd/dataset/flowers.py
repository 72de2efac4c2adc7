"""Oxford 102 Flowers (reference python/paddle/dataset/flowers.py).

Reads from ``DATA_HOME/flowers``: ``102flowers.tgz`` (``jpg/image_%05d.jpg``),
``imagelabels.mat`` (``labels``, 1-based class per image) and ``setid.mat``
(``trnid`` / ``tstid`` / ``valid`` image numbers; as in the reference, ``train()``
reads the larger ``tstid`` split and ``test()`` ``trnid``).  Each image is decoded
(PIL), resized so the short side is 256, cropped to 224 (random + random
horizontal flip for training, centre otherwise), laid out CHW in BGR order minus
the per-channel mean [103.94, 116.78, 123.68] and flattened: sample =
(float32[3*224*224], label in [1, 102]).  Without the files: deterministic
synthetic samples of that shape.
"""
from __future__ import annotations

import io
import tarfile

import numpy as np

from . import common

DATA_URL = "http://paddlemodels.cdn.bcebos.com/flowers/102flowers.tgz"
LABEL_URL = "http://paddlemodels.cdn.bcebos.com/flowers/imagelabels.mat"
SETID_URL = "http://paddlemodels.cdn.bcebos.com/flowers/setid.mat"
DATA_MD5 = "52808999861908f626f3c1f4e79d11fa"
LABEL_MD5 = "e0620be6f572b9609742df49c70aed4d"
SETID_MD5 = "a5357ecc9cb78c4bef273ce3793fc85c"
TRAIN_FLAG, TEST_FLAG, VALID_FLAG = "tstid", "trnid", "valid"
MEAN_BGR = np.array([103.94, 116.78, 123.68], dtype=np.float32)
TRAIN_SIZE, TEST_SIZE = 6149, 1020


def transform(img_bytes, is_train, rng=None, resize=256, crop=224):
    from PIL import Image

    im = Image.open(io.BytesIO(img_bytes)).convert("RGB")
    w, h = im.size
    s = resize / min(w, h)
    im = im.resize((max(crop, round(w * s)), max(crop, round(h * s))), Image.BILINEAR)
    a = np.asarray(im, dtype=np.float32)[:, :, ::-1]  # HWC BGR
    H, W = a.shape[:2]
    if is_train:
        rng = rng or np.random
        y, x = int(rng.randint(0, H - crop + 1)), int(rng.randint(0, W - crop + 1))
    else:
        y, x = (H - crop) // 2, (W - crop) // 2
    a = a[y:y + crop, x:x + crop]
    if is_train and rng.randint(0, 2):
        a = a[:, ::-1]
    return (a - MEAN_BGR).transpose(2, 0, 1).reshape(-1).astype(np.float32)


def reader_creator(data_file, label_file, setid_file, flag, is_train, seed=0):
    from scipy.io import loadmat

    labels = loadmat(label_file)["labels"].reshape(-1)
    ids = [int(i) for i in loadmat(setid_file)[flag].reshape(-1)]

    def reader():
        rng = np.random.RandomState(seed)
        wanted = {f"jpg/image_{i:05d}.jpg": int(labels[i - 1]) for i in ids}
        with tarfile.open(data_file) as tf:
            for m in tf:
                lab = wanted.get(m.name)
                if lab is None or not m.isfile():
                    continue
                yield transform(tf.extractfile(m).read(), is_train, rng), lab
    return reader


def _synthetic(n, seed):
    def reader():
        rng = np.random.RandomState(seed)
        for _ in range(n):
            yield rng.uniform(-128, 128, 3 * 224 * 224).astype("float32"), int(rng.randint(1, 103))
    return reader


def _make(flag, is_train, n, seed):
    paths = [common.download(DATA_URL, "flowers", DATA_MD5), common.download(LABEL_URL, "flowers", LABEL_MD5),
             common.download(SETID_URL, "flowers", SETID_MD5)]
    if any(p is None for p in paths):
        common.synthetic_notice("flowers", "102flowers.tgz / imagelabels.mat / setid.mat")
        return _synthetic(n, seed)
    return reader_creator(*paths, flag, is_train, seed)


def train(*args, **kwargs):
    return _make(TRAIN_FLAG, True, TRAIN_SIZE, 1)


def test(*args, **kwargs):
    return _make(TEST_FLAG, False, TEST_SIZE, 2)


def valid(*args, **kwargs):
    return _make(VALID_FLAG, False, TEST_SIZE, 3)


def fetch():
    for u, m in ((DATA_URL, DATA_MD5), (LABEL_URL, LABEL_MD5), (SETID_URL, SETID_MD5)):
        common.download(u, "flowers", m)
