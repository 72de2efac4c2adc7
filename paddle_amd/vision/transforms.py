"""Minimal paddle.vision.transforms (numpy CHW float pipeline)."""
from __future__ import annotations

import numpy as np


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class Normalize:
    def __init__(self, mean=0.0, std=1.0, data_format="CHW", to_rgb=False, keys=None):
        self.mean = np.asarray(mean, dtype="float32").reshape(-1, 1, 1)
        self.std = np.asarray(std, dtype="float32").reshape(-1, 1, 1)

    def __call__(self, x):
        return ((np.asarray(x, dtype="float32") - self.mean) / self.std).astype("float32")


class ToTensor:
    def __init__(self, data_format="CHW", keys=None):
        self.df = data_format

    def __call__(self, x):
        a = np.asarray(x, dtype="float32")
        if a.ndim == 3 and self.df == "CHW" and a.shape[-1] in (1, 3) and a.shape[0] not in (1, 3):
            a = a.transpose(2, 0, 1)
        return a / 255.0 if a.max() > 1.0 else a


class Transpose:
    def __init__(self, order=(2, 0, 1), keys=None):
        self.order = order

    def __call__(self, x):
        return np.asarray(x).transpose(self.order)


class RandomHorizontalFlip:
    def __init__(self, prob=0.5, keys=None):
        self.p = prob

    def __call__(self, x):
        return np.ascontiguousarray(x[..., ::-1]) if np.random.rand() < self.p else x


class CenterCrop:
    def __init__(self, size, keys=None):
        self.size = (size, size) if isinstance(size, int) else tuple(size)

    def __call__(self, x):
        h, w = x.shape[-2:]
        th, tw = self.size
        i, j = (h - th) // 2, (w - tw) // 2
        return x[..., i:i + th, j:j + tw]


class RandomCrop(CenterCrop):
    def __call__(self, x):
        h, w = x.shape[-2:]
        th, tw = self.size
        i, j = np.random.randint(0, h - th + 1), np.random.randint(0, w - tw + 1)
        return x[..., i:i + th, j:j + tw]
