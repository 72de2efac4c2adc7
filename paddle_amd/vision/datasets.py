"""paddle.vision.datasets with synthetic data (no network in this environment):
shapes and label ranges match the real datasets so training code runs unchanged."""
from __future__ import annotations

import numpy as np

from ..io import Dataset


class _Synthetic(Dataset):
    shape = (1, 28, 28)
    classes = 10
    sizes = {"train": 60000, "test": 10000}

    def __init__(self, image_path=None, label_path=None, mode="train", transform=None, download=True,
                 backend=None, num_samples=None, seed=0):
        self.mode, self.transform = mode, transform
        self.n = num_samples or self.sizes.get(mode, 1000)
        self.seed = seed + (0 if mode == "train" else 1)

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        rng = np.random.RandomState(self.seed * 1000003 + i)
        label = rng.randint(0, self.classes)
        img = rng.rand(*self.shape).astype("float32") * 0.5
        # class-dependent bright stripe so models can actually learn
        c = self.shape[-2] * label // self.classes
        img[..., c:c + max(1, self.shape[-2] // self.classes), :] += 0.5
        if self.transform is not None:
            img = self.transform(img)
        return img, np.array([label], dtype="int64")


class MNIST(_Synthetic):
    pass


class FashionMNIST(_Synthetic):
    pass


class Cifar10(_Synthetic):
    shape = (3, 32, 32)
    sizes = {"train": 50000, "test": 10000}


class Cifar100(Cifar10):
    classes = 100


class Flowers(_Synthetic):
    shape = (3, 224, 224)
    classes = 102
    sizes = {"train": 6149, "test": 1020, "valid": 1020}


class ImageNetSynthetic(_Synthetic):
    shape = (3, 224, 224)
    classes = 1000
    sizes = {"train": 1281167, "test": 50000}
