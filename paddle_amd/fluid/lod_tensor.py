"""create_lod_tensor / create_random_int_lodtensor (python/paddle/fluid/lod_tensor.py)."""
from __future__ import annotations

import numpy as np

from ..framework import core
from .data_feeder import DataToLoDTensorConverter


def create_lod_tensor(data, recursive_seq_lens, place):
    if isinstance(data, core.LoDTensor):
        return create_lod_tensor(np.array(data), recursive_seq_lens, place)
    if isinstance(data, list):
        new_lod = []
        flat = []
        for seq in data:
            new_lod.append(len(seq))
            flat.extend(seq)
        assert [new_lod] == recursive_seq_lens, "data and recursive_seq_lens do not match"
        arr = np.array(flat)
        if arr.ndim == 1:
            arr = arr.reshape(-1, 1)
        return create_lod_tensor(arr, recursive_seq_lens, place)
    if isinstance(data, np.ndarray):
        t = core.LoDTensor()
        t.set(data, place)
        t.set_recursive_sequence_lengths(recursive_seq_lens)
        assert t.has_valid_recursive_sequence_lengths(), "the provided lod info is invalid"
        return t
    raise TypeError("data should be either a LoDTensor, a Numpy array or a list")


def create_random_int_lodtensor(recursive_seq_lens, base_shape, place, low, high):
    overall = [sum(recursive_seq_lens[-1])] + list(base_shape)
    data = np.random.random_integers(low, high, overall).astype("int64") if hasattr(np.random, "random_integers") \
        else np.random.randint(low, high + 1, overall).astype("int64")
    return create_lod_tensor(data, recursive_seq_lens, place)
