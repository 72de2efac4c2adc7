"""DataFeeder: python samples -> LoDTensors (python/paddle/fluid/data_feeder.py:83)."""
from __future__ import annotations

import numpy as np

from ..framework import core
from .framework import Variable, default_main_program


class DataToLoDTensorConverter:
    def __init__(self, place, lod_level, shape, dtype):
        self.place, self.lod_level, self.shape = place, lod_level, shape
        self.dtype = {core.VT.FP32: "float32", core.VT.INT64: "int64", core.VT.FP64: "float64",
                      core.VT.INT32: "int32", core.VT.UINT8: "uint8", core.VT.BOOL: "bool",
                      core.VT.FP16: "float16"}.get(dtype, "float32")
        self.data = []
        self.lod = [[] for _ in range(lod_level)]

    def feed(self, data):
        self._feed_impl_(data, self.lod, self.lod_level)

    def _feed_impl_(self, data, lod, lod_level):
        if lod_level == 0:
            self.data.append(data)
        else:
            lod[0].append(len(data))
            for each in data:
                self._feed_impl_(each, lod[1:], lod_level - 1)

    def done(self):
        arr = np.array(self.data, dtype=self.dtype)
        if self.shape and self.lod_level == 0:
            shape = [s if s >= 0 else -1 for s in self.shape]
            if shape.count(-1) <= 1:
                arr = arr.reshape(shape)
        elif self.lod_level > 0 and arr.ndim == 1:
            arr = arr.reshape(-1, 1)
        t = core.LoDTensor()
        t.set(arr, self.place)
        if self.lod_level > 0:
            t.set_recursive_sequence_lengths(self.lod)
        return t


class DataFeeder:
    def __init__(self, feed_list, place, program=None):
        self.feed_dtypes, self.feed_names, self.feed_shapes, self.feed_lod_level = [], [], [], []
        if program is None:
            program = default_main_program()
        for each in feed_list:
            if isinstance(each, str):
                each = program.global_block().var(each)
            if not isinstance(each, Variable):
                raise TypeError("Feed list should contain a list of variable")
            self.feed_dtypes.append(each.dtype)
            self.feed_names.append(each.name)
            self.feed_lod_level.append(each.lod_level)
            self.feed_shapes.append(list(each.shape))
        self.place = place

    def feed(self, iterable):
        converters = [DataToLoDTensorConverter(self.place, l, s, d) for l, s, d in
                      zip(self.feed_lod_level, self.feed_shapes, self.feed_dtypes)]
        for each_sample in iterable:
            assert len(each_sample) == len(converters), "sample/feed_list length mismatch"
            for each_converter, each_slot in zip(converters, each_sample):
                each_converter.feed(each_slot)
        return {n: c.done() for n, c in zip(self.feed_names, converters)}

    def feed_parallel(self, iterable, num_places=None):
        for batch in iterable:
            yield self.feed(batch)

    def decorate_reader(self, reader, multi_devices, num_places=None, drop_last=True):
        def r():
            for item in reader():
                yield self.feed(item)

        return r
