"""Record files and tensor serialisation helpers shared by fluid and dygraph.

RecordIO via the native runtime (csrc/runtime/recordio.cc); each record written
by ``write_tensors`` is a concatenation of LoDTensor streams (framework/
serialization.py format), so recordio readers yield ready-to-feed LoDTensors.
"""
from __future__ import annotations

import io as _io

from ..framework import serialization as S


class Compressor:
    NoCompress = 0
    Snappy = 1  # not available in this image: written as Gzip (2)
    Gzip = 2


class RecordIOWriter:
    def __init__(self, filename, compressor=Compressor.Gzip, max_num_records=1000):
        from ..runtime import RecordIOWriter as _W

        self._w = _W(filename, compressor, max_num_records)

    def write(self, record: bytes):
        self._w.write(record)

    def write_tensors(self, lod_tensors):
        b = _io.BytesIO()
        for t in lod_tensors:
            S.write_lod_tensor(b, t)
        self._w.write(b.getvalue())

    def close(self):
        self._w.close()


def recordio_records(filename):
    from ..runtime import RecordIOScanner

    yield from RecordIOScanner(filename)


def recordio_iter(filename, n_slots=None):
    """Yields lists of numpy arrays (one per slot) from a tensor RecordIO file."""
    for rec in recordio_records(filename):
        b = _io.BytesIO(rec)
        out = []
        while b.tell() < len(rec):
            out.append(S.read_lod_tensor(b).numpy())
        yield out
