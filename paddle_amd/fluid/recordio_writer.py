"""RecordIO conversion helpers (python/paddle/fluid/recordio_writer.py).

Records are serialized LoDTensor lists written through :mod:`paddle_amd.io`
(native C++ RecordIO writer when the runtime library is built)."""
from __future__ import annotations

import contextlib

from .. import io as pio

__all__ = ["convert_reader_to_recordio_file", "convert_reader_to_recordio_files"]


@contextlib.contextmanager
def create_recordio_writer(filename, compressor=pio.Compressor.Snappy, max_num_records=1000):
    w = pio.RecordIOWriter(filename, compressor, max_num_records)
    try:
        yield w
    finally:
        w.close()


def convert_reader_to_recordio_file(filename, reader_creator, feeder, compressor=pio.Compressor.Snappy,
                                    max_num_records=1000, feed_order=None):
    if feed_order is None:
        feed_order = feeder.feed_names
    counter = 0
    with create_recordio_writer(filename, compressor, max_num_records) as writer:
        for batch in reader_creator():
            res = feeder.feed(batch)
            writer.write_tensors([res[n] for n in feed_order])
            counter += 1
    return counter


def convert_reader_to_recordio_files(filename, batch_per_file, reader_creator, feeder,
                                     compressor=pio.Compressor.Snappy, max_num_records=1000, feed_order=None):
    if feed_order is None:
        feed_order = feeder.feed_names
    f_name, f_ext = filename.rsplit(".", 1) if "." in filename else (filename, "recordio")
    lines = []
    f_idx = 0
    counter = 0
    for idx, batch in enumerate(reader_creator()):
        lines.append(batch)
        if idx >= batch_per_file and idx % batch_per_file == 0:
            fn = f"{f_name}-{f_idx:05d}.{f_ext}"
            with create_recordio_writer(fn, compressor, max_num_records) as writer:
                for l in lines:
                    res = feeder.feed(l)
                    writer.write_tensors([res[n] for n in feed_order])
                    counter += 1
            lines = []
            f_idx += 1
    if lines:
        fn = f"{f_name}-{f_idx:05d}.{f_ext}"
        with create_recordio_writer(fn, compressor, max_num_records) as writer:
            for l in lines:
                res = feeder.feed(l)
                writer.write_tensors([res[n] for n in feed_order])
                counter += 1
    return counter
