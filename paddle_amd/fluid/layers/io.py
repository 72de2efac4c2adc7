"""Data-input layers (python/paddle/fluid/layers/io.py: data :38, py_reader :474,
open_files :724, double_buffer :891, read_file, shuffle, batch)."""
from __future__ import annotations

import contextlib

from ...framework import core
from ..framework import Variable, default_main_program, default_startup_program
from ..layer_helper import LayerHelper


def data(name, shape, append_batch_size=True, dtype="float32", lod_level=0, type=core.VT.LOD_TENSOR,
         stop_gradient=True):
    helper = LayerHelper("data", name=name)
    shape = list(shape)
    for i in range(len(shape)):
        if shape[i] is None:
            shape[i] = -1
            append_batch_size = False
        elif shape[i] < 0:
            append_batch_size = False
    if append_batch_size:
        shape = [-1] + shape
    return helper.create_global_variable(name=name, shape=shape, dtype=dtype, type=type,
                                         stop_gradient=stop_gradient, lod_level=lod_level, is_data=True)


class _PyReaderHandle:
    """Host-side reader feeding a list of data vars (py_reader semantics, reference
    layers/io.py:474 + operators/reader/create_py_reader_op.cc).

    ``start()`` runs the decorated provider on a Python thread that pushes every
    batch into the native double-buffer pipeline (paddle_amd.runtime.
    DoubleBufferReader, csrc/runtime/reader.cc): pinned host staging, a C++
    prefetch thread copying the next batches to the device on its own HIP stream
    (``use_double_buffer`` on a GPU), and a stream-ordered hand-off to the
    executor's stream.  ``Executor.run`` pulls one batch per call for programs
    that own a started reader; ``next_feed`` raises EOFException at the end.
    Without the runtime library a Python queue is used instead.
    """

    def __init__(self, capacity, feed_vars, use_double_buffer=True):
        self.capacity = capacity
        self.feed_vars = feed_vars
        self._provider = None
        self._thread = None
        self._native = None
        self._q = None
        self.started = False
        self.use_double_buffer = use_double_buffer
        self._error = None

    def decorate_tensor_provider(self, provider):
        p = provider
        for fn in getattr(self, "_decorators", []):   # in-graph batch()/shuffle() applied earlier
            p = (lambda p=p, fn=fn: fn(p()))
        self._provider = p

    decorate_paddle_reader = decorate_tensor_provider
    decorate_batch_generator = decorate_tensor_provider

    def _make_native(self):
        try:
            import torch

            from ... import runtime
            if not runtime.available():
                return None
            dev = "cuda" if self.use_double_buffer and torch.cuda.is_available() else None
            return runtime.DoubleBufferReader(capacity=max(1, self.capacity), nslots=2, device=dev)
        except (OSError, RuntimeError):
            return None

    def start(self):
        import queue
        import threading

        import numpy as np

        if self._provider is None:
            raise RuntimeError("py_reader: decorate a provider before start()")
        if self._native is None:
            self._native = self._make_native()
        else:
            self._native.reset()
        if self._native is None:
            self._q = queue.Queue(maxsize=self.capacity)
        self._error = None

        def run():
            try:
                for item in self._provider():
                    arrs = [np.asarray(x.numpy() if hasattr(x, "numpy") else x) for x in item]
                    if self._native is not None:
                        if not self._native.push(arrs):
                            return  # reset() closed the pipeline
                    else:
                        self._q.put(arrs)
            except BaseException as e:  # surfaces in next_feed
                self._error = e
            finally:
                if self._native is not None:
                    self._native.close()
                else:
                    self._q.put(None)

        self._thread = threading.Thread(target=run, daemon=True)
        self._thread.start()
        self.started = True

    def reset(self):
        if self._native is not None:
            self._native.close()
        elif self._q is not None:
            while self._q.qsize():
                self._q.get_nowait()
        if self._thread is not None:
            self._thread.join(timeout=5)
        self._thread = None
        self.started = False

    def next_feed(self):
        if self._native is not None:
            item = self._native.next()
        else:
            item = self._q.get()
        if self._error is not None:
            raise self._error
        if item is None:
            self.started = False
            raise core_EOF()
        return {v.name: x for v, x in zip(self.feed_vars, item)}


core_EOF = core.EOFException  # raised when a reader is exhausted (platform/enforce.h)


EOFException = core_EOF


def py_reader(capacity, shapes, dtypes, lod_levels=None, name=None, use_double_buffer=True):
    lod_levels = lod_levels or [0] * len(shapes)
    vars_ = []
    for i, (s, d, l) in enumerate(zip(shapes, dtypes, lod_levels)):
        vars_.append(data(name=f"{name or 'py_reader'}_data_{i}", shape=s, dtype=d, lod_level=l,
                          append_batch_size=False))
    r = _PyReaderHandle(capacity, vars_, use_double_buffer)
    r.vars = vars_
    prog = default_main_program()
    if not hasattr(prog, "_py_readers"):
        prog._py_readers = []
    prog._py_readers.append(r)
    return r


def read_file(reader):
    return reader.vars if len(reader.vars) > 1 else reader.vars[0]


def double_buffer(reader, place=None, name=None):
    reader.use_double_buffer = True
    return reader


def _wrap_provider(reader, fn):
    inner = reader._provider
    reader._provider = (lambda: fn(inner())) if inner is not None else None
    reader._decorators = getattr(reader, "_decorators", []) + [fn]
    return reader


def batch(reader, batch_size):
    """create_batch_reader: stack ``batch_size`` consecutive samples per field."""
    import numpy as np

    def gen(it):
        buf = []
        for item in it:
            buf.append(item)
            if len(buf) == batch_size:
                yield [np.stack([np.asarray(b[i]) for b in buf]) for i in range(len(buf[0]))]
                buf = []
        if buf:
            yield [np.stack([np.asarray(b[i]) for b in buf]) for i in range(len(buf[0]))]

    return _wrap_provider(reader, gen)


def shuffle(reader, buffer_size):
    """create_shuffle_reader: buffered shuffle over ``buffer_size`` items."""
    import random

    def gen(it):
        buf = []
        for item in it:
            buf.append(item)
            if len(buf) >= buffer_size:
                random.shuffle(buf)
                yield from buf
                buf = []
        random.shuffle(buf)
        yield from buf

    return _wrap_provider(reader, gen)


def open_recordio_file(filename, shapes, lod_levels, dtypes, pass_num=1, for_parallel=True):
    """Reader over one RecordIO file (reference io.py open_recordio_file)."""
    return open_files([filename], shapes, lod_levels, dtypes, pass_num=pass_num)


class Preprocessor:
    """Per-batch preprocessing sub-program on a reader's output (reference
    io.py Preprocessor / create_custom_reader_op.cc)::

        p = fluid.layers.io.Preprocessor(reader=r)
        with p.block():
            img, lbl = p.inputs()
            p.outputs(img / 2, lbl + 1)
        r2 = p()
    """

    BEFORE_SUB_BLOCK, IN_SUB_BLOCK, AFTER_SUB_BLOCK = 0, 1, 2

    def __init__(self, reader, name=None):
        from ..framework import Program

        self.underlying_reader = reader
        self.name = name or "preprocessor"
        self.status = Preprocessor.BEFORE_SUB_BLOCK
        self.prog, self.startup = Program(), Program()
        self.source_vars = None
        self.sink_vars = None

    @contextlib.contextmanager
    def block(self):
        from ..framework import program_guard

        self.status = Preprocessor.IN_SUB_BLOCK
        with program_guard(self.prog, self.startup):
            yield
        self.status = Preprocessor.AFTER_SUB_BLOCK
        if self.sink_vars is None:
            raise RuntimeError("Preprocessor: outputs() was not called inside block()")

    def inputs(self):
        if self.status != Preprocessor.IN_SUB_BLOCK:
            raise RuntimeError("Preprocessor.inputs() can only be invoked inside the sub-block.")
        self.source_vars = [data(name=f"{self.name}_in_{i}", shape=list(v.shape), dtype=v.dtype,
                                 lod_level=v.lod_level, append_batch_size=False)
                            for i, v in enumerate(self.underlying_reader.vars)]
        return self.source_vars

    def outputs(self, *outs):
        if self.status != Preprocessor.IN_SUB_BLOCK:
            raise RuntimeError("Preprocessor.outputs() can only be invoked inside the sub-block.")
        self.sink_vars = list(outs)

    def __call__(self, *args, **kwargs):
        if self.status != Preprocessor.AFTER_SUB_BLOCK:
            raise RuntimeError("Preprocessor output can only be retrieved after rnn block.")
        from ...framework import core as _core
        from ..executor import Executor

        out = py_reader(capacity=self.underlying_reader.capacity, shapes=[list(v.shape) for v in self.sink_vars],
                        dtypes=[v.dtype for v in self.sink_vars], lod_levels=[v.lod_level or 0 for v in self.sink_vars],
                        name=self.name)
        src, sink, prog, inner = self.source_vars, self.sink_vars, self.prog, self.underlying_reader

        def provider():
            exe = Executor(_core.CPUPlace())
            scope = _core.Scope()
            from ..executor import scope_guard

            with scope_guard(scope):
                for item in inner._provider():
                    yield exe.run(prog, feed={v.name: x for v, x in zip(src, item)}, fetch_list=sink)

        out.decorate_tensor_provider(provider)
        return out


def open_files(filenames, shapes, lod_levels, dtypes, thread_num=None, buffer_size=None, pass_num=1,
               is_test=None):
    from ... import io as pio

    r = py_reader(capacity=buffer_size or 64, shapes=shapes, dtypes=dtypes, lod_levels=lod_levels)

    def provider():
        for _ in range(pass_num):
            for fn in filenames:
                for rec in pio.recordio_iter(fn):
                    yield rec

    r.decorate_tensor_provider(provider)
    return r


def random_data_generator(low, high, shapes, lod_levels, for_parallel=True):
    import numpy as np

    r = py_reader(capacity=8, shapes=shapes, dtypes=["float32"] * len(shapes), lod_levels=lod_levels)

    def provider():
        while True:
            yield [np.random.uniform(low, high, [abs(x) for x in s]).astype("float32") for s in shapes]

    r.decorate_tensor_provider(provider)
    return r


def load(out, file_path, load_as_fp16=None):
    helper = LayerHelper("load")
    attrs = {"file_path": file_path}
    if load_as_fp16 is not None:
        attrs["load_as_fp16"] = load_as_fp16
    helper.append_op(type="load", inputs={}, outputs={"Out": [out]}, attrs=attrs)
