"""Reader decorators: a reader is a zero-arg callable returning an iterator."""
from __future__ import annotations

import itertools
import queue
import random
import threading


class ComposeNotAligned(ValueError):
    pass


def batch(reader, batch_size, drop_last=False):
    def batch_reader():
        b = []
        for instance in reader():
            b.append(instance)
            if len(b) == batch_size:
                yield b
                b = []
        if drop_last is False and len(b) != 0:
            yield b

    if int(batch_size) <= 0:
        raise ValueError("batch_size should be a positive integer")
    return batch_reader


def map_readers(func, *readers):
    def reader():
        rs = [r() for r in readers]
        for e in map(func, *rs):
            yield e

    return reader


def shuffle(reader, buf_size):
    def data_reader():
        buf = []
        for e in reader():
            buf.append(e)
            if len(buf) >= buf_size:
                random.shuffle(buf)
                yield from buf
                buf = []
        if buf:
            random.shuffle(buf)
            yield from buf

    return data_reader


def chain(*readers):
    def reader():
        return itertools.chain(*[r() for r in readers])

    return reader


def compose(*readers, **kwargs):
    check_alignment = kwargs.pop("check_alignment", True)

    def make_tuple(x):
        return x if isinstance(x, tuple) else (x,)

    def reader():
        rs = [r() for r in readers]
        if not check_alignment:
            for outputs in zip(*rs):
                yield sum(list(map(make_tuple, outputs)), ())
        else:
            for outputs in itertools.zip_longest(*rs):
                for o in outputs:
                    if o is None:
                        raise ComposeNotAligned("outputs of readers are not aligned.")
                yield sum(list(map(make_tuple, outputs)), ())

    return reader


def buffered(reader, size):
    class EndSignal:
        pass

    end = EndSignal()

    def read_worker(r, q):
        for d in r:
            q.put(d)
        q.put(end)

    def data_reader():
        r = reader()
        q = queue.Queue(maxsize=size)
        t = threading.Thread(target=read_worker, args=(r, q), daemon=True)
        t.start()
        e = q.get()
        while e is not end:
            yield e
            e = q.get()

    return data_reader


def firstn(reader, n):
    def firstn_reader():
        for i, item in enumerate(reader()):
            if i == n:
                break
            yield item

    return firstn_reader


def cache(reader):
    all_data = tuple(reader())

    def __impl__():
        yield from all_data

    return __impl__


def xmap_readers(mapper, reader, process_num, buffer_size, order=False):
    end = object()

    def xreader():
        in_q, out_q = queue.Queue(buffer_size), queue.Queue(buffer_size)

        def feed():
            for i, s in enumerate(reader()):
                in_q.put((i, s))
            for _ in range(process_num):
                in_q.put(end)

        def work():
            while True:
                it = in_q.get()
                if it is end:
                    out_q.put(end)
                    return
                out_q.put((it[0], mapper(it[1])))

        threading.Thread(target=feed, daemon=True).start()
        for _ in range(process_num):
            threading.Thread(target=work, daemon=True).start()
        finished, pending, nxt = 0, {}, 0
        while finished < process_num:
            r = out_q.get()
            if r is end:
                finished += 1
                continue
            if not order:
                yield r[1]
                continue
            pending[r[0]] = r[1]
            while nxt in pending:
                yield pending.pop(nxt)
                nxt += 1
        for k in sorted(pending):
            yield pending[k]

    return xreader


def multiprocess_reader(readers, use_pipe=True, queue_size=1000):
    return chain(*readers)
