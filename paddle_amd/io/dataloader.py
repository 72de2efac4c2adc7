"""``paddle.io``: Dataset / Sampler / BatchSampler / DistributedBatchSampler / DataLoader.

Reference parity: the Fluid reader stack -- ``py_reader`` over a
``LoDTensorBlockingQueue`` with a double-buffered async H2D copy
(paddle/fluid/operators/reader/{create_py_reader_op.cc, buffered_reader.cc,
lod_tensor_blocking_queue.h}) and the ``paddle.reader`` decorators
(xmap_readers, buffered).

MI355X design: worker *threads* (``num_workers``) produce collated batches into a
bounded queue (numpy/torch collation releases the GIL for the heavy copies); the
consumer side pins host memory and issues the H2D copy on a dedicated HIP stream
one batch ahead (``prefetch_to_device``), so the copy of batch i+1 overlaps the
compute of batch i -- the MI355X analogue of the reference's double buffer.
"""
from __future__ import annotations

import math
import queue
import random
import threading

import numpy as np
import torch


class Dataset:
    def __getitem__(self, idx):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError


class IterableDataset(Dataset):
    def __iter__(self):
        raise NotImplementedError


class TensorDataset(Dataset):
    def __init__(self, tensors):
        self.tensors = list(tensors)
        n = len(self.tensors[0])
        if any(len(t) != n for t in self.tensors):
            raise ValueError("tensors must share the first dimension")

    def __getitem__(self, i):
        return tuple(t[i] for t in self.tensors)

    def __len__(self):
        return len(self.tensors[0])


class ComposeDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __len__(self):
        return len(self.datasets[0])

    def __getitem__(self, i):
        out = []
        for d in self.datasets:
            s = d[i]
            out.extend(s if isinstance(s, (tuple, list)) else [s])
        return tuple(out)


class ChainDataset(IterableDataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __iter__(self):
        for d in self.datasets:
            yield from d


class Subset(Dataset):
    def __init__(self, dataset, indices):
        self.dataset, self.indices = dataset, list(indices)

    def __getitem__(self, i):
        return self.dataset[self.indices[i]]

    def __len__(self):
        return len(self.indices)


def random_split(dataset, lengths, generator=None):
    n = len(dataset)
    if all(0 < x < 1 for x in lengths):
        lengths = [int(math.floor(n * x)) for x in lengths]
        lengths[-1] += n - sum(lengths)
    perm = np.random.permutation(n).tolist()
    out, o = [], 0
    for L in lengths:
        out.append(Subset(dataset, perm[o:o + L]))
        o += L
    return out


# ------------------------------------------------------------------- samplers
class Sampler:
    def __init__(self, data_source=None):
        self.data_source = data_source


class SequenceSampler(Sampler):
    def __iter__(self):
        return iter(range(len(self.data_source)))

    def __len__(self):
        return len(self.data_source)


class RandomSampler(Sampler):
    def __init__(self, data_source, replacement=False, num_samples=None, generator=None):
        super().__init__(data_source)
        self.replacement, self.num_samples = replacement, num_samples

    def __iter__(self):
        n = len(self.data_source)
        k = self.num_samples or n
        if self.replacement:
            return iter(np.random.randint(0, n, k).tolist())
        return iter(np.random.permutation(n)[:k].tolist())

    def __len__(self):
        return self.num_samples or len(self.data_source)


class WeightedRandomSampler(Sampler):
    def __init__(self, weights, num_samples, replacement=True):
        self.weights = np.asarray(weights, dtype=np.float64)
        self.num_samples, self.replacement = num_samples, replacement

    def __iter__(self):
        p = self.weights / self.weights.sum()
        return iter(np.random.choice(len(p), self.num_samples, self.replacement, p).tolist())

    def __len__(self):
        return self.num_samples


class BatchSampler(Sampler):
    def __init__(self, dataset=None, sampler=None, shuffle=False, batch_size=1, drop_last=False):
        if sampler is None:
            sampler = RandomSampler(dataset) if shuffle else SequenceSampler(dataset)
        self.sampler, self.batch_size, self.drop_last = sampler, batch_size, drop_last

    def __iter__(self):
        b = []
        for i in self.sampler:
            b.append(i)
            if len(b) == self.batch_size:
                yield b
                b = []
        if b and not self.drop_last:
            yield b

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size


class DistributedBatchSampler(BatchSampler):
    """Each rank sees a disjoint 1/world slice of the (optionally shuffled, padded)
    index list; ``set_epoch`` reseeds the shuffle identically on every rank."""

    def __init__(self, dataset, batch_size, num_replicas=None, rank=None, shuffle=False, drop_last=False):
        from ..parallel import comm

        self.dataset, self.batch_size, self.shuffle, self.drop_last = dataset, batch_size, shuffle, drop_last
        self.nranks = num_replicas if num_replicas is not None else comm.get_world_size()
        self.local_rank = rank if rank is not None else comm.get_rank()
        self.epoch = 0
        self.num_samples = int(math.ceil(len(dataset) / self.nranks))
        self.total_size = self.num_samples * self.nranks

    def set_epoch(self, epoch):
        self.epoch = epoch

    def __iter__(self):
        idx = list(range(len(self.dataset)))
        if self.shuffle:
            rng = np.random.RandomState(self.epoch)
            rng.shuffle(idx)
            self.epoch += 1
        idx += idx[:self.total_size - len(idx)]
        idx = idx[self.local_rank:self.total_size:self.nranks]
        b = []
        for i in idx:
            b.append(i)
            if len(b) == self.batch_size:
                yield b
                b = []
        if b and not self.drop_last:
            yield b

    def __len__(self):
        n = self.num_samples
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size


# ------------------------------------------------------------------- collation
def default_collate_fn(batch):
    s = batch[0]
    if torch.is_tensor(s):
        return torch.stack(batch)
    if isinstance(s, np.ndarray):
        return torch.from_numpy(np.stack(batch))
    if isinstance(s, (int, np.integer)):
        return torch.tensor(batch, dtype=torch.int64)
    if isinstance(s, (float, np.floating)):
        return torch.tensor(batch, dtype=torch.float32)
    if isinstance(s, dict):
        return {k: default_collate_fn([b[k] for b in batch]) for k in s}
    if isinstance(s, (tuple, list)):
        return [default_collate_fn(list(x)) for x in zip(*batch)]
    return batch


def default_convert_fn(batch):
    return batch


def _to_device(x, device, stream=None):
    if torch.is_tensor(x):
        if x.device.type == "cpu" and device.type == "cuda":
            x = x.pin_memory() if not x.is_pinned() else x
        return x.to(device, non_blocking=True)
    if isinstance(x, dict):
        return {k: _to_device(v, device) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_device(v, device) for v in x)
    return x


_END = object()


class DataLoader:
    def __init__(self, dataset, feed_list=None, places=None, return_list=True, batch_sampler=None, batch_size=1,
                 shuffle=False, drop_last=False, collate_fn=None, num_workers=0, use_buffer_reader=True,
                 prefetch_factor=2, use_shared_memory=True, timeout=0, worker_init_fn=None,
                 persistent_workers=False, device=None):
        self.dataset = dataset
        self.collate_fn = collate_fn or default_collate_fn
        self.num_workers = num_workers
        self.prefetch = max(1, prefetch_factor) * max(1, num_workers)
        self.iterable = isinstance(dataset, IterableDataset)
        self.batch_size = batch_size
        self.drop_last = drop_last
        if batch_sampler is not None:
            self.batch_sampler = batch_sampler
        elif not self.iterable and batch_size is not None:
            self.batch_sampler = BatchSampler(dataset, shuffle=shuffle, batch_size=batch_size, drop_last=drop_last)
        else:
            self.batch_sampler = None
        if device is None and places is not None:
            pl = places[0] if isinstance(places, (list, tuple)) else places
            device = getattr(pl, "torch_device", None)
            device = device() if callable(device) else device
        self.device = torch.device(device) if device is not None else None
        self.use_buffer_reader = use_buffer_reader
        self.worker_init_fn = worker_init_fn

    def __len__(self):
        if self.batch_sampler is None:
            raise TypeError("length of an IterableDataset loader is unknown")
        return len(self.batch_sampler)

    def _batches(self):
        if self.iterable:
            if self.batch_size is None:
                yield from self.dataset
                return
            b = []
            for s in self.dataset:
                b.append(s)
                if len(b) == self.batch_size:
                    yield self.collate_fn(b)
                    b = []
            if b and not self.drop_last:
                yield self.collate_fn(b)
            return
        if self.batch_sampler is None:
            for i in range(len(self.dataset)):
                yield self.dataset[i]
            return
        if self.num_workers <= 0:
            for idx in self.batch_sampler:
                yield self.collate_fn([self.dataset[i] for i in idx])
            return
        # threaded workers, ordered output
        idx_q: queue.Queue = queue.Queue()
        out: dict = {}
        cv = threading.Condition()
        batches = list(self.batch_sampler)
        for k, b in enumerate(batches):
            idx_q.put((k, b))
        stop = threading.Event()

        def work(wid):
            if self.worker_init_fn is not None:
                self.worker_init_fn(wid)
            while not stop.is_set():
                try:
                    k, b = idx_q.get_nowait()
                except queue.Empty:
                    return
                with cv:
                    while k - nxt[0] >= self.prefetch and not stop.is_set():
                        cv.wait(0.05)
                try:
                    r = self.collate_fn([self.dataset[i] for i in b])
                except Exception as e:  # noqa: BLE001
                    r = e
                with cv:
                    out[k] = r
                    cv.notify_all()

        nxt = [0]
        ts = [threading.Thread(target=work, args=(w,), daemon=True) for w in range(self.num_workers)]
        for t in ts:
            t.start()
        try:
            for k in range(len(batches)):
                with cv:
                    while k not in out:
                        cv.wait(0.05)
                    r = out.pop(k)
                    nxt[0] = k + 1
                    cv.notify_all()
                if isinstance(r, Exception):
                    raise r
                yield r
        finally:
            stop.set()

    def __iter__(self):
        it = self._batches()
        if self.device is None or self.device.type != "cuda":
            yield from it
            return
        stream = torch.cuda.Stream(device=self.device)
        nxt = None
        for b in it:
            with torch.cuda.stream(stream):
                cur = _to_device(b, self.device)
            ev = stream.record_event()
            if nxt is not None:
                yield nxt
            torch.cuda.current_stream(self.device).wait_event(ev)
            nxt = cur
        if nxt is not None:
            yield nxt

    def __call__(self):
        return self.__iter__()


def get_worker_info():
    return None
