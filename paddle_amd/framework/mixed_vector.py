"""Device mirror of LoD offsets (the reference's MixedVector, framework/
mixed_vector.h: a host vector with a lazily synced device copy, which is how LoD
reaches CUDA kernels).

LoD offsets live on the host as Python lists (lod_tensor.h keeps them host-side
too); sequence kernels need them on the device.  ``device_offsets`` uploads a given
offset vector once -- from a pinned staging copy, asynchronously on the current
stream -- and hands the same device tensor to every later op that sees the same
offsets (forward and backward of a sequence op, several ops over one batch), so a
LoD op costs no synchronous host-to-device copy.  Entries are keyed by value (the
offsets are immutable tuples) in a small LRU."""
from __future__ import annotations

import collections
import threading

import torch

_CAP = 512
_cache: "collections.OrderedDict" = collections.OrderedDict()
_lock = threading.Lock()
_stats = {"hits": 0, "uploads": 0}


def device_offsets(offsets, device, dtype=torch.int64):
    """The device tensor holding ``offsets`` (read-only for the kernels)."""
    device = torch.device(device)
    if device.type != "cuda":
        return torch.as_tensor(list(offsets), dtype=dtype)
    key = (tuple(int(o) for o in offsets), device.index, dtype)
    with _lock:
        ent = _cache.get(key)
        if ent is not None:
            _cache.move_to_end(key)
            _stats["hits"] += 1
            return ent[0]
    host = torch.tensor(key[0], dtype=dtype).pin_memory()
    dev = host.to(device, non_blocking=True)
    with _lock:
        _cache[key] = (dev, host)  # the pinned source stays alive while the copy may run
        _stats["uploads"] += 1
        while len(_cache) > _CAP:
            _cache.popitem(last=False)
    return dev


def stats():
    return dict(_stats)


def clear():
    with _lock:
        _cache.clear()
