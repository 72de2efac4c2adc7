"""Parameter-block -> pserver dispatchers (transpiler/ps_dispatcher.py)."""
from __future__ import annotations

import zlib


class PSDispatcher:
    def __init__(self, pserver_endpoints):
        self._eps = pserver_endpoints
        self._step = 0

    @property
    def eps(self):
        return self._eps

    def reset(self):
        self._step = 0

    def dispatch(self, varlist):
        raise NotImplementedError


class HashName(PSDispatcher):
    def _hash_block(self, block_str, total):
        return zlib.crc32(block_str.encode()) % total

    def dispatch(self, varlist):
        return [self._eps[self._hash_block(v.name if hasattr(v, "name") else str(v), len(self._eps))]
                for v in varlist]


class RoundRobin(PSDispatcher):
    def dispatch(self, varlist):
        eplist = []
        for _ in varlist:
            eplist.append(self._eps[self._step])
            self._step = (self._step + 1) % len(self._eps)
        return eplist
