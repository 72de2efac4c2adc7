"""Named timer statistics (reference paddle/legacy/utils/Stat.h: StatSet, Stat,
REGISTER_TIMER / TimerOnce, ``globalStat.printAllStatus()`` / ``reset()``): total,
count, max, min and average wall time per name, thread-safe; the v1 trainer
(``--log_stat=1``) prints and resets them every log period."""
from __future__ import annotations

import contextlib
import threading
import time


class Stat:
    __slots__ = ("name", "total", "count", "max", "min")

    def __init__(self, name):
        self.name = name
        self.total, self.count, self.max, self.min = 0.0, 0, 0.0, float("inf")

    def add(self, seconds):
        self.total += seconds
        self.count += 1
        self.max = max(self.max, seconds)
        self.min = min(self.min, seconds)

    def line(self):
        avg = self.total / self.count if self.count else 0.0
        mn = self.min if self.count else 0.0
        return (f"Stat={self.name:<24} total={self.total * 1e3:10.3f}ms avg={avg * 1e3:9.3f}ms "
                f"max={self.max * 1e3:9.3f}ms min={mn * 1e3:9.3f}ms count={self.count}")


class StatSet:
    def __init__(self, name="GlobalStatInfo"):
        self.name = name
        self._stats: dict[str, Stat] = {}
        self._lock = threading.Lock()

    def get(self, name) -> Stat:
        with self._lock:
            s = self._stats.get(name)
            if s is None:
                s = self._stats[name] = Stat(name)
            return s

    def add(self, name, seconds):
        s = self.get(name)
        with self._lock:
            s.add(seconds)

    @contextlib.contextmanager
    def timer(self, name):
        """REGISTER_TIMER(name): time the enclosed block into stat ``name``."""
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.add(name, time.perf_counter() - t0)

    def status(self) -> str:
        with self._lock:
            lines = [s.line() for s in sorted(self._stats.values(), key=lambda s: -s.total)]
        return "\n".join([f"======= StatSet: [{self.name}] status ======"] + lines)

    def print_all_status(self, file=None):
        print(self.status(), file=file, flush=True)

    def reset(self):
        with self._lock:
            self._stats.clear()

    def as_dict(self):
        with self._lock:
            return {k: {"total": s.total, "count": s.count, "max": s.max, "min": s.min}
                    for k, s in self._stats.items()}


global_stat = StatSet()
timer = global_stat.timer
