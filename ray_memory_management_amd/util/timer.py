"""Running-mean timer. Parity: reference python/ray/util/timer.py (_Timer)."""
from __future__ import annotations

import time


class _Timer:
    def __init__(self, window_size: int = 10):
        self._window_size = window_size
        self._samples = []
        self._units_processed = []
        self._start_time = None
        self._total_time = 0.0
        self.count = 0

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *exc):
        self.stop()

    def start(self):
        self._start_time = time.perf_counter()

    def stop(self):
        self.push(time.perf_counter() - self._start_time)
        self._start_time = None

    def push(self, dt):
        self._samples.append(dt)
        self._samples = self._samples[-self._window_size:]
        self._total_time += dt
        self.count += 1

    def push_units_processed(self, n):
        self._units_processed.append(n)
        self._units_processed = self._units_processed[-self._window_size:]

    def reset(self):
        self.__init__(self._window_size)

    @property
    def mean(self):
        return sum(self._samples) / len(self._samples) if self._samples else 0.0

    @property
    def median(self):
        s = sorted(self._samples)
        return s[len(s) // 2] if s else 0.0

    @property
    def sum(self):
        return self._total_time

    @property
    def max(self):
        return max(self._samples) if self._samples else 0.0

    @property
    def mean_units_processed(self):
        return sum(self._units_processed) / len(self._units_processed) if self._units_processed else 0.0

    @property
    def mean_throughput(self):
        t = sum(self._samples)
        return sum(self._units_processed) / t if t else 0.0
