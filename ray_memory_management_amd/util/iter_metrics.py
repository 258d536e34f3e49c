"""Execution metrics shared along a LocalIterator chain.

Role parity: reference python/ray/util/iter_metrics.py (``MetricsContext``, ``SharedMetrics``, used by
RLlib's execution-plan operators through ``LocalIterator.get_metrics()``). Every operator of one
driver-side iterator chain sees the same context; ``union`` points the contexts of the joined chains
at one object.
"""
from __future__ import annotations

import collections
from typing import List, Optional

from ray_memory_management_amd.util.timer import _Timer


class MetricsContext:
    """counters (monotone ints), timers (latency windows), info (misc values) and the actor that
    produced the current item (set by ``ParallelIterator.gather_async``)."""

    def __init__(self):
        self.counters = collections.defaultdict(int)
        self.timers = collections.defaultdict(_Timer)
        self.info = {}
        self.current_actor = None

    def save(self) -> dict:
        """A picklable snapshot (timers are not persisted)."""
        return {"counters": dict(self.counters), "info": dict(self.info), "timers": None}

    def restore(self, values: dict) -> None:
        self.counters.clear()
        self.counters.update(values.get("counters") or {})
        self.timers.clear()
        self.info = dict(values.get("info") or {})


class SharedMetrics:
    """Indirection to a MetricsContext; setting one re-points every parent as well."""

    def __init__(self, metrics: Optional[MetricsContext] = None, parents: Optional[List["SharedMetrics"]] = None):
        self.parents = list(parents or [])
        self.metrics = metrics or MetricsContext()
        self.set(self.metrics)

    def set(self, metrics: MetricsContext) -> None:
        self.metrics = metrics
        for p in self.parents:
            p.set(metrics)

    def get(self) -> MetricsContext:
        return self.metrics


__all__ = ["MetricsContext", "SharedMetrics"]
