"""Stoppers. Parity: reference python/ray/tune/stopper.py (Stopper, CombinedStopper,
FunctionStopper, MaximumIterationStopper, ExperimentPlateauStopper, TrialPlateauStopper,
TimeoutStopper)."""
from __future__ import annotations

import collections
import time
from typing import Callable, Dict, Optional

import numpy as np


class Stopper:
    def __call__(self, trial_id: str, result: Dict) -> bool:
        raise NotImplementedError

    def stop_all(self) -> bool:
        raise NotImplementedError


class NoopStopper(Stopper):
    def __call__(self, trial_id, result):
        return False

    def stop_all(self):
        return False


class CombinedStopper(Stopper):
    def __init__(self, *stoppers: Stopper):
        self._stoppers = stoppers

    def __call__(self, trial_id, result):
        return any(s(trial_id, result) for s in self._stoppers)

    def stop_all(self):
        return any(s.stop_all() for s in self._stoppers)


class FunctionStopper(Stopper):
    def __init__(self, function: Callable[[str, Dict], bool]):
        self._fn = function

    def __call__(self, trial_id, result):
        return bool(self._fn(trial_id, result))

    def stop_all(self):
        return False

    @classmethod
    def is_valid_function(cls, fn) -> bool:
        return callable(fn) and not isinstance(fn, Stopper)


class DictStopper(Stopper):
    """{"metric": threshold}: stop when result[metric] >= threshold (reference semantics)."""

    def __init__(self, spec: Dict):
        self._spec = spec

    def __call__(self, trial_id, result):
        for k, v in self._spec.items():
            if k in result and result[k] >= v:
                return True
        return False

    def stop_all(self):
        return False


class MaximumIterationStopper(Stopper):
    def __init__(self, max_iter: int):
        self._max_iter = max_iter
        self._iter = collections.defaultdict(int)

    def __call__(self, trial_id, result):
        self._iter[trial_id] += 1
        return self._iter[trial_id] >= self._max_iter

    def stop_all(self):
        return False


class ExperimentPlateauStopper(Stopper):
    def __init__(self, metric: str, std: float = 0.001, top: int = 10, mode: str = "min", patience: int = 0):
        self._metric, self._std, self._top, self._mode, self._patience = metric, std, top, mode, patience
        self._top_values = []
        self._iter = 0
        self._stop = False

    def __call__(self, trial_id, result):
        self._top_values.append(result[self._metric])
        self._top_values = sorted(self._top_values, reverse=self._mode == "max")[: self._top]
        if len(self._top_values) == self._top and np.std(self._top_values) <= self._std:
            self._iter += 1
        else:
            self._iter = 0
        if self._iter > self._patience:
            self._stop = True
        return self._stop

    def stop_all(self):
        return self._stop


class TrialPlateauStopper(Stopper):
    def __init__(self, metric: str, std: float = 0.01, num_results: int = 4, grace_period: int = 4,
                 metric_threshold: Optional[float] = None, mode: Optional[str] = None):
        self._metric, self._std, self._n, self._grace = metric, std, num_results, grace_period
        self._thresh, self._mode = metric_threshold, mode
        self._results = collections.defaultdict(lambda: collections.deque(maxlen=num_results))
        self._count = collections.defaultdict(int)

    def __call__(self, trial_id, result):
        v = result.get(self._metric)
        if v is None:
            return False
        self._count[trial_id] += 1
        self._results[trial_id].append(v)
        if self._count[trial_id] < self._grace or len(self._results[trial_id]) < self._n:
            return False
        if self._thresh is not None:
            if self._mode == "min" and v > self._thresh:
                return False
            if self._mode == "max" and v < self._thresh:
                return False
        return float(np.std(self._results[trial_id])) < self._std

    def stop_all(self):
        return False


class TimeoutStopper(Stopper):
    def __init__(self, timeout):
        import datetime

        if isinstance(timeout, datetime.timedelta):
            timeout = timeout.total_seconds()
        self._timeout = float(timeout)
        self._start = time.time()

    def __call__(self, trial_id, result):
        return False

    def stop_all(self):
        return time.time() - self._start >= self._timeout
