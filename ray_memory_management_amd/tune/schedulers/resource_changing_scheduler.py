"""ResourceChangingScheduler: change a running trial's resources as the experiment evolves.

Parity: reference python/ray/tune/schedulers/resource_changing_scheduler.py:586
(ResourceChangingScheduler wrapping a base scheduler; DistributeResources /
DistributeResourcesToTopJob allocation functions; a trial whose allocation changes is paused —
checkpointed — and restarted with the new placement-group factory; the trainable sees its current
resources through ``trial_resources`` / its trial info).
"""
from __future__ import annotations

import math
from typing import Callable, Dict, Optional

from ray_memory_management_amd.tune.schedulers import FIFOScheduler, TrialScheduler
from ray_memory_management_amd.tune.trainable import PlacementGroupFactory


class DistributeResources:
    """Spread the cluster's CPUs (and GPUs) evenly over the live trials: each gets
    max(its base request, floor(total / live trials)), in steps of `increase_by` (defaults to the
    base bundle). `add_bundles=True` grows the trial by extra bundles instead of a bigger head."""

    def __init__(self, add_bundles: bool = False, increase_by: Optional[Dict[str, float]] = None,
                 increase_by_times: int = -1, reserve_resources: Optional[Dict[str, float]] = None,
                 metric: Optional[str] = None, mode: Optional[str] = None):
        self.add_bundles = add_bundles
        self.increase_by = dict(increase_by or {})
        self.increase_by_times = increase_by_times
        self.reserve = dict(reserve_resources or {})
        self.metric, self.mode = metric, mode
        self._base: Dict[str, PlacementGroupFactory] = {}

    def _live(self, runner):
        return [t for t in runner.get_trials() if t.status in ("RUNNING", "PENDING", "PAUSED")]

    def _weights(self, runner, trials):
        return {t.trial_id: 1.0 for t in trials}

    def __call__(self, runner, trial, result: Dict, scheduler) -> Optional[PlacementGroupFactory]:
        import ray_memory_management_amd as ray

        base = self._base.setdefault(trial.trial_id, trial.resources)
        total = ray.cluster_resources()
        live = self._live(runner)
        if not live:
            return None
        weights = self._weights(runner, live)
        wsum = sum(weights.values()) or 1.0
        share = weights.get(trial.trial_id, 1.0) / wsum
        step = self.increase_by or {k: v for k, v in base.head_bundle.items() if k in ("CPU", "GPU") and v}
        if not step:
            return None
        # how many `step` units this trial's share of the (reserved-adjusted) cluster affords
        units = None
        for k, v in step.items():
            avail = max(0.0, float(total.get(k, 0)) - float(self.reserve.get(k, 0)))
            u = math.floor(avail * share / v + 1e-9)
            units = u if units is None else min(units, u)
        base_units = min(max(1, math.floor(base.head_bundle.get(k, 0) / v + 1e-9)) for k, v in step.items())
        units = max(base_units, units or 0)
        if self.increase_by_times >= 0:
            units = min(units, base_units + self.increase_by_times)
        if self.add_bundles:
            bundles = [dict(base.head_bundle)] + [dict(step) for _ in range(units - base_units)]
        else:
            head = dict(base.head_bundle)
            for k, v in step.items():
                head[k] = max(head.get(k, 0), v * units)
            bundles = [head] + [dict(b) for b in base.bundles[1:]]
        new = PlacementGroupFactory(bundles, base.strategy)
        return None if new == trial.resources else new


class DistributeResourcesToTopJob(DistributeResources):
    """All spare resources go to the best trial by `metric` (reference: same name)."""

    def _weights(self, runner, trials):
        metric = self.metric
        if not metric:
            return super()._weights(runner, trials)
        sign = 1.0 if (self.mode or "max") == "max" else -1.0
        scored = [(sign * t.last_result.get(metric, float("-inf")), t.trial_id) for t in trials if t.last_result]
        if not scored:
            return super()._weights(runner, trials)
        best = max(scored)[1]
        return {t.trial_id: (len(trials) if t.trial_id == best else 1e-9) for t in trials}


class ResourceChangingScheduler(TrialScheduler):
    """Wrap `base_scheduler`; after every result ask `resources_allocation_function(runner, trial,
    result, scheduler)` for a new PlacementGroupFactory. A changed allocation pauses the trial
    (checkpoint) and it restarts from that checkpoint with the new resources when they fit."""

    def __init__(self, base_scheduler: Optional[TrialScheduler] = None,
                 resources_allocation_function: Optional[Callable] = None, metric: Optional[str] = None,
                 mode: Optional[str] = None):
        self.base = base_scheduler or FIFOScheduler()
        self.fn = resources_allocation_function if resources_allocation_function is not None else DistributeResources()
        self._metric, self._mode = metric, mode
        self._reallocated: Dict[str, PlacementGroupFactory] = {}
        self.num_reallocations = 0

    def set_search_properties(self, metric, mode, **spec):
        ok = self.base.set_search_properties(metric, mode, **spec)
        if metric:
            self._metric = metric
        if mode:
            self._mode = mode
        if isinstance(self.fn, DistributeResources):
            self.fn.metric = self.fn.metric or self._metric
            self.fn.mode = self.fn.mode or self._mode
        return ok

    def on_trial_add(self, runner, trial):
        self.base.on_trial_add(runner, trial)

    def on_trial_error(self, runner, trial):
        self.base.on_trial_error(runner, trial)

    def on_trial_complete(self, runner, trial, result):
        self.base.on_trial_complete(runner, trial, result)

    def on_trial_remove(self, runner, trial):
        self.base.on_trial_remove(runner, trial)

    def on_trial_result(self, runner, trial, result: Dict) -> str:
        decision = self.base.on_trial_result(runner, trial, result)
        if decision != TrialScheduler.CONTINUE or trial.status != "RUNNING":
            return decision
        new = self.fn(runner, trial, result, self)
        if new is None or new == trial.resources:
            return decision
        trial.resources = trial.placement_group_factory = new
        self._reallocated[trial.trial_id] = new
        self.num_reallocations += 1
        return TrialScheduler.PAUSE  # the runner checkpoints it; choose_trial_to_run restarts it

    def choose_trial_to_run(self, runner):
        # restart re-allocated trials first (they already hold progress)
        for t in runner.get_trials():
            if t.status == "PAUSED" and t.trial_id in self._reallocated and runner.has_resources_for_trial(t):
                self._reallocated.pop(t.trial_id)
                return t
        return self.base.choose_trial_to_run(runner)

    def debug_string(self) -> str:
        return f"ResourceChangingScheduler({self.base.debug_string()})"
