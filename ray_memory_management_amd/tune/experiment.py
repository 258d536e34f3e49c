"""Experiment spec + searcher / scheduler factories.
Parity: reference python/ray/tune/experiment/experiment.py (Experiment(name, run, stop, config,
resources_per_trial, num_samples, local_dir, checkpoint_freq, checkpoint_at_end, max_failures, ...),
Experiment.from_json, convert_to_experiment_list; accepted by tune.run / run_experiments),
tune/search/__init__.py:create_searcher and tune/schedulers/__init__.py:create_scheduler."""
from __future__ import annotations

from typing import Any, Dict, List, Optional


class Experiment:
    _RUN_KEYS = ("stop", "config", "resources_per_trial", "num_samples", "local_dir", "checkpoint_freq",
                 "checkpoint_at_end", "keep_checkpoints_num", "checkpoint_score_attr", "max_failures",
                 "time_budget_s", "trial_name_creator", "trial_dirname_creator", "sync_config")

    def __init__(self, name: str, run, stop=None, time_budget_s=None, config: Optional[Dict] = None,
                 resources_per_trial=None, num_samples: int = 1, local_dir: Optional[str] = None,
                 checkpoint_freq: int = 0, checkpoint_at_end: bool = False, keep_checkpoints_num=None,
                 checkpoint_score_attr=None, max_failures: int = 0, trial_name_creator=None,
                 trial_dirname_creator=None, sync_config=None, **kw):
        if run is None:
            raise ValueError("Experiment needs a trainable (`run`)")
        self.name = name
        self.run_identifier = run
        self.spec = {"stop": stop or {}, "config": dict(config or {}), "resources_per_trial": resources_per_trial,
                     "num_samples": int(num_samples), "local_dir": local_dir, "checkpoint_freq": checkpoint_freq,
                     "checkpoint_at_end": checkpoint_at_end, "keep_checkpoints_num": keep_checkpoints_num,
                     "checkpoint_score_attr": checkpoint_score_attr, "max_failures": max_failures,
                     "time_budget_s": time_budget_s, "trial_name_creator": trial_name_creator,
                     "trial_dirname_creator": trial_dirname_creator, "sync_config": sync_config}

    @classmethod
    def from_json(cls, name: str, spec: Dict[str, Any]) -> "Experiment":
        spec = dict(spec)
        if "run" not in spec:
            raise ValueError(f"No trainable specified in experiment {name!r}")
        env = spec.pop("env", None)
        if env is not None:
            spec.setdefault("config", {})["env"] = env
        return cls(name, spec.pop("run"), **spec)

    def run_kwargs(self) -> Dict[str, Any]:
        return {k: v for k, v in self.spec.items() if v is not None}


def convert_to_experiment_list(experiments) -> List[Experiment]:
    if experiments is None:
        return []
    if isinstance(experiments, Experiment):
        return [experiments]
    if isinstance(experiments, dict):
        return [Experiment.from_json(n, s) for n, s in experiments.items()]
    if isinstance(experiments, (list, tuple)):
        return [e if isinstance(e, Experiment) else Experiment.from_json(*e) for e in experiments]
    raise TypeError(f"invalid experiments {experiments!r}")


def create_searcher(search_alg: str, **kwargs):
    from ray_memory_management_amd.tune.search import BasicVariantGenerator, BayesOptSearch

    table = {"variant_generator": BasicVariantGenerator, "random": BasicVariantGenerator,
             "bayesopt": BayesOptSearch}
    if search_alg not in table:
        raise ValueError(f"search algorithm {search_alg!r} is not available here (installed: {sorted(table)})")
    return table[search_alg](**kwargs)


def create_scheduler(scheduler: str, **kwargs):
    from ray_memory_management_amd.tune import schedulers as S

    table = {"fifo": S.FIFOScheduler, "async_hyperband": S.AsyncHyperBandScheduler,
             "asynchyperband": S.AsyncHyperBandScheduler, "asha": S.AsyncHyperBandScheduler,
             "hyperband": S.HyperBandScheduler, "median_stopping_rule": S.MedianStoppingRule,
             "pbt": S.PopulationBasedTraining}
    try:
        from ray_memory_management_amd.tune.schedulers.resource_changing_scheduler import ResourceChangingScheduler

        table["resource_changing"] = ResourceChangingScheduler
    except ImportError:  # pragma: no cover
        pass
    if scheduler not in table:
        raise ValueError(f"unknown scheduler {scheduler!r} (known: {sorted(table)})")
    return table[scheduler](**kwargs)
