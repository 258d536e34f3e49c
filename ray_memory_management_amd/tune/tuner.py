"""Tuner + tune.run. Parity: reference python/ray/tune/tuner.py (Tuner(trainable, param_space,
tune_config, run_config).fit() -> ResultGrid, Tuner.restore) and python/ray/tune/tune.py
(tune.run(...) -> ExperimentAnalysis)."""
from __future__ import annotations

import os
import pickle
import time
from typing import Any, Callable, Dict, Optional, Union

import ray_memory_management_amd as ray
from ray_memory_management_amd.air.config import RunConfig
from ray_memory_management_amd.tune.execution import TrialRunner
from ray_memory_management_amd.tune.result_grid import ExperimentAnalysis, ResultGrid
from ray_memory_management_amd.tune.search.variant_generator import BasicVariantGenerator, Searcher
from ray_memory_management_amd.tune.trainable import PlacementGroupFactory, wrap_function
from ray_memory_management_amd.tune.tune_config import TuneConfig


def _resolve_trainable(trainable):
    """Returns (Trainable class, default resources, param-space prefix)."""
    from ray_memory_management_amd.train.base_trainer import BaseTrainer

    if isinstance(trainable, BaseTrainer):
        fn = trainable.as_trainable()
        sc = trainable.scaling_config
        # the trial actor only coordinates: the trainer's worker group reserves its own resources
        res = PlacementGroupFactory([{"CPU": 0}] + [sc._resources_per_worker_not_none
                                                     for _ in range(sc.num_workers or 1)])
        cls = wrap_function(fn)
        cls._resources = res
        return cls
    if isinstance(trainable, str):
        from ray_memory_management_amd.tune.registry import get_trainable_cls

        trainable = get_trainable_cls(trainable)
    return wrap_function(trainable)


def _search(search_alg, metric, mode, space, num_samples) -> Searcher:
    if search_alg is None:
        search_alg = BasicVariantGenerator()
    if isinstance(search_alg, BasicVariantGenerator):
        search_alg.set_search_properties(metric, mode, space, num_samples=num_samples)
    else:
        inner = getattr(search_alg, "searcher", None)
        if isinstance(inner, BasicVariantGenerator):
            inner.set_search_properties(metric, mode, space, num_samples=num_samples)
        else:
            try:  # model-based searchers stop after num_samples suggestions themselves
                search_alg.set_search_properties(metric, mode, space, num_samples=num_samples)
            except TypeError:
                search_alg.set_search_properties(metric, mode, space)
    return search_alg


class _ListSearcher(Searcher):
    def __init__(self, configs):
        super().__init__()
        self._configs = list(configs)

    def suggest(self, trial_id):
        return self._configs.pop(0) if self._configs else Searcher.FINISHED


class Tuner:
    def __init__(self, trainable=None, *, param_space: Optional[Dict[str, Any]] = None,
                 tune_config: Optional[TuneConfig] = None, run_config: Optional[RunConfig] = None,
                 _tuner_kwargs: Optional[Dict] = None):
        self.trainable = trainable
        self.param_space = param_space or {}
        self.tune_config = tune_config or TuneConfig()
        self.run_config = run_config or RunConfig()
        self._restored_trials = None

    def fit(self) -> ResultGrid:
        if not ray.is_initialized():
            ray.init()
        tc, rc = self.tune_config, self.run_config
        cls = _resolve_trainable(self.trainable)
        name = rc.name or f"{cls.__name__}_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
        exp_dir = os.path.join(rc.storage_path or rc.local_dir or os.path.expanduser("~/rmm_results"), name)
        sched = tc.scheduler
        if sched is not None:
            sched.set_search_properties(tc.metric, tc.mode)
        fc = rc.failure_config
        cc = rc.checkpoint_config
        search = _search(tc.search_alg, tc.metric, tc.mode, self.param_space, tc.num_samples)
        if self._restored_trials is not None:
            search = _ListSearcher([s["config"] for s in self._restored_trials
                                    if s["status"] not in ("TERMINATED",)])
        runner = TrialRunner(cls, search, sched, exp_dir, stopper=rc.stop, metric=tc.metric, mode=tc.mode,
                             max_concurrent_trials=tc.max_concurrent_trials, time_budget_s=tc.time_budget_s,
                             checkpoint_freq=(cc.checkpoint_frequency if cc else 0),
                             checkpoint_at_end=bool(cc and cc.checkpoint_at_end),
                             max_failures=(fc.max_failures if fc else 0), fail_fast=bool(fc and fc.fail_fast),
                             callbacks=rc.callbacks, num_to_keep=(cc.num_to_keep if cc else None),
                             verbose=rc.verbose, progress_reporter=rc.progress_reporter,
                             sync_config=rc.sync_config)
        if self._restored_trials is not None:  # finished trials keep their recorded results
            from ray_memory_management_amd.tune.execution import Trial

            for s in self._restored_trials:
                if s["status"] == "TERMINATED":
                    t = Trial(cls.__name__, s["config"], s["trial_id"], exp_dir, runner.pgf)
                    t.status = "TERMINATED"
                    t.update_last_result(s["last_result"])
                    runner._trials.append(t)
        trials = runner.run()
        self._save_state(exp_dir, trials)
        return ResultGrid(trials, tc.metric, tc.mode)

    @staticmethod
    def _save_state(exp_dir, trials):
        state = [{"trial_id": t.trial_id, "config": t.config, "status": t.status, "last_result": t.last_result,
                  "logdir": t.logdir} for t in trials]
        os.makedirs(exp_dir, exist_ok=True)
        with open(os.path.join(exp_dir, "experiment_state.pkl"), "wb") as f:
            pickle.dump(state, f)

    @classmethod
    def restore(cls, path: str, trainable=None, **kw) -> "Tuner":
        """Re-run unfinished trials of a previous experiment (finished ones keep their results)."""
        with open(os.path.join(path, "experiment_state.pkl"), "rb") as f:
            state = pickle.load(f)
        t = cls(trainable, param_space={}, run_config=RunConfig(name=os.path.basename(path),
                                                                 local_dir=os.path.dirname(path)))
        t._restored_trials = state
        return t

    def get_results(self) -> ResultGrid:
        raise NotImplementedError("call fit()")


def run(run_or_experiment, *, name: Optional[str] = None, metric: Optional[str] = None, mode: Optional[str] = None,
        stop=None, time_budget_s=None, config: Optional[Dict] = None, resources_per_trial=None,
        num_samples: int = 1, local_dir: Optional[str] = None, search_alg=None, scheduler=None,
        keep_checkpoints_num: Optional[int] = None, checkpoint_score_attr: Optional[str] = None,
        checkpoint_freq: int = 0, checkpoint_at_end: bool = False, verbose: int = 0, progress_reporter=None,
        log_to_file: bool = False, trial_name_creator=None, trial_dirname_creator=None, sync_config=None,
        export_formats=None, max_failures: int = 0, fail_fast: bool = False, restore: Optional[str] = None,
        server_port=None, resume=False, reuse_actors=None, raise_on_failed_trial: bool = True, callbacks=None,
        max_concurrent_trials: Optional[int] = None, **kwargs) -> ExperimentAnalysis:
    """Run hyperparameter search; returns an ExperimentAnalysis."""
    from ray_memory_management_amd.tune.experiment import Experiment

    if isinstance(run_or_experiment, Experiment):  # an Experiment carries its own run arguments
        exp = run_or_experiment
        merged = {**exp.run_kwargs(), **{k: v for k, v in dict(stop=stop, config=config, local_dir=local_dir).items()
                                          if v}}
        return run(exp.run_identifier, name=name or exp.name, metric=metric, mode=mode, search_alg=search_alg,
                   scheduler=scheduler, verbose=verbose, callbacks=callbacks, **merged)
    from ray_memory_management_amd.tune.error import TuneError

    if not ray.is_initialized():
        ray.init()
    if mode and mode not in ("min", "max"):
        raise ValueError("`mode` must be one of ['min', 'max']")
    cls = _resolve_trainable(run_or_experiment)
    exp_dir = os.path.join(local_dir or os.path.expanduser("~/rmm_results"),
                           name or f"{cls.__name__}_{time.strftime('%Y-%m-%d_%H-%M-%S')}")
    if scheduler is not None:
        scheduler.set_search_properties(metric, mode)
    runner = TrialRunner(cls, _search(search_alg, metric, mode, config or {}, num_samples), scheduler, exp_dir,
                         stopper=stop, metric=metric, mode=mode, max_concurrent_trials=max_concurrent_trials,
                         time_budget_s=time_budget_s, checkpoint_freq=checkpoint_freq,
                         checkpoint_at_end=checkpoint_at_end, max_failures=max_failures, fail_fast=fail_fast,
                         callbacks=callbacks, resources=resources_per_trial, num_to_keep=keep_checkpoints_num,
                         verbose=verbose, progress_reporter=progress_reporter, sync_config=sync_config,
                         server_port=server_port)
    if restore:
        ck = None
        from ray_memory_management_amd.air.checkpoint import Checkpoint

        ck = Checkpoint.from_directory(restore)
        orig = runner._start_trial

        def start_with_restore(t, checkpoint=None):
            return orig(t, checkpoint or ck)

        runner._start_trial = start_with_restore
    trials = runner.run()
    Tuner._save_state(exp_dir, trials)
    errored = [t for t in trials if t.status == "ERROR"]
    if errored and raise_on_failed_trial and not fail_fast:
        raise TuneError(f"Trials did not complete: {errored}")
    if errored and fail_fast and raise_on_failed_trial:
        raise TuneError(f"Trials did not complete: {errored}")
    return ExperimentAnalysis(trials, metric, mode, exp_dir)


def run_experiments(experiments, **kw):
    """Run Experiment objects or {name: spec} dicts in sequence; returns all their trials."""
    from ray_memory_management_amd.tune.experiment import convert_to_experiment_list

    out = []
    for exp in convert_to_experiment_list(experiments):
        out.extend(run(exp.run_identifier, name=exp.name, **exp.run_kwargs(), **kw).trials)
    return out
