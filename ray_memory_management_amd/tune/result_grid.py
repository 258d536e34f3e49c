"""ResultGrid + ExperimentAnalysis. Parity: reference python/ray/tune/result_grid.py and
python/ray/tune/analysis/experiment_analysis.py (best trial/config/result/checkpoint by
metric/mode/scope, dataframes)."""
from __future__ import annotations

import os
from typing import Dict, List, Optional

from ray_memory_management_amd.air.checkpoint import Checkpoint
from ray_memory_management_amd.air.result import Result


def _score(trial, metric, mode, scope):
    if scope == "last":
        v = trial.last_result.get(metric)
    else:
        a = trial.metric_analysis.get(metric)
        if a is None:
            return None
        if scope == "all":
            v = a["max"] if mode == "max" else a["min"]
        elif scope in ("avg", "last-5-avg", "last-10-avg"):
            if scope == "avg":
                v = a["avg"]
            else:
                k = 5 if scope == "last-5-avg" else 10
                vals = [r[metric] for r in trial.results if metric in r][-k:]
                v = sum(vals) / len(vals) if vals else None
        else:
            v = a.get(scope)
    return v


def _best(trials, metric, mode, scope="last", filter_nan_and_inf=True):
    import math

    if mode not in ("max", "min"):
        raise ValueError("`mode` must be 'max' or 'min'")
    best, best_v = None, None
    for t in trials:
        v = _score(t, metric, mode, scope)
        if v is None or (filter_nan_and_inf and isinstance(v, float) and (math.isnan(v) or math.isinf(v))):
            continue
        if best is None or (v > best_v if mode == "max" else v < best_v):
            best, best_v = t, v
    return best


def _trial_checkpoint(t) -> Optional[Checkpoint]:
    if t.saved_checkpoints:
        return Checkpoint.from_directory(t.saved_checkpoints[-1][0])
    if t.checkpoint is not None:
        return t.checkpoint
    return None


def _to_result(t) -> Result:
    return Result(metrics=dict(t.last_result), checkpoint=_trial_checkpoint(t),
                  error=t.error if t.status == "ERROR" else None, log_dir=t.logdir,
                  metrics_history=list(t.results),
                  best_checkpoints=[(Checkpoint.from_directory(p), m) for p, m in t.saved_checkpoints])


class ResultGrid:
    def __init__(self, trials, default_metric: Optional[str] = None, default_mode: Optional[str] = None):
        self._trials = list(trials)
        self._metric, self._mode = default_metric, default_mode
        self._results = [_to_result(t) for t in self._trials]

    def get_best_result(self, metric: Optional[str] = None, mode: Optional[str] = None, scope: str = "last",
                        filter_nan_and_inf: bool = True) -> Result:
        metric = metric or self._metric
        mode = mode or self._mode
        if not metric or not mode:
            raise ValueError("No metric/mode given: pass them here or in TuneConfig(metric=..., mode=...)")
        t = _best(self._trials, metric, mode, scope, filter_nan_and_inf)
        if t is None:
            raise RuntimeError(f"No best trial found for metric {metric!r}")
        return self._results[self._trials.index(t)]

    def get_dataframe(self, filter_metric: Optional[str] = None, filter_mode: Optional[str] = None):
        import pandas as pd

        rows = []
        for t in self._trials:
            r = dict(t.last_result)
            if filter_metric and filter_mode:
                best = None
                for x in t.results:
                    if filter_metric in x and (best is None or (x[filter_metric] > best[filter_metric]
                                                                if filter_mode == "max" else
                                                                x[filter_metric] < best[filter_metric])):
                        best = x
                r = dict(best or r)
            cfg = r.pop("config", {})
            for k, v in cfg.items():
                r[f"config/{k}"] = v
            r["logdir"] = t.logdir
            rows.append(r)
        return pd.DataFrame(rows)

    @property
    def errors(self):
        return [r.error for r in self._results if r.error is not None]

    @property
    def num_errors(self) -> int:
        return len(self.errors)

    @property
    def num_terminated(self) -> int:
        return sum(1 for t in self._trials if t.status == "TERMINATED")

    def __len__(self):
        return len(self._results)

    def __getitem__(self, i) -> Result:
        return self._results[i]

    def __iter__(self):
        return iter(self._results)

    def __repr__(self):
        return f"ResultGrid<{len(self)} results>"


class _LoadedTrial:
    """A finished trial read back from its directory (params.json + result.json)."""

    def __init__(self, logdir: str):
        import json

        self.logdir = logdir
        self.trial_id = os.path.basename(logdir.rstrip("/")).rsplit("_", 1)[-1]
        self.experiment_tag = os.path.basename(logdir.rstrip("/"))
        with open(os.path.join(logdir, "params.json")) as f:
            self.config = json.load(f)
        self.results = []
        rp = os.path.join(logdir, "result.json")
        if os.path.exists(rp):
            with open(rp) as f:
                self.results = [json.loads(line) for line in f if line.strip()]
        self.last_result = dict(self.results[-1]) if self.results else {}
        self.metric_analysis = {}
        self.saved_checkpoints = sorted(
            [(os.path.join(logdir, d), {}) for d in os.listdir(logdir)
             if d.startswith("checkpoint_") and os.path.isdir(os.path.join(logdir, d))])
        self.checkpoint = None
        self.status = self.last_result.get("trial_status", "TERMINATED")
        self.error = None


def load_trials(experiment_dir: str) -> List[_LoadedTrial]:
    """Every trial directory (one with a params.json) under an experiment directory."""
    out = []
    for d in sorted(os.listdir(experiment_dir)):
        full = os.path.join(experiment_dir, d)
        if os.path.isdir(full) and os.path.exists(os.path.join(full, "params.json")):
            out.append(_LoadedTrial(full))
    return out


class ExperimentAnalysis:
    """Analysis of a Tune experiment: from the trials of a run, or (reference
    tune/analysis/experiment_analysis.py) from an experiment directory on disk."""

    def __init__(self, trials, default_metric=None, default_mode=None, experiment_dir=None):
        if isinstance(trials, (str, os.PathLike)):
            experiment_dir = os.fspath(trials)
            if os.path.isfile(experiment_dir):  # an experiment_state file: its directory
                experiment_dir = os.path.dirname(experiment_dir)
            trials = load_trials(experiment_dir)
        self.trials = list(trials)
        self.default_metric, self.default_mode = default_metric, default_mode
        self._experiment_dir = experiment_dir

    def _mm(self, metric, mode):
        metric = metric or self.default_metric
        mode = mode or self.default_mode
        if not metric or not mode:
            raise ValueError("To fetch the best trial, pass `metric` and `mode` here or to tune.run().")
        return metric, mode

    def get_best_trial(self, metric=None, mode=None, scope="last", filter_nan_and_inf=True):
        metric, mode = self._mm(metric, mode)
        return _best(self.trials, metric, mode, scope, filter_nan_and_inf)

    def get_best_config(self, metric=None, mode=None, scope="last"):
        t = self.get_best_trial(metric, mode, scope)
        return t.config if t else None

    def get_best_logdir(self, metric=None, mode=None, scope="last"):
        t = self.get_best_trial(metric, mode, scope)
        return t.logdir if t else None

    def get_best_checkpoint(self, trial, metric=None, mode=None):
        metric, mode = self._mm(metric, mode)
        if not trial.saved_checkpoints:
            return trial.checkpoint
        path, _ = max(trial.saved_checkpoints, key=lambda pm: (pm[1].get(metric, float("-inf")) if mode == "max"
                                                               else -pm[1].get(metric, float("inf"))))
        return Checkpoint.from_directory(path)

    def get_all_configs(self, prefix=False) -> Dict[str, Dict]:
        return {t.logdir: t.config for t in self.trials}

    @property
    def best_trial(self):
        return self.get_best_trial()

    @property
    def best_config(self):
        return self.get_best_config()

    @property
    def best_logdir(self):
        return self.get_best_logdir()

    @property
    def best_checkpoint(self):
        return self.get_best_checkpoint(self.best_trial)

    @property
    def best_result(self):
        return self.best_trial.last_result

    @property
    def results(self):
        return {t.trial_id: t.last_result for t in self.trials}

    @property
    def results_df(self):
        import pandas as pd

        return pd.DataFrame([dict(t.last_result, trial_id=t.trial_id) for t in self.trials]).set_index("trial_id")

    def dataframe(self, metric=None, mode=None):
        return ResultGrid(self.trials, metric, mode).get_dataframe(metric, mode)

    @property
    def trial_dataframes(self):
        import pandas as pd

        return {t.logdir: pd.DataFrame(t.results) for t in self.trials}

    @property
    def experiment_path(self):
        return self._experiment_dir
