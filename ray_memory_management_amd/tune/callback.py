"""Tune callbacks. Parity: reference python/ray/tune/callback.py (Callback hooks invoked by the
trial runner) and tune/logger (JsonLoggerCallback / CSVLoggerCallback)."""
from __future__ import annotations

import csv
import json
import os


class Callback:
    def setup(self, **info):
        pass

    def on_trial_add(self, iteration, trials, trial, **info):
        pass

    def on_trial_start(self, iteration, trials, trial, **info):
        pass

    def on_trial_result(self, iteration, trials, trial, result, **info):
        pass

    def on_trial_complete(self, iteration, trials, trial, **info):
        pass

    def on_trial_error(self, iteration, trials, trial, **info):
        pass

    def on_experiment_end(self, trials, **info):
        pass


class CSVLoggerCallback(Callback):
    def __init__(self):
        self._files = {}

    def on_trial_result(self, iteration, trials, trial, result, **info):
        flat = {k: v for k, v in result.items() if isinstance(v, (int, float, str, bool))}
        path = os.path.join(trial.logdir, "progress.csv")
        new = trial.trial_id not in self._files
        with open(path, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=sorted(flat), extrasaction="ignore")
            if new:
                w.writeheader()
                self._files[trial.trial_id] = sorted(flat)
            w.writerow(flat)


class JsonLoggerCallback(Callback):
    def on_trial_result(self, iteration, trials, trial, result, **info):
        pass  # result.json is always written by the runner
