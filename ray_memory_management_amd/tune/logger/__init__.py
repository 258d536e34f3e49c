"""Tune result loggers. Parity: reference python/ray/tune/logger/{logger,csv,json,tensorboardx,
noop,unified}.py: per-trial Logger objects (on_result / flush / close) and LoggerCallback
(per-trial log_trial_start / log_trial_result / log_trial_end), the legacy bridge that drives
Logger classes from callback hooks, and pretty_print. TensorBoardX is not installed here; its
logger raises a clear ImportError."""
from __future__ import annotations

import csv
import json
import os
from typing import Dict, List, Optional, Type

from ray_memory_management_amd.tune.callback import Callback, CSVLoggerCallback, JsonLoggerCallback  # noqa: F401


def _flat(result: Dict, prefix: str = "") -> Dict:
    out = {}
    for k, v in result.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(_flat(v, key + "/"))
        elif isinstance(v, (int, float, str, bool)) or v is None:
            out[key] = v
    return out


def pretty_print(result: Dict) -> str:
    """YAML-like dump of a result dict (reference tune/logger/logger.py pretty_print)."""
    lines: List[str] = []

    def emit(d, ind):
        for k, v in d.items():
            if k in ("config", "hist_stats") or v is None:
                continue
            if isinstance(v, dict):
                lines.append(" " * ind + f"{k}:")
                emit(v, ind + 2)
            else:
                lines.append(" " * ind + f"{k}: {v}")

    emit(result, 0)
    return "\n".join(lines) + "\n"


class Logger:
    def __init__(self, config: Dict, logdir: str, trial=None):
        self.config, self.logdir, self.trial = config, logdir, trial
        os.makedirs(logdir, exist_ok=True)
        self._init()

    def _init(self):
        pass

    def on_result(self, result: Dict):
        raise NotImplementedError

    def update_config(self, config: Dict):
        self.config = config

    def flush(self):
        pass

    def close(self):
        self.flush()


class NoopLogger(Logger):
    def on_result(self, result):
        pass


class JsonLogger(Logger):
    def _init(self):
        self._f = open(os.path.join(self.logdir, "result.json"), "a")
        with open(os.path.join(self.logdir, "params.json"), "w") as f:
            json.dump({k: v for k, v in (self.config or {}).items() if _jsonable(v)}, f)

    def on_result(self, result):
        self._f.write(json.dumps({k: v for k, v in result.items() if _jsonable(v)}) + "\n")

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


class CSVLogger(Logger):
    def _init(self):
        path = os.path.join(self.logdir, "progress.csv")
        self._continuing = os.path.exists(path) and os.path.getsize(path) > 0
        self._f = open(path, "a", newline="")
        self._w = None

    def on_result(self, result):
        flat = _flat(result)
        if self._w is None:
            self._w = csv.DictWriter(self._f, fieldnames=sorted(flat), extrasaction="ignore")
            if not self._continuing:
                self._w.writeheader()
        self._w.writerow(flat)

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


class TBXLogger(Logger):
    def _init(self):
        raise ImportError("TBXLogger needs tensorboardX, which is not installed; use CSVLogger / JsonLogger")

    def on_result(self, result):  # pragma: no cover
        pass


DEFAULT_LOGGERS = (JsonLogger, CSVLogger)


class UnifiedLogger(Logger):
    """Fan-out to several Logger classes (default: JSON + CSV)."""

    def __init__(self, config, logdir, trial=None, loggers: Optional[List[Type[Logger]]] = None):
        self._classes = list(loggers or DEFAULT_LOGGERS)
        super().__init__(config, logdir, trial)

    def _init(self):
        self._loggers = [cls(self.config, self.logdir, self.trial) for cls in self._classes]

    def on_result(self, result):
        for lg in self._loggers:
            lg.on_result(result)

    def flush(self):
        for lg in self._loggers:
            lg.flush()

    def close(self):
        for lg in self._loggers:
            lg.close()


class LoggerCallback(Callback):
    """Callback that routes runner hooks to per-trial log_trial_* methods."""

    def log_trial_start(self, trial):
        pass

    def log_trial_result(self, iteration: int, trial, result: Dict):
        pass

    def log_trial_end(self, trial, failed: bool = False):
        pass

    def on_trial_start(self, iteration, trials, trial, **info):
        self.log_trial_start(trial)

    def on_trial_result(self, iteration, trials, trial, result, **info):
        self.log_trial_result(iteration, trial, result)

    def on_trial_complete(self, iteration, trials, trial, **info):
        self.log_trial_end(trial, failed=False)

    def on_trial_error(self, iteration, trials, trial, **info):
        self.log_trial_end(trial, failed=True)


class LegacyLoggerCallback(LoggerCallback):
    """Drive Logger classes (one instance per trial and class) from the callback hooks."""

    def __init__(self, logger_classes):
        self.logger_classes = list(logger_classes)
        self._loggers: Dict[str, List[Logger]] = {}

    def _for(self, trial) -> List[Logger]:
        if trial.trial_id not in self._loggers:
            self._loggers[trial.trial_id] = [cls(trial.config, os.path.join(trial.logdir, "legacy"), trial)
                                             for cls in self.logger_classes]
        return self._loggers[trial.trial_id]

    def log_trial_start(self, trial):
        for lg in self._for(trial):
            lg.update_config(trial.config)

    def log_trial_result(self, iteration, trial, result):
        for lg in self._for(trial):
            lg.on_result(result)
            lg.flush()

    def log_trial_end(self, trial, failed=False):
        for lg in self._loggers.pop(trial.trial_id, []):
            lg.close()


class TBXLoggerCallback(LoggerCallback):
    def __init__(self):
        raise ImportError("TBXLoggerCallback needs tensorboardX, which is not installed")


def _jsonable(v) -> bool:
    try:
        json.dumps(v)
        return True
    except (TypeError, ValueError):
        return False


__all__ = ["Logger", "LoggerCallback", "LegacyLoggerCallback", "pretty_print", "CSVLogger", "CSVLoggerCallback",
           "JsonLogger", "JsonLoggerCallback", "NoopLogger", "TBXLogger", "TBXLoggerCallback", "UnifiedLogger"]
