"""Experiment progress reporting. Parity: reference python/ray/tune/progress_reporter.py
(ProgressReporter.should_report/report, TuneReporterBase with metric/parameter columns,
max_progress_rows, max_report_frequency, sort_by_metric, CLIReporter printing a trial table with
a status summary; JupyterNotebookReporter renders the same table)."""
from __future__ import annotations

import sys
import time
from typing import Dict, List, Optional, Union

from tabulate import tabulate


class ProgressReporter:
    def should_report(self, trials: List, done: bool = False) -> bool:
        return True

    def report(self, trials: List, done: bool, *sys_info: Dict):
        raise NotImplementedError

    def setup(self, start_time: Optional[float] = None, total_samples: Optional[int] = None, metric=None, mode=None,
              **kw):
        pass


def _get(d: Dict, path: str):
    cur = d
    for p in path.split("/"):
        if not isinstance(cur, dict) or p not in cur:
            return None
        cur = cur[p]
    return cur


class TuneReporterBase(ProgressReporter):
    DEFAULT_COLUMNS = {"episode_reward_mean": "reward", "mean_accuracy": "acc", "mean_loss": "loss", "loss": "loss",
                       "training_iteration": "iter", "time_total_s": "total time (s)", "timesteps_total": "ts"}

    def __init__(self, *, metric_columns: Union[None, List[str], Dict[str, str]] = None,
                 parameter_columns: Union[None, List[str], Dict[str, str]] = None, total_samples: Optional[int] = None,
                 max_progress_rows: int = 20, max_error_rows: int = 20, max_column_length: int = 20,
                 max_report_frequency: float = 5, infer_limit: int = 3, print_intermediate_tables: Optional[bool] = None,
                 metric: Optional[str] = None, mode: Optional[str] = None, sort_by_metric: bool = False):
        self._metric_columns = metric_columns
        self._parameter_columns = parameter_columns
        self.max_progress_rows = max_progress_rows
        self.max_error_rows = max_error_rows
        self.max_column_length = max_column_length
        self.max_report_frequency = max_report_frequency
        self.infer_limit = infer_limit
        self.print_intermediate_tables = print_intermediate_tables
        self.metric, self.mode = metric, mode
        self.sort_by_metric = sort_by_metric
        self._last_report = 0.0
        self._start = time.time()

    def setup(self, start_time=None, total_samples=None, metric=None, mode=None, **kw):
        self._start = start_time or self._start
        self.metric = self.metric or metric
        self.mode = self.mode or mode

    def add_metric_column(self, metric: str, representation: Optional[str] = None):
        if isinstance(self._metric_columns, dict):
            self._metric_columns[metric] = representation or metric
        else:
            self._metric_columns = list(self._metric_columns or []) + [metric]

    def add_parameter_column(self, parameter: str, representation: Optional[str] = None):
        if isinstance(self._parameter_columns, dict):
            self._parameter_columns[parameter] = representation or parameter
        else:
            self._parameter_columns = list(self._parameter_columns or []) + [parameter]

    def should_report(self, trials, done=False):
        now = time.time()
        if done or now - self._last_report >= self.max_report_frequency:
            self._last_report = now
            return True
        return False

    def _columns(self, trials):
        mc = self._metric_columns
        if mc is None:  # infer: the default columns any trial reports
            mc = {k: v for k, v in self.DEFAULT_COLUMNS.items()
                  if any(_get(t.last_result or {}, k) is not None for t in trials)}
        elif isinstance(mc, list):
            mc = {k: k for k in mc}
        pc = self._parameter_columns
        if pc is None:
            keys = []
            for t in trials:
                for k, v in (t.config or {}).items():
                    if k not in keys and isinstance(v, (int, float, str, bool)):
                        keys.append(k)
            pc = {k: k for k in keys[:self.infer_limit]}
        elif isinstance(pc, list):
            pc = {k: k for k in pc}
        return mc, pc

    def trial_table(self, trials) -> str:
        mc, pc = self._columns(trials)
        rows = list(trials)
        if self.sort_by_metric and self.metric:
            sign = -1 if (self.mode or "max") == "max" else 1
            rows.sort(key=lambda t: sign * (_get(t.last_result or {}, self.metric) or 0))
        shown = rows[:self.max_progress_rows]
        table = []
        for t in shown:
            r = t.last_result or {}
            row = [str(t), t.status]
            row += [_fmt(_get(t.config or {}, k), self.max_column_length) for k in pc]
            row += [_fmt(_get(r, k), self.max_column_length) for k in mc]
            table.append(row)
        head = ["Trial name", "status"] + list(pc.values()) + list(mc.values())
        out = tabulate(table, headers=head, tablefmt="psql")
        if len(rows) > len(shown):
            out += f"\n... {len(rows) - len(shown)} more trials not shown"
        return out

    def _progress_str(self, trials, done, *sys_info) -> str:
        counts: Dict[str, int] = {}
        for t in trials:
            counts[t.status] = counts.get(t.status, 0) + 1
        lines = [f"== Status == (elapsed {time.time() - self._start:.1f}s)",
                 "Number of trials: " + ", ".join(f"{v} {k}" for k, v in sorted(counts.items()))]
        if self.metric:
            best = _best(trials, self.metric, self.mode)
            if best is not None:
                lines.append(f"Current best trial: {best} with {self.metric}={_get(best.last_result, self.metric)}")
        lines += [str(s) for s in sys_info if s]
        if done or self.print_intermediate_tables is not False:
            lines.append(self.trial_table(trials))
        errored = [t for t in trials if t.status == "ERROR"][:self.max_error_rows]
        if errored:
            lines.append("Errored trials: " + ", ".join(str(t) for t in errored))
        return "\n".join(lines)


def _fmt(v, n):
    if v is None:
        return ""
    if isinstance(v, float):
        return f"{v:.5g}"
    s = str(v)
    return s if len(s) <= n else s[:n - 3] + "..."


def _best(trials, metric, mode):
    scored = [t for t in trials if _get(t.last_result or {}, metric) is not None]
    if not scored:
        return None
    key = lambda t: _get(t.last_result, metric)  # noqa: E731
    return max(scored, key=key) if (mode or "max") == "max" else min(scored, key=key)


class CLIReporter(TuneReporterBase):
    def __init__(self, *args, out=None, **kw):
        super().__init__(*args, **kw)
        self._out = out

    def report(self, trials, done, *sys_info):
        print(self._progress_str(trials, done, *sys_info), file=self._out or sys.stdout, flush=True)


class JupyterNotebookReporter(CLIReporter):
    """Same table; the reference renders HTML in a notebook (no IPython dependency here)."""

    def __init__(self, overwrite: bool = True, *args, **kw):
        super().__init__(*args, **kw)
        self.overwrite = overwrite


def detect_reporter(**kw) -> TuneReporterBase:
    return CLIReporter(**kw)
