"""Implementation of the tune CLI commands (reference tune/cli/commands.py)."""
from __future__ import annotations

import operator
import os
from typing import List, Optional

import pandas as pd

from ray_memory_management_amd.tune.result_grid import load_trials

DEFAULT_TRIAL_COLUMNS = ["trial_id", "training_iteration", "time_total_s"]
_OPS = {"<": operator.lt, "<=": operator.le, "==": operator.eq, "!=": operator.ne, ">=": operator.ge, ">": operator.gt}


def _flatten(d, prefix=""):
    out = {}
    for k, v in d.items():
        if isinstance(v, dict):
            out.update(_flatten(v, f"{prefix}{k}/"))
        else:
            out[f"{prefix}{k}"] = v
    return out


def _apply(df: pd.DataFrame, sort: Optional[List[str]], filter_op: Optional[str], columns: Optional[List[str]],
           limit: Optional[int], desc: bool) -> pd.DataFrame:
    if filter_op:
        col, op, val = filter_op.split(" ", 2)
        if op not in _OPS:
            raise ValueError(f"filter operator must be one of {sorted(_OPS)}")
        try:
            v = float(val)
        except ValueError:
            v = val
        df = df[df[col].apply(lambda x: _OPS[op](x, v))]
    if sort:
        missing = [c for c in sort if c not in df.columns]
        if missing:
            raise KeyError(f"sort columns not found: {missing}")
        df = df.sort_values(by=list(sort), ascending=not desc)
    if columns:
        df = df[[c for c in columns if c in df.columns]]
    if limit:
        df = df.head(int(limit))
    return df


def _emit(df: pd.DataFrame, output: Optional[str]) -> str:
    if output:
        if output.endswith(".pkl"):
            raise ValueError("pickle output is not supported; use .csv or .json")
        (df.to_json(output, orient="records") if output.endswith(".json") else df.to_csv(output, index=False))
        return output
    try:
        from tabulate import tabulate

        return tabulate(df, headers="keys", tablefmt="psql", showindex=False)
    except ImportError:
        return df.to_string(index=False)


def trials_frame(experiment_path: str) -> pd.DataFrame:
    rows = []
    for t in load_trials(os.path.expanduser(experiment_path)):
        r = {"trial_id": t.trial_id, "logdir": t.logdir, **_flatten(t.last_result)}
        r.update({f"config/{k}": v for k, v in _flatten(t.config).items()})
        rows.append(r)
    return pd.DataFrame(rows)


def list_trials(experiment_path: str, sort: Optional[List[str]] = None, output: Optional[str] = None,
                filter_op: Optional[str] = None, info_keys: Optional[List[str]] = None, limit: Optional[int] = None,
                desc: bool = False) -> str:
    df = trials_frame(experiment_path)
    if df.empty:
        return "(no trials)"
    cols = info_keys or [c for c in DEFAULT_TRIAL_COLUMNS if c in df.columns] + \
        [c for c in df.columns if c.startswith("config/")]
    return _emit(_apply(df, sort, filter_op, cols, limit, desc), output)


def list_experiments(project_path: str, sort: Optional[List[str]] = None, output: Optional[str] = None,
                     filter_op: Optional[str] = None, info_keys: Optional[List[str]] = None,
                     limit: Optional[int] = None, desc: bool = False) -> str:
    base = os.path.expanduser(project_path)
    rows = []
    for d in sorted(os.listdir(base)):
        full = os.path.join(base, d)
        if not os.path.isdir(full):
            continue
        trials = load_trials(full)
        if not trials:
            continue
        last = max((os.path.getmtime(t.logdir) for t in trials), default=0.0)
        rows.append({"name": d, "total_trials": len(trials),
                     "running_trials": sum(t.status == "RUNNING" for t in trials),
                     "terminated_trials": sum(t.status == "TERMINATED" for t in trials),
                     "error_trials": sum(t.status == "ERROR" for t in trials), "last_updated": last})
    df = pd.DataFrame(rows)
    if df.empty:
        return "(no experiments)"
    return _emit(_apply(df, sort, filter_op, info_keys, limit, desc), output)
