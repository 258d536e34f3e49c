"""TuneConfig. Parity: reference python/ray/tune/tune_config.py."""
from __future__ import annotations

import dataclasses
from typing import Any, Optional


@dataclasses.dataclass
class TuneConfig:
    metric: Optional[str] = None
    mode: Optional[str] = None
    search_alg: Optional[Any] = None
    scheduler: Optional[Any] = None
    num_samples: int = 1
    max_concurrent_trials: Optional[int] = None
    time_budget_s: Optional[float] = None
    reuse_actors: Optional[bool] = None
    trial_name_creator: Optional[Any] = None
    trial_dirname_creator: Optional[Any] = None
    chdir_to_trial_dir: bool = True
