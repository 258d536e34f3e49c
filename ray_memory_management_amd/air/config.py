"""AIR configs. Parity: reference python/ray/air/config.py."""
from __future__ import annotations

import dataclasses
import os
from typing import Any, Callable, Dict, List, Optional, Union


@dataclasses.dataclass
class ScalingConfig:
    trainer_resources: Optional[Dict[str, float]] = None
    num_workers: Optional[int] = None
    use_gpu: bool = False
    resources_per_worker: Optional[Dict[str, float]] = None
    placement_strategy: str = "PACK"
    _max_cpu_fraction_per_node: Optional[float] = None

    @property
    def _resources_per_worker_not_none(self) -> Dict[str, float]:
        r = dict(self.resources_per_worker or {})
        r.setdefault("CPU", 1.0)
        if self.use_gpu:
            r.setdefault("GPU", 1.0)
        return {k: float(v) for k, v in r.items() if v}

    @property
    def num_cpus_per_worker(self):
        return self._resources_per_worker_not_none.get("CPU", 0)

    @property
    def num_gpus_per_worker(self):
        return self._resources_per_worker_not_none.get("GPU", 0)

    def as_placement_group_factory(self):
        bundles = [dict(self.trainer_resources or {"CPU": 0})] + \
            [self._resources_per_worker_not_none for _ in range(self.num_workers or 1)]
        return bundles


@dataclasses.dataclass
class FailureConfig:
    max_failures: int = 0
    fail_fast: bool = False


@dataclasses.dataclass
class CheckpointConfig:
    num_to_keep: Optional[int] = None
    checkpoint_score_attribute: Optional[str] = None
    checkpoint_score_order: str = "max"
    checkpoint_frequency: int = 0
    checkpoint_at_end: Optional[bool] = None

    def __post_init__(self):
        if self.num_to_keep is not None and self.num_to_keep <= 0:
            raise ValueError(f"Received invalid num_to_keep: {self.num_to_keep}. Must be None or an integer >= 1.")
        if self.checkpoint_score_order not in ("max", "min"):
            raise ValueError("checkpoint_score_order must be either 'max' or 'min'")


@dataclasses.dataclass
class RunConfig:
    name: Optional[str] = None
    local_dir: Optional[str] = None
    storage_path: Optional[str] = None
    callbacks: Optional[List[Any]] = None
    stop: Optional[Union[Dict[str, Any], Callable]] = None
    failure_config: Optional[FailureConfig] = None
    sync_config: Optional[Any] = None
    checkpoint_config: Optional[CheckpointConfig] = None
    progress_reporter: Optional[Any] = None
    verbose: int = 1
    log_to_file: bool = False

    def resolved_dir(self, default_name: str) -> str:
        base = self.storage_path or self.local_dir or os.path.expanduser("~/rmm_results")
        return os.path.join(base, self.name or default_name)


@dataclasses.dataclass
class DatasetConfig:
    fit: Optional[bool] = None
    split: Optional[bool] = None
    required: Optional[bool] = None
    transform: Optional[bool] = None
    use_stream_api: Optional[bool] = None
    global_shuffle: Optional[bool] = None
