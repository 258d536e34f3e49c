"""Serve configs. Parity: reference python/ray/serve/config.py (AutoscalingConfig,
DeploymentConfig, HTTPOptions, ReplicaConfig)."""
from __future__ import annotations

import dataclasses
from typing import Any, Dict, Optional


@dataclasses.dataclass
class AutoscalingConfig:
    min_replicas: int = 1
    max_replicas: int = 1
    target_num_ongoing_requests_per_replica: float = 1.0
    metrics_interval_s: float = 0.5
    look_back_period_s: float = 2.0
    smoothing_factor: float = 1.0
    downscale_delay_s: float = 2.0
    upscale_delay_s: float = 0.5

    def __post_init__(self):
        if self.min_replicas < 0 or self.max_replicas < max(self.min_replicas, 1):
            raise ValueError("require 0 <= min_replicas <= max_replicas and max_replicas >= 1")


@dataclasses.dataclass
class DeploymentConfig:
    num_replicas: int = 1
    max_concurrent_queries: int = 100
    user_config: Any = None
    graceful_shutdown_timeout_s: float = 2.0
    health_check_period_s: float = 2.0
    health_check_timeout_s: float = 30.0
    autoscaling_config: Optional[AutoscalingConfig] = None


@dataclasses.dataclass
class HTTPOptions:
    host: str = "127.0.0.1"
    port: int = 8000
    root_path: str = ""
    location: str = "HeadOnly"
    middlewares: Any = None
