"""Result of a training/tuning run. Parity: reference python/ray/air/result.py."""
from __future__ import annotations

import dataclasses
from typing import Any, Dict, List, Optional, Tuple

from ray_memory_management_amd.air.checkpoint import Checkpoint


@dataclasses.dataclass
class Result:
    metrics: Optional[Dict[str, Any]]
    checkpoint: Optional[Checkpoint]
    error: Optional[BaseException] = None
    log_dir: Optional[str] = None
    metrics_history: Optional[List[Dict[str, Any]]] = None
    best_checkpoints: Optional[List[Tuple[Checkpoint, Dict[str, Any]]]] = None

    @property
    def config(self) -> Optional[Dict[str, Any]]:
        return (self.metrics or {}).get("config")

    @property
    def metrics_dataframe(self):
        import pandas as pd

        return pd.DataFrame(self.metrics_history or [])
