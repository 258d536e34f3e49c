"""Per-process Dataset execution options. Parity: reference python/ray/data/context.py
(DatasetContext.get_current(): target block size, push-based shuffle, lazy/eager knobs)."""
from __future__ import annotations

import os
import threading

_lock = threading.Lock()
_ctx = None


class DatasetContext:
    def __init__(self):
        self.target_max_block_size = 512 * 1024 * 1024
        self.target_min_block_size = 1 * 1024 * 1024
        self.block_splitting_enabled = False
        self.use_push_based_shuffle = bool(int(os.environ.get("RAY_DATASET_PUSH_BASED_SHUFFLE", "0")))
        self.optimize_fuse_stages = True
        self.block_until_stage_done = False
        self.default_parallelism = 200
        self.min_parallelism = 8
        self.scheduling_strategy = "DEFAULT"

    @staticmethod
    def get_current() -> "DatasetContext":
        global _ctx
        with _lock:
            if _ctx is None:
                _ctx = DatasetContext()
            return _ctx

    @staticmethod
    def _set_current(ctx: "DatasetContext") -> None:
        global _ctx
        _ctx = ctx
