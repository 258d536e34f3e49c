"""Per-worker session used inside training/tuning functions. Parity: reference
python/ray/air/session.py (report, get_checkpoint, get_world_rank/size, get_local_rank,
get_dataset_shard, get_trial_name/id/resources)."""
from __future__ import annotations

import queue
import threading
from typing import Any, Dict, Optional

from ray_memory_management_amd.air.checkpoint import Checkpoint


class _Session:
    def __init__(self, world_rank=0, world_size=1, local_rank=0, local_world_size=1, node_rank=0, checkpoint=None,
                 dataset_shards=None, trial_name=None, trial_id=None, trial_resources=None, trial_dir=None,
                 config=None):
        self.world_rank = world_rank
        self.world_size = world_size
        self.local_rank = local_rank
        self.local_world_size = local_world_size
        self.node_rank = node_rank
        self.checkpoint = checkpoint
        self.dataset_shards = dataset_shards or {}
        self.trial_name = trial_name
        self.trial_id = trial_id
        self.trial_resources = trial_resources
        self.trial_dir = trial_dir
        self.config = config or {}
        self.results: "queue.Queue" = queue.Queue(maxsize=1)
        self.continue_event = threading.Event()
        self.iteration = 0
        self.stop_requested = False

    def report(self, metrics: Dict[str, Any], checkpoint: Optional[Checkpoint] = None):
        self.iteration += 1
        m = dict(metrics)
        m.setdefault("training_iteration", self.iteration)
        if checkpoint is not None and checkpoint._data_dict is None and checkpoint._local_path is not None:
            # directory checkpoints are materialised as dicts so they can travel through the store
            checkpoint = Checkpoint.from_dict(checkpoint.to_dict())
        self.continue_event.clear()
        self.results.put(("report", m, checkpoint))
        # lock-step with the driver (reference: synchronous session.report semantics)
        self.continue_event.wait()
        if self.stop_requested:
            raise SystemExit(0)


_session: Optional[_Session] = None


def _set_session(s: Optional[_Session]):
    global _session
    _session = s


def _get_session(warn: bool = True) -> Optional[_Session]:
    return _session


def report(metrics: Dict[str, Any], *, checkpoint: Optional[Checkpoint] = None) -> None:
    s = _session
    if s is None:
        raise RuntimeError("session.report() called outside of a training/tuning function")
    s.report(metrics, checkpoint)


def get_checkpoint() -> Optional[Checkpoint]:
    return _session.checkpoint if _session else None


def get_world_rank() -> int:
    return _session.world_rank if _session else 0


def get_world_size() -> int:
    return _session.world_size if _session else 1


def get_local_rank() -> int:
    return _session.local_rank if _session else 0


def get_local_world_size() -> int:
    return _session.local_world_size if _session else 1


def get_node_rank() -> int:
    return _session.node_rank if _session else 0


def get_dataset_shard(dataset_name: Optional[str] = None):
    if _session is None:
        return None
    shards = _session.dataset_shards
    if dataset_name is None:
        if len(shards) != 1:
            raise ValueError("get_dataset_shard() needs a name when several datasets were passed")
        return next(iter(shards.values()))
    return shards.get(dataset_name)


def get_trial_name():
    return _session.trial_name if _session else None


def get_trial_id():
    return _session.trial_id if _session else None


def get_trial_resources():
    return _session.trial_resources if _session else None


def get_trial_dir():
    return _session.trial_dir if _session else None
