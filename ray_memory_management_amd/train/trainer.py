"""Legacy (v1) Train API kept by the reference next to the AIR trainers.

Parity: reference python/ray/train/trainer.py (Trainer(backend, num_workers, use_gpu,
resources_per_worker).start / run / run_iterator / latest_checkpoint / shutdown /
to_tune_trainable, TrainingIterator), train/callbacks (TrainingCallback.handle_result),
train/train_loop_utils.py (report, world_rank, local_rank, world_size, get_dataset_shard,
save_checkpoint, load_checkpoint), train/checkpoint.py (CheckpointStrategy) and
train/backend.py (BackendConfig). Runs on the same worker group / session machinery as
DataParallelTrainer (train/_internal/worker_group.py)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Union

from ray_memory_management_amd.air import session
from ray_memory_management_amd.air.checkpoint import Checkpoint
from ray_memory_management_amd.air.config import ScalingConfig

TRAIN_DATASET_KEY = "train"


class BackendConfig:
    """Base for backend configs (TorchConfig etc.): `backend_cls` names the worker-group Backend."""

    @property
    def backend_cls(self):
        from ray_memory_management_amd.train.base_trainer import Backend

        return Backend


@dataclass
class CheckpointStrategy:
    num_to_keep: Optional[int] = None
    checkpoint_score_attribute: str = "_timestamp"
    checkpoint_score_order: str = "max"


class TrainingCallback:
    def start_training(self, logdir: str, config: Dict, **info) -> None:
        pass

    def handle_result(self, results: List[Dict], **info) -> None:
        pass

    def finish_training(self, error: bool = False, **info) -> None:
        pass


# --- in-loop helpers (v1 names over the AIR session) -------------------------------------------
def report(**metrics) -> None:
    session.report(dict(metrics))


def world_rank() -> int:
    return session.get_world_rank()


def local_rank() -> int:
    return session.get_local_rank()


def world_size() -> int:
    return session.get_world_size()


def get_dataset_shard(dataset_name: Optional[str] = None):
    return session.get_dataset_shard(dataset_name)


def save_checkpoint(**kwargs) -> None:
    session.report({"_checkpoint_only": True}, checkpoint=Checkpoint.from_dict(dict(kwargs)))


def load_checkpoint() -> Optional[Dict]:
    ck = session.get_checkpoint()
    return ck.to_dict() if ck is not None else None


def _backend_for(backend: Union[str, BackendConfig]):
    if not isinstance(backend, str):  # BackendConfig / TorchConfig instance
        return backend
    if backend == "torch":
        from ray_memory_management_amd.train.torch import TorchConfig

        return TorchConfig()
    raise ValueError(f"backend {backend!r}: this framework ships the 'torch' backend (TensorFlow / Horovod "
                     "are not part of the MI355X stack)")


class TrainingIterator:
    """Iterates the per-report results: yields one list per report round (rank 0's metrics)."""

    def __init__(self, results: List[List[Dict]], returns: List[Any]):
        self._results, self._returns = results, returns

    def __iter__(self):
        return iter(self._results)

    def get_final_results(self, force: bool = False) -> List[Any]:
        return self._returns

    def is_finished(self) -> bool:
        return True


class Trainer:
    def __init__(self, backend: Union[str, BackendConfig], num_workers: int, use_gpu: bool = False,
                 resources_per_worker: Optional[Dict[str, float]] = None, logdir: Optional[str] = None,
                 max_retries: int = 3):
        self.backend_config = _backend_for(backend)
        self.scaling = ScalingConfig(num_workers=num_workers, use_gpu=use_gpu,
                                     resources_per_worker=resources_per_worker)
        self.logdir, self.max_retries = logdir, max_retries
        self.latest_checkpoint: Optional[Dict] = None
        self._started = False

    def start(self) -> None:
        import ray_memory_management_amd as ray

        if not ray.is_initialized():
            ray.init()
        self._started = True

    def _run(self, train_func: Callable, config: Optional[Dict], dataset, checkpoint):
        from ray_memory_management_amd.train._internal.worker_group import run_training
        from ray_memory_management_amd.train.torch import TorchTrainer

        if not self._started:
            raise RuntimeError("Trainer.start() must be called before run()")
        reports: List[Dict] = []

        def on_report(metrics, ckpt):
            if metrics and not metrics.get("_checkpoint_only"):
                reports.append(dict(metrics))
            if ckpt is not None:
                self.latest_checkpoint = ckpt.to_dict()
            return False

        fn = train_func
        if train_func.__code__.co_argcount == 0:
            fn = lambda _cfg: train_func()  # noqa: E731
        datasets = dataset if isinstance(dataset, dict) else ({TRAIN_DATASET_KEY: dataset} if dataset else {})
        ck = Checkpoint.from_dict(checkpoint) if isinstance(checkpoint, dict) else checkpoint
        backend = TorchTrainer(lambda c: None, torch_config=self.backend_config)._backend()
        returns = run_training(fn, dict(config or {}), backend, self.scaling, ck, datasets, on_report,
                               trial_info={"trial_dir": self.logdir or ""}, max_failures=self.max_retries)
        # one entry per report round; the session forwards rank 0's metrics (AIR semantics), which
        # every rank computed from the same collective state
        return [[r] for r in reports], returns

    def run(self, train_func: Callable, config: Optional[Dict] = None,
            callbacks: Optional[List[TrainingCallback]] = None, dataset=None, checkpoint=None,
            checkpoint_strategy: Optional[CheckpointStrategy] = None) -> List[Any]:
        callbacks = callbacks or []
        for cb in callbacks:
            cb.start_training(self.logdir or "", dict(config or {}))
        err = False
        try:
            rounds, returns = self._run(train_func, config, dataset, checkpoint)
            for r in rounds:
                for cb in callbacks:
                    cb.handle_result(r)
            return returns
        except BaseException:
            err = True
            raise
        finally:
            for cb in callbacks:
                cb.finish_training(error=err)

    def run_iterator(self, train_func: Callable, config: Optional[Dict] = None, dataset=None,
                     checkpoint=None, checkpoint_strategy=None) -> TrainingIterator:
        rounds, returns = self._run(train_func, config, dataset, checkpoint)
        return TrainingIterator(rounds, returns)

    def to_tune_trainable(self, train_func: Callable, dataset=None):
        trainer = self

        def trainable(config):
            trainer.start()
            rounds, _ = trainer._run(train_func, config, dataset, None)
            for r in rounds:
                session.report(r[0])

        return trainable

    def shutdown(self) -> None:
        self._started = False
