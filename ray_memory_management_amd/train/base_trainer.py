"""Trainer base + DataParallelTrainer. Parity: reference python/ray/train/base_trainer.py and
python/ray/train/data_parallel_trainer.py (fit() → Result, checkpoint bookkeeping per
CheckpointConfig, resume_from_checkpoint, FailureConfig)."""
from __future__ import annotations

import json
import os
import shutil
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

from ray_memory_management_amd.air.checkpoint import Checkpoint
from ray_memory_management_amd.air.config import CheckpointConfig, FailureConfig, RunConfig, ScalingConfig
from ray_memory_management_amd.air.result import Result


class Backend:
    """Process-group setup hooks executed on the worker group (reference train/backend.py)."""

    def on_start(self, worker_group):
        pass

    def on_shutdown(self):
        pass


class BaseTrainer:
    def __init__(self, *, scaling_config: Optional[ScalingConfig] = None, run_config: Optional[RunConfig] = None,
                 datasets: Optional[Dict[str, Any]] = None, preprocessor=None,
                 resume_from_checkpoint: Optional[Checkpoint] = None):
        self.scaling_config = scaling_config or ScalingConfig(num_workers=1)
        self.run_config = run_config or RunConfig()
        self.datasets = datasets or {}
        self.preprocessor = preprocessor
        self.resume_from_checkpoint = resume_from_checkpoint

    def fit(self) -> Result:
        raise NotImplementedError

    def as_trainable(self):
        """A function trainable for Tune: runs fit() with the trial's config merged in."""
        trainer = self

        def trainable(config):
            from ray_memory_management_amd.air import session

            t = trainer._with_config(config)
            res = t.fit()
            if res.error:
                raise res.error
            session.report(res.metrics or {}, checkpoint=res.checkpoint)

        trainable.__name__ = type(self).__name__
        return trainable

    def _with_config(self, config):
        return self


class _CheckpointManager:
    def __init__(self, run_dir: str, cfg: CheckpointConfig):
        self.run_dir = run_dir
        self.cfg = cfg
        self.kept: List[Tuple[str, Dict[str, Any]]] = []
        self.latest: Optional[Checkpoint] = None
        self.count = 0

    def register(self, ckpt: Checkpoint, metrics: Dict[str, Any]) -> Checkpoint:
        path = os.path.join(self.run_dir, f"checkpoint_{self.count:06d}")
        self.count += 1
        ckpt.to_directory(path)
        persisted = Checkpoint.from_directory(path)
        self.latest = persisted
        self.kept.append((path, dict(metrics)))
        n = self.cfg.num_to_keep
        if n is not None and len(self.kept) > n:
            attr = self.cfg.checkpoint_score_attribute
            if attr:
                sign = 1 if self.cfg.checkpoint_score_order == "max" else -1
                # never delete the latest checkpoint
                cand = sorted(self.kept[:-1], key=lambda kv: sign * float(kv[1].get(attr, float("-inf") * sign)))
                victim = cand[0]
            else:
                victim = self.kept[0]
            self.kept.remove(victim)
            shutil.rmtree(victim[0], ignore_errors=True)
        return persisted

    def best(self) -> Optional[Checkpoint]:
        attr = self.cfg.checkpoint_score_attribute
        if not self.kept:
            return None
        if not attr:
            return Checkpoint.from_directory(self.kept[-1][0])
        sign = 1 if self.cfg.checkpoint_score_order == "max" else -1
        path, _ = max(self.kept, key=lambda kv: sign * float(kv[1].get(attr, float("-inf") * sign)))
        return Checkpoint.from_directory(path)

    def all(self):
        return [(Checkpoint.from_directory(p), m) for p, m in self.kept]


class DataParallelTrainer(BaseTrainer):
    _backend_cls = Backend

    def __init__(self, train_loop_per_worker: Callable, *, train_loop_config: Optional[Dict] = None,
                 backend_config=None, scaling_config: Optional[ScalingConfig] = None,
                 run_config: Optional[RunConfig] = None, datasets: Optional[Dict[str, Any]] = None,
                 preprocessor=None, resume_from_checkpoint: Optional[Checkpoint] = None, dataset_config=None):
        super().__init__(scaling_config=scaling_config, run_config=run_config, datasets=datasets,
                         preprocessor=preprocessor, resume_from_checkpoint=resume_from_checkpoint)
        self.train_loop_per_worker = train_loop_per_worker
        self.train_loop_config = dict(train_loop_config or {})
        self.backend_config = backend_config

    def _with_config(self, config):
        import copy

        t = copy.copy(self)
        t.train_loop_config = {**self.train_loop_config, **(config or {}).get("train_loop_config", config or {})}
        return t

    def _backend(self):
        return self._backend_cls()

    def fit(self) -> Result:
        import ray_memory_management_amd as ray
        from ray_memory_management_amd.train._internal.worker_group import TrainingFailedError, run_training

        if not ray.is_initialized():
            ray.init()
        run_dir = self.run_config.resolved_dir(f"{type(self).__name__}_{time.strftime('%Y-%m-%d_%H-%M-%S')}")
        os.makedirs(run_dir, exist_ok=True)
        cm = _CheckpointManager(run_dir, self.run_config.checkpoint_config or CheckpointConfig())
        history: List[Dict[str, Any]] = []
        stop = self.run_config.stop

        def on_report(metrics, ckpt):
            metrics = dict(metrics)
            metrics.setdefault("timestamp", time.time())
            history.append(metrics)
            with open(os.path.join(run_dir, "result.json"), "a") as f:
                f.write(json.dumps({k: v for k, v in metrics.items() if isinstance(v, (int, float, str, bool))}) + "\n")
            if ckpt is not None:
                cm.register(ckpt, metrics)
            for cb in self.run_config.callbacks or []:
                if hasattr(cb, "on_trial_result"):
                    cb.on_trial_result(0, [], None, metrics)
            if callable(stop):
                return stop("train", metrics)
            if isinstance(stop, dict):
                return any(metrics.get(k) is not None and metrics[k] >= v for k, v in stop.items())
            return False

        fc = self.run_config.failure_config or FailureConfig()
        err = None
        datasets = self.datasets
        if self.preprocessor is not None and datasets:
            if "train" in datasets:
                self.preprocessor.fit(datasets["train"])
            datasets = {k: self.preprocessor.transform(v) for k, v in datasets.items()}
        try:
            run_training(self.train_loop_per_worker, self.train_loop_config, self._backend(), self.scaling_config,
                         self.resume_from_checkpoint, datasets, on_report,
                         trial_info={"trial_dir": run_dir}, max_failures=fc.max_failures)
        except TrainingFailedError as e:
            err = e
        return Result(metrics=history[-1] if history else None, checkpoint=cm.latest, error=err, log_dir=run_dir,
                      metrics_history=history, best_checkpoints=cm.all())
