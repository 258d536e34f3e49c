"""scikit-learn on the runtime. Parity: reference python/ray/train/sklearn/{sklearn_trainer,
sklearn_checkpoint,sklearn_predictor}.py: SklearnTrainer fits an estimator in ONE worker actor
(n_jobs set to the worker's CPUs), scores it on every extra dataset, optionally cross-validates
with the cluster-backed joblib backend (`util.joblib`, CV folds fanned out as tasks), and returns a
checkpoint holding the fitted estimator; SklearnPredictor scores numpy / pandas batches."""
from __future__ import annotations

import os
import pickle
import time
from typing import Any, Dict, List, Optional, Union

import numpy as np

from ray_memory_management_amd.air.checkpoint import Checkpoint
from ray_memory_management_amd.air.config import RunConfig, ScalingConfig
from ray_memory_management_amd.air.result import Result
from ray_memory_management_amd.train.base_trainer import BaseTrainer
from ray_memory_management_amd.train.predictor import Predictor

MODEL_KEY = "model"


def _xy(ds, label_column: Optional[str]):
    df = ds.to_pandas() if hasattr(ds, "to_pandas") else ds
    if label_column is None:
        return df, None
    return df.drop(columns=[label_column]), df[label_column]


def _fit_in_worker(estimator, train, label_column, evals: Dict[str, Any], scoring, cv, parallelize_cv: bool,
                   params: Dict, return_train_score_cv: bool, n_cpus: int):
    from sklearn.base import clone
    from sklearn.metrics import check_scoring

    est = clone(estimator).set_params(**params) if params else clone(estimator)
    if hasattr(est, "n_jobs"):
        try:
            est.set_params(n_jobs=max(1, n_cpus))
        except ValueError:
            pass
    X, y = _xy(train, label_column)
    metrics: Dict[str, Any] = {}
    if cv:
        from sklearn.model_selection import cross_validate

        kw = dict(cv=cv, scoring=scoring, return_train_score=return_train_score_cv)
        import ray_memory_management_amd as ray

        folds = cv if isinstance(cv, int) else getattr(cv, "n_splits", 5)
        free = int(ray.available_resources().get("CPU", 0)) if parallelize_cv else 0
        if parallelize_cv and free >= 1:  # one fold per free CPU (this task holds its own)
            import joblib

            from ray_memory_management_amd.util.joblib import register_ray

            register_ray()
            with joblib.parallel_backend("ray"):
                res = cross_validate(est, X, y, n_jobs=max(1, min(folds, free)), **kw)
        else:
            res = cross_validate(est, X, y, **kw)
        metrics["cv"] = {k: np.asarray(v).tolist() for k, v in res.items()}
        for k, v in res.items():
            metrics[f"cv/{k}_mean"] = float(np.mean(v))
    t0 = time.time()
    est.fit(X, y)
    metrics["fit_time"] = time.time() - t0
    for name, ds in evals.items():
        Xe, ye = _xy(ds, label_column)
        if isinstance(scoring, dict):
            for sname, sc in scoring.items():
                metrics[f"{name}/{sname}"] = float(check_scoring(est, sc)(est, Xe, ye))
        else:
            metrics[f"{name}/score"] = float(check_scoring(est, scoring)(est, Xe, ye))
    return pickle.dumps(est), metrics


class SklearnTrainer(BaseTrainer):
    def __init__(self, *, estimator, datasets: Dict[str, Any], label_column: Optional[str] = None,
                 params: Optional[Dict[str, Any]] = None, scoring=None, cv=None, return_train_score_cv: bool = False,
                 parallelize_cv: Optional[bool] = None, set_estimator_cpus: bool = True,
                 scaling_config: Optional[ScalingConfig] = None, run_config: Optional[RunConfig] = None,
                 preprocessor=None, **kw):
        if "train" not in datasets:
            raise KeyError("SklearnTrainer needs a 'train' dataset")
        if scaling_config is not None and scaling_config.num_workers not in (None, 1):
            raise ValueError("SklearnTrainer runs one worker (num_workers must be 1); CV folds parallelise "
                             "across the cluster instead")
        super().__init__(scaling_config=scaling_config or ScalingConfig(num_workers=1), run_config=run_config,
                         datasets=datasets, preprocessor=preprocessor)
        self.estimator, self.label_column, self.params = estimator, label_column, dict(params or {})
        self.scoring, self.cv, self.return_train_score_cv = scoring, cv, return_train_score_cv
        self.parallelize_cv = bool(cv) if parallelize_cv is None else parallelize_cv
        self.set_estimator_cpus = set_estimator_cpus

    def _with_config(self, config):
        import copy

        t = copy.copy(self)
        t.params = {**self.params, **(config or {}).get("params", {})}
        return t

    def fit(self) -> Result:
        import ray_memory_management_amd as ray

        if not ray.is_initialized():
            ray.init()
        datasets = dict(self.datasets)
        if self.preprocessor is not None:
            self.preprocessor.fit(datasets["train"])
            datasets = {k: self.preprocessor.transform(v) for k, v in datasets.items()}
        # materialise to pandas once on the driver; the frames travel through the object store
        frames = {k: (v.to_pandas() if hasattr(v, "to_pandas") else v) for k, v in datasets.items()}
        train = frames.pop("train")
        cpus = int((self.scaling_config.resources_per_worker or {}).get("CPU", 1) or 1)
        fn = ray.remote(_fit_in_worker).options(num_cpus=cpus)
        run_dir = self.run_config.resolved_dir(f"SklearnTrainer_{time.strftime('%Y-%m-%d_%H-%M-%S')}")
        os.makedirs(run_dir, exist_ok=True)
        try:
            blob, metrics = ray.get(fn.remote(self.estimator, train, self.label_column, frames, self.scoring, self.cv,
                                              self.parallelize_cv, self.params, self.return_train_score_cv,
                                              cpus if self.set_estimator_cpus else 1))
        except Exception as e:  # noqa: BLE001
            return Result(metrics=None, checkpoint=None, error=e, log_dir=run_dir)
        ck = Checkpoint.from_dict({MODEL_KEY: blob, "preprocessor": self.preprocessor})
        path = os.path.join(run_dir, "checkpoint_000000")
        ck.to_directory(path)
        metrics = {k: v for k, v in metrics.items()}
        metrics["done"] = True
        return Result(metrics=metrics, checkpoint=Checkpoint.from_directory(path), error=None, log_dir=run_dir,
                      metrics_history=[metrics])


def load_estimator(checkpoint: Checkpoint):
    d = checkpoint.to_dict()
    return pickle.loads(d[MODEL_KEY]), d.get("preprocessor")


class SklearnPredictor(Predictor):
    def __init__(self, estimator, preprocessor=None):
        super().__init__(preprocessor)
        self.estimator = estimator

    @classmethod
    def from_checkpoint(cls, checkpoint: Checkpoint, **kw) -> "SklearnPredictor":
        est, pre = load_estimator(checkpoint)
        return cls(est, pre)

    def predict(self, data, feature_columns: Optional[List[str]] = None, **kw):
        import pandas as pd

        if self._preprocessor is not None:
            data = self._preprocessor.transform_batch(data)
        if isinstance(data, pd.DataFrame):
            X = data[feature_columns] if feature_columns else data
            return pd.DataFrame({"predictions": self.estimator.predict(X)})
        X = np.asarray(data)
        if feature_columns:
            X = X[:, feature_columns]
        return self.estimator.predict(X)


class SklearnCheckpoint(Checkpoint):
    """Checkpoint holding a fitted estimator (+ optional preprocessor) (reference
    train/sklearn/sklearn_checkpoint.py); readable by SklearnPredictor.from_checkpoint."""

    @classmethod
    def from_estimator(cls, estimator, *, preprocessor=None) -> "SklearnCheckpoint":
        d = {MODEL_KEY: pickle.dumps(estimator)}  # same layout SklearnTrainer writes
        if preprocessor is not None:
            d["preprocessor"] = preprocessor
        return cls.from_dict(d)

    def get_estimator(self):
        return load_estimator(self)[0]

    def get_preprocessor(self):
        return self.to_dict().get("preprocessor")
