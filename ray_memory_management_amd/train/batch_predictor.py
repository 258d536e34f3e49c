"""BatchPredictor: score a Dataset with a Predictor built from a Checkpoint on a pool of actors.

Parity: reference python/ray/train/batch_predictor.py:19 (from_checkpoint, predict(dataset,
batch_size, min/max_scoring_workers, num_cpus/num_gpus_per_worker, feature_columns, keep_columns,
**predict_kwargs) -> Dataset via map_batches on an ActorPoolStrategy; predict_pipelined).
Each scoring actor builds the predictor once (the checkpoint travels through the object store) and
keeps it resident, so a GPU scoring worker loads its weights into HBM exactly once.
"""
from __future__ import annotations

from typing import List, Optional, Type


class BatchPredictor:
    def __init__(self, checkpoint, predictor_cls: Type, **predictor_kwargs):
        self._checkpoint = checkpoint
        self._predictor_cls = predictor_cls
        self._predictor_kwargs = predictor_kwargs

    @classmethod
    def from_checkpoint(cls, checkpoint, predictor_cls: Type, **kwargs) -> "BatchPredictor":
        return cls(checkpoint, predictor_cls, **kwargs)

    def get_preprocessor(self):
        return self._checkpoint.to_dict().get("preprocessor")

    def predict(self, data, *, feature_columns: Optional[List[str]] = None,
                keep_columns: Optional[List[str]] = None, batch_size: int = 4096, min_scoring_workers: int = 1,
                max_scoring_workers: Optional[int] = None, num_cpus_per_worker: Optional[float] = None,
                num_gpus_per_worker: Optional[float] = None, separate_gpu_stage: bool = True,
                ray_remote_args: Optional[dict] = None, **predict_kwargs):
        from ray_memory_management_amd.data import ActorPoolStrategy

        ckpt, pcls, pkw = self._checkpoint, self._predictor_cls, dict(self._predictor_kwargs)
        if num_gpus_per_worker:
            pkw.setdefault("use_gpu", True)

        class ScoringWrapper:
            def __init__(self):
                self.predictor = pcls.from_checkpoint(ckpt, **pkw)

            def __call__(self, batch):
                import pandas as pd

                df = batch if isinstance(batch, pd.DataFrame) else pd.DataFrame(batch)
                features = df[feature_columns] if feature_columns else (
                    df.drop(columns=keep_columns) if keep_columns else df)
                out = self.predictor.predict(features, **predict_kwargs)
                if not isinstance(out, pd.DataFrame):
                    out = pd.DataFrame(out)
                if keep_columns:
                    out = out.reset_index(drop=True)
                    for c in keep_columns:
                        out[c] = df[c].reset_index(drop=True)
                return out

        opts = dict(ray_remote_args or {})
        if num_cpus_per_worker is not None:
            opts["num_cpus"] = num_cpus_per_worker
        if num_gpus_per_worker is not None:
            opts["num_gpus"] = num_gpus_per_worker
        compute = ActorPoolStrategy(min_scoring_workers, max_scoring_workers or min_scoring_workers)
        return data.map_batches(ScoringWrapper, batch_size=batch_size, batch_format="pandas", compute=compute,
                                **opts)

    def predict_pipelined(self, data, *, blocks_per_window: Optional[int] = None,
                          bytes_per_window: Optional[int] = None, **kwargs):
        """Windowed scoring: a DatasetPipeline whose windows are predicted as they are consumed
        (bounded memory for datasets larger than the object store)."""
        pipe = data.window(blocks_per_window=blocks_per_window or 1, bytes_per_window=bytes_per_window)
        return pipe.foreach_window(lambda ds: self.predict(ds, **kwargs))
