"""Predictors. Parity: reference python/ray/train/predictor.py (Predictor.from_checkpoint,
predict(data) on numpy / pandas batches, preprocessor applied first) and
python/ray/train/torch/torch_predictor.py (TorchPredictor: model from a TorchCheckpoint, optional
GPU, dtype handling, ``predictions`` column)."""
from __future__ import annotations

from typing import Any, Dict, Optional, Union

import numpy as np

DataBatchType = Union[np.ndarray, Dict[str, np.ndarray], "pandas.DataFrame"]  # noqa: F821


class Predictor:
    def __init__(self, preprocessor=None):
        self._preprocessor = preprocessor

    @classmethod
    def from_checkpoint(cls, checkpoint, **kwargs) -> "Predictor":
        raise NotImplementedError

    def get_preprocessor(self):
        return self._preprocessor

    def set_preprocessor(self, preprocessor):
        self._preprocessor = preprocessor

    def predict(self, data: DataBatchType, **kwargs) -> DataBatchType:
        """Apply the preprocessor, then `_predict_numpy` / `_predict_pandas` on the batch."""
        if self._preprocessor is not None:
            data = self._preprocessor.transform_batch(data)
        try:
            import pandas as pd

            if isinstance(data, pd.DataFrame):
                return self._predict_pandas(data, **kwargs)
        except ImportError:  # pragma: no cover
            pass
        return self._predict_numpy(data, **kwargs)

    def _predict_pandas(self, df, **kwargs):
        import pandas as pd

        cols = list(df.columns)
        scalar = all(np.ndim(df[c].iloc[0]) == 0 for c in cols) if len(df) else True
        if len(cols) == 1:
            v = df[cols[0]].to_numpy()
            arr = np.stack(list(v)) if not scalar else v
        elif scalar:  # feature columns → one [N, C] matrix (reference convert_pandas_to_torch_tensor)
            arr = np.stack([df[c].to_numpy() for c in cols], axis=1)
        else:
            arr = {c: np.stack(list(df[c].to_numpy())) for c in cols}
        out = self._predict_numpy(arr, **kwargs)
        if isinstance(out, dict):
            return pd.DataFrame({k: list(v) if np.ndim(v) > 1 else v for k, v in out.items()})
        return pd.DataFrame({"predictions": list(out) if np.ndim(out) > 1 else out})

    def _predict_numpy(self, data, **kwargs):
        raise NotImplementedError


class TorchPredictor(Predictor):
    """Runs a torch module on batches; on a GPU worker (use_gpu=True) inputs go to the device once
    per batch and the forward runs in bf16 autocast when `amp=True`."""

    def __init__(self, model, preprocessor=None, use_gpu: bool = False, amp: bool = False):
        import torch

        super().__init__(preprocessor)
        self.use_gpu = bool(use_gpu) and torch.cuda.is_available()
        self.device = torch.device("cuda") if self.use_gpu else torch.device("cpu")
        self.model = model.to(self.device).eval()
        self.amp = amp and self.use_gpu

    @classmethod
    def from_checkpoint(cls, checkpoint, model=None, use_gpu: bool = False, **kwargs) -> "TorchPredictor":
        d = checkpoint.to_dict()
        m = d.get("model")
        if isinstance(m, dict):
            if model is None:
                raise ValueError("the checkpoint holds a state_dict: pass `model=` (an instance to load it into)")
            model.load_state_dict(m)
            m = model
        return cls(m, preprocessor=d.get("preprocessor"), use_gpu=use_gpu, **kwargs)

    def _predict_numpy(self, data, dtype=None, **kwargs):
        import torch

        def tens(x):
            t = torch.as_tensor(np.asarray(x))
            if dtype is not None:
                t = t.to(dtype)
            elif t.dtype == torch.float64:
                t = t.float()
            return t.to(self.device, non_blocking=True)

        with torch.inference_mode():
            ctx = torch.autocast("cuda", dtype=torch.bfloat16) if self.amp else _null()
            with ctx:
                if isinstance(data, dict):
                    out = self.model(**{k: tens(v) for k, v in data.items()})
                else:
                    out = self.model(tens(data))
        if isinstance(out, dict):
            return {k: v.float().cpu().numpy() for k, v in out.items()}
        return {"predictions": out.float().cpu().numpy()}


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
