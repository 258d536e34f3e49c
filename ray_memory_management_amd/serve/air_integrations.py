"""Serving AIR predictors. Parity: reference python/ray/serve/air_integrations.py
(PredictorWrapper / PredictorDeployment: load `predictor_cls.from_checkpoint(checkpoint)` once per
replica, convert the HTTP body with `http_adapter` (default json_to_ndarray), optionally batch
requests with @serve.batch, and return the predictions)."""
from __future__ import annotations

import inspect
from typing import Any, Dict, Optional, Type, Union

import numpy as np

from ray_memory_management_amd.serve.api import deployment
from ray_memory_management_amd.serve.http_adapters import json_to_ndarray, resolve


class PredictorWrapper:
    def __init__(self, predictor_cls, checkpoint, http_adapter=json_to_ndarray, batching_params=None,
                 predict_kwargs: Optional[Dict[str, Any]] = None, **predictor_from_checkpoint_kwargs):
        if isinstance(predictor_cls, str):
            import importlib

            mod, _, name = predictor_cls.rpartition(".")
            predictor_cls = getattr(importlib.import_module(mod), name)
        if isinstance(checkpoint, str):
            from ray_memory_management_amd.air.checkpoint import Checkpoint

            checkpoint = Checkpoint.from_directory(checkpoint)
        self.model = predictor_cls.from_checkpoint(checkpoint, **predictor_from_checkpoint_kwargs)
        self.adapter = resolve(http_adapter)
        self.predict_kwargs = dict(predict_kwargs or {})
        self.batching = batching_params
        if batching_params is not False and batching_params is not None:
            from ray_memory_management_amd.serve.batching import batch

            self._batched = batch(**batching_params)(type(self)._predict_list)
        else:
            self._batched = None

    @staticmethod
    def _to_array(out):
        try:
            import pandas as pd

            if isinstance(out, pd.DataFrame):
                col = "predictions" if "predictions" in out.columns else out.columns[0]
                return np.stack([np.asarray(v) for v in out[col].to_numpy()])
        except ImportError:  # pragma: no cover
            pass
        if isinstance(out, dict):
            out = out.get("predictions", next(iter(out.values())))
        return np.asarray(out)

    async def _predict_list(self, inputs):
        stacked = np.concatenate([np.asarray(x) for x in inputs])
        out = self._to_array(self.model.predict(stacked, **self.predict_kwargs))
        sizes = np.cumsum([len(np.asarray(x)) for x in inputs])[:-1]
        return list(np.split(out, sizes))

    async def predict(self, inp):
        if self._batched is not None:
            return await self._batched(self, inp)
        return self.model.predict(inp, **self.predict_kwargs)

    async def __call__(self, request):
        inp = self.adapter(request)
        if inspect.isawaitable(inp):
            inp = await inp
        out = await self.predict(inp)
        try:
            import pandas as pd

            if isinstance(out, pd.DataFrame):
                return out.to_dict(orient="records")
        except ImportError:  # pragma: no cover
            pass
        return np.asarray(out).tolist() if isinstance(out, np.ndarray) else out


PredictorDeployment = deployment(name="PredictorDeployment")(PredictorWrapper)
