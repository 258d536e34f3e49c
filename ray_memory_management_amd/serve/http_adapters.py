"""HTTP adapters: turn a Starlette request into the input a deployment graph expects.
Parity: reference python/ray/serve/http_adapters.py (starlette_request, json_request,
json_to_ndarray / NdArray, json_to_multi_ndarray, pandas_read_json)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import numpy as np


def starlette_request(request):
    return request


async def json_request(request) -> Any:
    return await request.json()


def _ndarray(payload: Dict[str, Any]) -> np.ndarray:
    if isinstance(payload, list):
        return np.asarray(payload)
    arr = np.asarray(payload["array"], dtype=payload.get("dtype"))
    if payload.get("shape") is not None:
        arr = arr.reshape(payload["shape"])
    return arr


async def json_to_ndarray(request) -> np.ndarray:
    """Body ``{"array": [...], "shape": [...]?, "dtype": "float32"?}`` (reference NdArray) or a
    plain JSON list."""
    return _ndarray(await request.json())


async def json_to_multi_ndarray(request) -> Dict[str, np.ndarray]:
    body = await request.json()
    return {k: _ndarray(v) for k, v in body.items()}


async def pandas_read_json(request):
    import pandas as pd

    return pd.read_json(await request.body(), orient="records")


def resolve(adapter):
    """A callable adapter from an object or an import path string."""
    if adapter is None:
        return starlette_request
    if isinstance(adapter, str):
        import importlib

        mod, _, name = adapter.rpartition(".")
        return getattr(importlib.import_module(mod), name)
    return adapter
