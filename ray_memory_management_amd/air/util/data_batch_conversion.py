"""Batch format conversion (reference air/util/data_batch_conversion.py): predictors and
preprocessors accept pandas DataFrames, numpy arrays or dicts of numpy arrays; internally they
work on pandas and convert back to the caller's format."""
from __future__ import annotations

import enum
from typing import Dict, Union

import numpy as np
import pandas as pd

TENSOR_COLUMN_NAME = "__value__"


class DataType(enum.Enum):
    PANDAS = 1
    ARROW = 2
    NUMPY = 3


def convert_batch_type_to_pandas(data: Union[np.ndarray, pd.DataFrame, Dict[str, np.ndarray]]) -> pd.DataFrame:
    if isinstance(data, pd.DataFrame):
        return data
    if isinstance(data, np.ndarray):
        return pd.DataFrame({TENSOR_COLUMN_NAME: list(data) if data.ndim > 1 else data})
    if isinstance(data, dict):
        return pd.DataFrame({k: list(v) if np.asarray(v).ndim > 1 else np.asarray(v) for k, v in data.items()})
    try:
        import pyarrow as pa

        if isinstance(data, pa.Table):
            return data.to_pandas()
    except ImportError:  # pragma: no cover
        pass
    raise ValueError(f"unsupported batch type {type(data).__name__}")


def convert_pandas_to_batch_type(df: pd.DataFrame, type: DataType):
    if type == DataType.PANDAS:
        return df
    if type == DataType.NUMPY:
        if list(df.columns) == [TENSOR_COLUMN_NAME]:
            return np.stack(df[TENSOR_COLUMN_NAME].to_numpy()) if df[TENSOR_COLUMN_NAME].dtype == object \
                else df[TENSOR_COLUMN_NAME].to_numpy()
        return {c: np.stack(df[c].to_numpy()) if df[c].dtype == object else df[c].to_numpy() for c in df.columns}
    if type == DataType.ARROW:
        import pyarrow as pa

        return pa.Table.from_pandas(df)
    raise ValueError(type)
