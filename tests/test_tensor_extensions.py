"""Tensor extension types (data.extensions): pandas TensorArray / TensorDtype and Arrow
ArrowTensorArray / ArrowTensorType, and tensor columns flowing through Data blocks.
Mirrors the reference python/ray/air/tests/test_tensor_extension.py."""
import io

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from ray_memory_management_amd.data.extensions import (ArrowTensorArray, ArrowTensorType, TensorArray,
                                                        TensorArrayElement, TensorDtype)


def test_tensor_array_basics_and_ops():
    t = np.arange(24, dtype=np.int64).reshape(4, 2, 3)
    ta = TensorArray(t)
    assert len(ta) == 4 and ta.dtype == TensorDtype((2, 3), np.int64) and ta.nbytes == t.nbytes
    assert isinstance(ta[1], TensorArrayElement) and np.array_equal(np.asarray(ta[1]), t[1])
    assert np.array_equal(ta[1:3].to_numpy(), t[1:3])
    assert np.array_equal(ta[np.array([True, False, True, False])].to_numpy(), t[[0, 2]])
    assert np.array_equal((ta + 1).to_numpy(), t + 1) and np.array_equal((2 * ta).to_numpy(), 2 * t)
    assert np.array_equal((ta == ta).to_numpy(), np.ones_like(t, dtype=bool))
    assert np.array_equal(np.sqrt(ta).to_numpy(), np.sqrt(t))
    assert np.array_equal(ta._reduce("sum").to_numpy(), t.sum(axis=0))
    with pytest.raises(TypeError):
        ta._reduce("kurt")
    # from a list of cells, and cell-shape validation
    assert TensorArray([t[0], t[1]]).numpy_shape == (2, 2, 3)
    with pytest.raises(ValueError):
        TensorArray([np.zeros(2), np.zeros(3)])
    # setitem / take with fill / copy independence
    c = ta.copy()
    c[0] = np.zeros((2, 3), dtype=np.int64)
    assert c.to_numpy()[0].sum() == 0 and ta.to_numpy()[0].sum() == 15
    f = TensorArray(t.astype(np.float64)).take([0, -1], allow_fill=True)
    assert np.isnan(f.to_numpy()[1]).all() and f.isna().tolist() == [False, True]
    assert TensorDtype.construct_from_string(str(ta.dtype)) == ta.dtype
    assert ta.astype(TensorDtype((2, 3), np.float32)).numpy_dtype == np.float32


def test_pandas_frame_with_tensor_column():
    t = np.arange(30, dtype=np.float32).reshape(5, 3, 2)
    df = pd.DataFrame({"x": TensorArray(t), "y": np.arange(5)})
    assert isinstance(df.dtypes["x"], TensorDtype)
    s = df.sort_values("y", ascending=False)
    assert np.array_equal(s["x"].array.to_numpy(), t[::-1])
    both = pd.concat([df, df.iloc[:2]])
    assert both["x"].array.numpy_shape == (7, 3, 2)
    assert np.array_equal(df.iloc[[1, 3]]["x"].to_numpy(), t[[1, 3]])
    assert np.array_equal(df["x"].sum().to_numpy(), t.sum(axis=0))
    codes, uniq = pd.factorize(pd.Series(TensorArray(np.array([[1, 2], [3, 4], [1, 2]]))))
    assert codes.tolist() == [0, 1, 0] and len(uniq) == 2


def test_arrow_tensor_array_zero_copy_and_roundtrips():
    t = np.arange(12.0).reshape(3, 4)
    a = ArrowTensorArray.from_numpy(t)
    assert isinstance(a.type, ArrowTensorType) and a.type.shape == (4,)
    back = a.to_numpy()
    assert np.array_equal(back, t)
    assert np.shares_memory(back, t)  # zero-copy both ways
    assert np.array_equal(a.slice(1, 2).to_numpy(), t[1:])
    assert np.array_equal(a[2], t[2]) and len(a.to_pylist()) == 3
    # pandas -> arrow -> parquet -> arrow -> pandas keeps the tensor type
    df = pd.DataFrame({"x": TensorArray(np.arange(24).reshape(4, 3, 2)), "y": list("abcd")})
    tb = pa.Table.from_pandas(df, preserve_index=False)
    assert isinstance(tb.schema.field("x").type, ArrowTensorType)
    buf = io.BytesIO()
    pq.write_table(tb, buf)
    buf.seek(0)
    df2 = pq.read_table(buf).to_pandas()
    assert isinstance(df2["x"].dtype, TensorDtype)
    assert np.array_equal(df2["x"].array.to_numpy(), np.arange(24).reshape(4, 3, 2))


def test_tensor_columns_through_data_blocks(ray_start):
    import ray_memory_management_amd.data as rd

    arr = np.arange(2 * 8 * 3, dtype=np.float32).reshape(8, 2, 3)
    ds = rd.from_numpy(arr)
    df = ds.to_pandas()
    col = df[df.columns[0]]
    assert isinstance(col.dtype, TensorDtype) and col.array.numpy_shape == (8, 2, 3)
    # a pandas UDF that works on the tensor column; result blocks keep the tensor type
    ds2 = ds.map_batches(lambda b: b.assign(**{b.columns[0]: b[b.columns[0]] * 2}), batch_format="pandas")
    out = np.concatenate([np.asarray(b) for b in ds2.iter_batches(batch_format="numpy")])
    assert np.array_equal(out, arr * 2)
