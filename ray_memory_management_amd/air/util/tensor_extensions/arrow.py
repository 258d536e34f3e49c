"""Tensor columns for Arrow: ``ArrowTensorType`` / ``ArrowTensorArray``.

Parity: reference python/ray/air/util/tensor_extensions/arrow.py. Storage is a FIXED-SIZE list of
the flattened cell (``prod(shape)`` values per row) over ONE contiguous value buffer, so
``from_numpy`` wraps the ndarray's memory without a copy and ``to_numpy`` is a reshape of the
value buffer (also zero-copy, slices included). The type is a registered Arrow extension type
(name ``rmm.tensor``, shape serialised as JSON), so it round-trips through IPC / Parquet and maps to
:class:`TensorDtype` in ``Table.to_pandas()``.
"""
from __future__ import annotations

import json
from typing import Tuple

import numpy as np
import pyarrow as pa

_EXT_NAME = "rmm.tensor"


class ArrowTensorType(pa.ExtensionType):
    """Arrow type of a tensor column: per-row `shape`, element type `dtype` (an Arrow DataType)."""

    def __init__(self, shape: Tuple[int, ...], dtype: pa.DataType):
        self._shape = tuple(int(s) for s in shape)
        size = int(np.prod(self._shape)) if self._shape else 1
        super().__init__(pa.list_(dtype, size), _EXT_NAME)

    @property
    def shape(self) -> Tuple[int, ...]:
        return self._shape

    @property
    def scalar_type(self) -> pa.DataType:
        return self.storage_type.value_type

    def __arrow_ext_serialize__(self) -> bytes:
        return json.dumps({"shape": list(self._shape)}).encode()

    @classmethod
    def __arrow_ext_deserialize__(cls, storage_type, serialized):
        meta = json.loads(serialized.decode())
        return cls(tuple(meta["shape"]), storage_type.value_type)

    def __arrow_ext_class__(self):
        return ArrowTensorArray

    def to_pandas_dtype(self):
        from ray_memory_management_amd.air.util.tensor_extensions.pandas import TensorDtype

        return TensorDtype(self._shape, self.scalar_type.to_pandas_dtype())

    def __reduce__(self):
        return ArrowTensorType, (self._shape, self.scalar_type)

    def __str__(self) -> str:
        return f"ArrowTensorType(shape={self._shape}, dtype={self.scalar_type})"

    __repr__ = __str__


try:
    pa.register_extension_type(ArrowTensorType((1,), pa.int64()))
except pa.ArrowKeyError:  # already registered (module reloaded)
    pass


class ArrowTensorArray(pa.ExtensionArray):
    """An Arrow array of equal-shape tensors (see module docstring)."""

    @classmethod
    def from_numpy(cls, arr) -> "ArrowTensorArray":
        """``arr`` of shape [rows, *shape] (or a list of equal-shape ndarrays) → zero-copy when
        ``arr`` is a C-contiguous numeric ndarray."""
        if isinstance(arr, (list, tuple)):
            arr = np.stack([np.asarray(a) for a in arr]) if arr else np.empty((0,))
        arr = np.asarray(arr)
        if arr.ndim < 1:
            raise ValueError("ArrowTensorArray.from_numpy needs at least one dimension (the rows)")
        if arr.dtype == object:
            raise ValueError("ArrowTensorArray.from_numpy needs a numeric / bool ndarray, not dtype=object")
        if not arr.flags.c_contiguous:
            arr = np.ascontiguousarray(arr)
        n, shape = arr.shape[0], arr.shape[1:]
        flat = pa.array(arr.reshape(-1)) if arr.dtype == np.bool_ or arr.dtype.kind in "US" else \
            pa.Array.from_buffers(pa.from_numpy_dtype(arr.dtype), arr.size, [None, pa.py_buffer(arr.reshape(-1))])
        size = int(np.prod(shape)) if shape else 1
        storage = pa.FixedSizeListArray.from_arrays(flat, size)
        typ = ArrowTensorType(shape, flat.type)
        out = pa.ExtensionArray.from_storage(typ, storage)
        assert len(out) == n
        return out

    def to_numpy(self, zero_copy_only: bool = True):
        typ = self.type
        values = self.storage.flatten()  # honours this array's offset / length
        np_vals = values.to_numpy(zero_copy_only=zero_copy_only and typ.scalar_type != pa.bool_())
        return np_vals.reshape((len(self),) + typ.shape)

    def __getitem__(self, key):
        if isinstance(key, slice):
            return super().__getitem__(key)
        i = int(key)
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(f"index {key} out of range for a tensor array of length {len(self)}")
        return self.slice(i, 1).to_numpy()[0]

    def __iter__(self):
        t = self.to_numpy(zero_copy_only=False)
        for i in range(len(self)):
            yield t[i]

    def to_pylist(self):
        return list(iter(self))
