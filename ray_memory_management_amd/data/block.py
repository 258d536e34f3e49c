"""Blocks: the unit of data a Dataset distributes through the object store.

Parity: reference python/ray/data/block.py (Block, BlockAccessor, BlockMetadata) and
_internal/{simple_block,arrow_block,pandas_block,tensor_block}.py.

Three block kinds:
  * ``list``            — "simple" blocks of arbitrary Python rows (from_items of non-dicts, range);
  * ``pyarrow.Table``   — tabular rows (dict rows, pandas batches, CSV/JSON/Parquet);
  * ``NumpyBlock``      — dict of equal-length numpy columns (range_tensor, from_numpy, numpy
    batches). Tensor columns live in the shm store as pickle-5 out-of-band buffers, so workers
    map them zero-copy, and `iter_torch_batches(device="cuda")` can DMA them straight to HBM.

BlockAccessor gives every operator a uniform view: num_rows / slice / take / concat / sort /
to_batch(format) / iter_rows / schema / size_bytes.
"""
from __future__ import annotations

import bisect
import random
from dataclasses import dataclass, field
from typing import Any, Dict, Iterator, List, Optional, Sequence, Union

import numpy as np

try:
    import pyarrow as pa
except ImportError:  # pragma: no cover
    pa = None

TENSOR_COL = "__value__"


class NumpyBlock(dict):
    """Columnar block of numpy arrays (all columns share the leading dimension)."""


Block = Union[list, "pa.Table", NumpyBlock]


@dataclass
class BlockMetadata:
    num_rows: Optional[int]
    size_bytes: Optional[int]
    schema: Any
    input_files: List[str] = field(default_factory=list)
    exec_stats: Optional[dict] = None


def _pandas():
    import pandas as pd

    return pd


class BlockAccessor:
    """Uniform operations over a block."""

    def __init__(self, block):
        self.block = block

    @staticmethod
    def for_block(block) -> "BlockAccessor":
        if isinstance(block, NumpyBlock):
            return NumpyAccessor(block)
        if isinstance(block, list):
            return SimpleAccessor(block)
        if pa is not None and isinstance(block, pa.Table):
            return ArrowAccessor(block)
        pd = _pandas()
        if isinstance(block, pd.DataFrame):
            return ArrowAccessor(pa.Table.from_pandas(block, preserve_index=False))
        if isinstance(block, dict):
            return NumpyAccessor(NumpyBlock({k: np.asarray(v) for k, v in block.items()}))
        if isinstance(block, np.ndarray):
            return NumpyAccessor(NumpyBlock({TENSOR_COL: block}))
        raise TypeError(f"Not a block type: {type(block)}")

    # subclasses implement ------------------------------------------------
    def num_rows(self) -> int: ...
    def size_bytes(self) -> int: ...
    def schema(self): ...
    def slice(self, start: int, end: int, copy: bool = False): ...
    def take(self, indices) -> Any: ...
    def iter_rows(self) -> Iterator: ...
    def to_pandas(self): ...
    def to_arrow(self): ...
    def to_numpy(self, column: Optional[str] = None): ...
    def column_names(self) -> Optional[List[str]]: return None

    # shared ----------------------------------------------------------------
    def get_metadata(self, input_files=None, exec_stats=None) -> BlockMetadata:
        return BlockMetadata(self.num_rows(), self.size_bytes(), self.schema(), list(input_files or []), exec_stats)

    def random_shuffle(self, seed: Optional[int]):
        idx = np.random.default_rng(seed).permutation(self.num_rows())
        return self.take(idx)

    def to_batch(self, batch_format: str):
        if batch_format in ("native", "default"):
            if isinstance(self, ArrowAccessor):
                return self.to_pandas()
            if isinstance(self, NumpyAccessor):
                return self.to_numpy()
            return self.block
        if batch_format == "pandas":
            return self.to_pandas()
        if batch_format in ("pyarrow", "arrow"):
            return self.to_arrow()
        if batch_format == "numpy":
            return self.to_numpy()
        raise ValueError(f"batch_format must be one of native/pandas/pyarrow/numpy, got {batch_format!r}")

    def sample(self, n: int, key) -> list:
        """n evenly-spaced sort-key values (for range partitioning)."""
        rows = self.num_rows()
        if rows == 0:
            return []
        k = min(n, rows)
        idx = np.linspace(0, rows - 1, k).astype(np.int64)
        return [_key_of(r, key) for r in BlockAccessor.for_block(self.take(idx)).iter_rows()]


def _key_of(row, key):
    if key is None:
        return row
    if callable(key):
        return key(row)
    if isinstance(key, (list, tuple)):
        return tuple(row[k] for k in key)
    return row[key]


class SimpleAccessor(BlockAccessor):
    def num_rows(self):
        return len(self.block)

    def size_bytes(self):
        import sys

        n = len(self.block)
        if n == 0:
            return 0
        sample = self.block[: min(n, 16)]
        return int(sum(sys.getsizeof(x) for x in sample) * n / len(sample))

    def schema(self):
        return type(self.block[0]) if self.block else None

    def slice(self, start, end, copy=False):
        return list(self.block[start:end])

    def take(self, indices):
        return [self.block[int(i)] for i in indices]

    def iter_rows(self):
        return iter(self.block)

    def to_pandas(self):
        pd = _pandas()
        return pd.DataFrame({"value": self.block})

    def to_arrow(self):
        return pa.Table.from_pandas(self.to_pandas(), preserve_index=False)

    def to_numpy(self, column=None):
        return np.asarray(self.block)

    def sort(self, key, descending=False):
        return sorted(self.block, key=(lambda r: _key_of(r, key)), reverse=descending)


class ArrowAccessor(BlockAccessor):
    def num_rows(self):
        return self.block.num_rows

    def size_bytes(self):
        return int(self.block.nbytes)

    def schema(self):
        return self.block.schema

    def column_names(self):
        return list(self.block.column_names)

    def slice(self, start, end, copy=False):
        return self.block.slice(start, max(end - start, 0))

    def take(self, indices):
        return self.block.take(pa.array(np.asarray(indices, dtype=np.int64)))

    def iter_rows(self):
        cols = self.block.column_names
        data = [c.to_pylist() for c in self.block.columns]
        for i in range(self.block.num_rows):
            yield {k: d[i] for k, d in zip(cols, data)}

    def to_pandas(self):
        return self.block.to_pandas()

    def to_arrow(self):
        return self.block

    def to_numpy(self, column=None):
        if column is not None:
            return _arrow_col_numpy(self.block.column(column))
        if self.block.column_names == [TENSOR_COL]:  # a tensor dataset: the ndarray itself
            return _arrow_col_numpy(self.block.column(TENSOR_COL))
        return {c: _arrow_col_numpy(self.block.column(c)) for c in self.block.column_names}

    def sort(self, key, descending=False):
        keys = [key] if isinstance(key, str) else list(key)
        order = "descending" if descending else "ascending"
        return self.block.sort_by([(k, order) for k in keys])


def _arrow_col_numpy(col):
    from ray_memory_management_amd.air.util.tensor_extensions.arrow import ArrowTensorType

    if isinstance(col.type, ArrowTensorType):  # tensor column: zero-copy reshape per chunk
        chunks = col.chunks if isinstance(col, pa.ChunkedArray) else [col]
        parts = [c.to_numpy(zero_copy_only=False) for c in chunks]
        return parts[0] if len(parts) == 1 else np.concatenate(parts) if parts else \
            np.empty((0,) + col.type.shape)
    try:
        return col.to_numpy(zero_copy_only=False)
    except Exception:
        return np.asarray(col.to_pylist())


class NumpyAccessor(BlockAccessor):
    def num_rows(self):
        return len(next(iter(self.block.values()))) if self.block else 0

    def size_bytes(self):
        return int(sum(v.nbytes for v in self.block.values()))

    def schema(self):
        return {k: (v.dtype, v.shape[1:]) for k, v in self.block.items()}

    def column_names(self):
        return list(self.block.keys())

    def slice(self, start, end, copy=False):
        return NumpyBlock({k: (v[start:end].copy() if copy else v[start:end]) for k, v in self.block.items()})

    def take(self, indices):
        idx = np.asarray(indices, dtype=np.int64)
        return NumpyBlock({k: v[idx] for k, v in self.block.items()})

    def iter_rows(self):
        keys = list(self.block.keys())
        if keys == [TENSOR_COL]:
            yield from self.block[TENSOR_COL]
            return
        for i in range(self.num_rows()):
            yield {k: self.block[k][i] for k in keys}

    def to_pandas(self):
        """Tensor columns (ndim > 1) become TensorArray columns (data.extensions), as in the
        reference: one contiguous ndarray per column, no per-cell Python objects."""
        pd = _pandas()
        from ray_memory_management_amd.air.util.tensor_extensions.pandas import TensorArray

        return pd.DataFrame({k: (TensorArray(v) if v.ndim > 1 else v) for k, v in self.block.items()})

    def to_arrow(self):
        from ray_memory_management_amd.air.util.tensor_extensions.arrow import ArrowTensorArray

        cols = {}
        for k, v in self.block.items():
            # tensor columns: zero-copy fixed-size-list extension arrays (ArrowTensorType)
            cols[k] = ArrowTensorArray.from_numpy(v) if v.ndim > 1 else pa.array(v)
        return pa.table(cols)

    def to_numpy(self, column=None):
        if column is not None:
            return self.block[column]
        if list(self.block.keys()) == [TENSOR_COL]:
            return self.block[TENSOR_COL]
        return dict(self.block)

    def sort(self, key, descending=False):
        keys = [key] if isinstance(key, str) else list(key)
        order = np.lexsort([self.block[k] for k in reversed(keys)])
        if descending:
            order = order[::-1]
        return self.take(order)


# ---------------------------------------------------------------------- building blocks
def batch_to_block(batch) -> Block:
    """Normalise a UDF's returned batch into a block."""
    if isinstance(batch, (list, NumpyBlock)):
        return batch
    if pa is not None and isinstance(batch, pa.Table):
        return batch
    pd = _pandas()
    if isinstance(batch, pd.DataFrame):
        return pa.Table.from_pandas(batch, preserve_index=False)
    if isinstance(batch, np.ndarray):
        return NumpyBlock({TENSOR_COL: batch})
    if isinstance(batch, dict):
        return NumpyBlock({k: np.asarray(v) for k, v in batch.items()})
    try:
        import torch

        if isinstance(batch, torch.Tensor):
            return NumpyBlock({TENSOR_COL: batch.detach().cpu().numpy()})
    except ImportError:  # pragma: no cover
        pass
    raise ValueError(f"The map batches UDF returned a value of type {type(batch)}, which is not allowed. "
                     "The return type must be one of: list, pandas.DataFrame, pyarrow.Table, numpy.ndarray, dict.")


class BlockBuilder:
    """Accumulates rows / blocks and emits one block of the right kind."""

    def __init__(self):
        self._rows: list = []
        self._blocks: list = []
        self._kind: Optional[str] = None

    def add(self, row):
        if self._kind is None:
            self._kind = "arrow" if isinstance(row, dict) else "simple"
        self._rows.append(row)

    def add_block(self, block):
        if BlockAccessor.for_block(block).num_rows() == 0:
            return
        self._flush_rows()
        self._blocks.append(block)

    def _flush_rows(self):
        if self._rows:
            if self._kind == "arrow":
                self._blocks.append(pa.Table.from_pylist(self._rows))
            else:
                self._blocks.append(list(self._rows))
            self._rows = []

    def build(self) -> Block:
        self._flush_rows()
        return concat_blocks(self._blocks)

    def num_rows(self):
        return len(self._rows) + sum(BlockAccessor.for_block(b).num_rows() for b in self._blocks)


def concat_blocks(blocks: Sequence) -> Block:
    blocks = [b for b in blocks if BlockAccessor.for_block(b).num_rows() > 0] or list(blocks[:1])
    if not blocks:
        return []
    if len(blocks) == 1:
        return blocks[0]
    kinds = {type(BlockAccessor.for_block(b)) for b in blocks}
    if kinds == {SimpleAccessor}:
        out = []
        for b in blocks:
            out.extend(b)
        return out
    if kinds == {NumpyAccessor}:
        keys = list(blocks[0].keys())
        return NumpyBlock({k: np.concatenate([b[k] for b in blocks]) for k in keys})
    tables = [BlockAccessor.for_block(b).to_arrow() for b in blocks]
    return pa.concat_tables(tables, promote_options="default")


def merge_sorted_blocks(blocks: Sequence, key, descending=False) -> Block:
    b = concat_blocks(blocks)
    acc = BlockAccessor.for_block(b)
    return acc.sort(key, descending) if acc.num_rows() else b


def partition_by_boundaries(block, key, boundaries: list, descending=False) -> List[Block]:
    """Split a SORTED block into len(boundaries)+1 range partitions."""
    acc = BlockAccessor.for_block(block)
    keys = [_key_of(r, key) for r in acc.iter_rows()] if not isinstance(acc, NumpyAccessor) or key is None \
        else list(acc.block[key] if isinstance(key, str) else zip(*[acc.block[k] for k in key]))
    if descending:
        neg = [_Desc(k) for k in keys]
        bnd = [_Desc(b) for b in boundaries]
        cuts = [bisect.bisect_left(neg, b) for b in bnd]
    else:
        cuts = [bisect.bisect_left(keys, b) for b in boundaries]
    out, prev = [], 0
    for c in cuts + [acc.num_rows()]:
        out.append(acc.slice(prev, c))
        prev = c
    return out


class _Desc:
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def __lt__(self, o):
        return self.v > o.v

    def __eq__(self, o):
        return self.v == o.v


def hash_partition(block, key, n: int) -> List[Block]:
    acc = BlockAccessor.for_block(block)
    buckets: List[List[int]] = [[] for _ in range(n)]
    for i, r in enumerate(acc.iter_rows()):
        buckets[stable_hash(_key_of(r, key)) % n].append(i)
    return [acc.take(b) if b else acc.slice(0, 0) for b in buckets]


def stable_hash(v) -> int:
    """Process-independent hash (Python's str hash is salted per process)."""
    import zlib

    if isinstance(v, np.generic):
        v = v.item()
    if isinstance(v, bool) or isinstance(v, int):
        return int(v) & 0x7FFFFFFFFFFFFFFF
    if isinstance(v, float):
        return hash(v) & 0x7FFFFFFFFFFFFFFF
    if isinstance(v, str):
        return zlib.crc32(v.encode())
    if isinstance(v, bytes):
        return zlib.crc32(v)
    if isinstance(v, tuple):
        h = 17
        for x in v:
            h = (h * 1000003 + stable_hash(x)) & 0x7FFFFFFFFFFFFFFF
        return h
    return zlib.crc32(repr(v).encode())


def random_split_block(block, n: int, seed: Optional[int]) -> List[Block]:
    acc = BlockAccessor.for_block(block)
    rng = random.Random(seed)
    assign: List[List[int]] = [[] for _ in range(n)]
    for i in range(acc.num_rows()):
        assign[rng.randrange(n)].append(i)
    return [acc.take(a) if a else acc.slice(0, 0) for a in assign]
