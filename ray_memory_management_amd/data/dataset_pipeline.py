"""DatasetPipeline: a (possibly infinite) sequence of Dataset windows processed in a pipelined
fashion. Parity: reference python/ray/data/dataset_pipeline.py (repeat / window, per-window
transforms map/map_batches/flat_map/filter/random_shuffle_each_window/repartition_each_window/
sort_each_window, foreach_window, iter_rows/iter_batches/iter_torch_batches, iter_epochs,
iter_datasets, split, take, show, count, sum, schema, stats).

Pipelining: the window after the one being consumed is produced (its transforms submitted) as
soon as consumption of the current one starts, so producing window i+1 overlaps with consuming i.
"""
from __future__ import annotations

import itertools
from typing import Any, Callable, Iterator, List, Optional


class DatasetPipeline:
    def __init__(self, base_iterable, stages: Optional[List[Callable]] = None, length=None,
                 epoch_len: Optional[int] = None):
        self._base = base_iterable        # iterable of zero-arg callables -> Dataset
        self._stages = list(stages or [])
        self._length = length
        self._epoch_len = epoch_len
        self._consumed = False

    def _with(self, fn) -> "DatasetPipeline":
        if self._consumed:
            raise RuntimeError("Pipeline cannot be read multiple times.")
        return DatasetPipeline(self._base, self._stages + [fn], self._length, self._epoch_len)

    def iter_datasets(self) -> Iterator:
        if self._consumed:
            raise RuntimeError("Pipeline cannot be read multiple times.")
        self._consumed = True
        stages = self._stages

        def make(w):
            ds = w()
            for st in stages:
                ds = st(ds)
            return ds

        it = iter(self._base)
        try:
            nxt = make(next(it))
        except StopIteration:
            return
        for w in it:
            cur, nxt = nxt, make(w)  # next window's tasks are in flight while `cur` is consumed
            yield cur
        yield nxt

    # ---- per-window transforms
    def map(self, fn, **kw):
        return self._with(lambda ds: ds.map(fn, **kw))

    def map_batches(self, fn, **kw):
        return self._with(lambda ds: ds.map_batches(fn, **kw))

    def flat_map(self, fn, **kw):
        return self._with(lambda ds: ds.flat_map(fn, **kw))

    def filter(self, fn, **kw):
        return self._with(lambda ds: ds.filter(fn, **kw))

    def add_column(self, col, fn, **kw):
        return self._with(lambda ds: ds.add_column(col, fn, **kw))

    def drop_columns(self, cols, **kw):
        return self._with(lambda ds: ds.drop_columns(cols, **kw))

    def random_shuffle_each_window(self, **kw):
        return self._with(lambda ds: ds.random_shuffle(**kw))

    def randomize_block_order_each_window(self, **kw):
        return self._with(lambda ds: ds.randomize_block_order(**kw))

    def repartition_each_window(self, num_blocks: int, shuffle: bool = False):
        return self._with(lambda ds: ds.repartition(num_blocks, shuffle=shuffle))

    def sort_each_window(self, key=None, descending=False):
        return self._with(lambda ds: ds.sort(key, descending))

    def foreach_window(self, fn: Callable) -> "DatasetPipeline":
        return self._with(fn)

    def rewindow(self, *, blocks_per_window: int, preserve_epoch: bool = True) -> "DatasetPipeline":
        parent = self

        def gen():
            from ray_memory_management_amd.data.dataset import Dataset, ExecutionPlan

            buf_b, buf_m = [], []
            for ds in parent.iter_datasets():
                buf_b += ds._blocks()
                buf_m += ds._metas()
                while len(buf_b) >= blocks_per_window:
                    b, m = buf_b[:blocks_per_window], buf_m[:blocks_per_window]
                    buf_b, buf_m = buf_b[blocks_per_window:], buf_m[blocks_per_window:]
                    yield lambda b=b, m=m: Dataset(ExecutionPlan(b, m))
            if buf_b:
                yield lambda b=buf_b, m=buf_m: Dataset(ExecutionPlan(b, m))

        return DatasetPipeline(gen())

    def repeat(self, times: Optional[int] = None) -> "DatasetPipeline":
        if self._length == float("inf"):
            raise ValueError("Cannot repeat a pipeline that is already infinite.")
        windows = list(self._base)
        stages = self._stages
        n = len(windows)

        def gen():
            for _ in (range(times) if times is not None else itertools.count()):
                yield from windows

        return DatasetPipeline(gen(), stages, length=(n * times) if times is not None else float("inf"),
                               epoch_len=n)

    # ---- consumption
    def iter_rows(self, *, prefetch_blocks: int = 0):
        for ds in self.iter_datasets():
            yield from ds.iter_rows(prefetch_blocks=prefetch_blocks)

    def iter_batches(self, *, batch_size: Optional[int] = 256, batch_format: str = "native",
                     drop_last: bool = False, prefetch_blocks: int = 0, **kw):
        for ds in self.iter_datasets():
            yield from ds.iter_batches(batch_size=batch_size, batch_format=batch_format, drop_last=drop_last,
                                       prefetch_blocks=prefetch_blocks, **kw)

    def iter_torch_batches(self, **kw):
        for ds in self.iter_datasets():
            yield from ds.iter_torch_batches(**kw)

    def iter_epochs(self, max_epoch: int = -1) -> Iterator["DatasetPipeline"]:
        if self._epoch_len is None:
            raise ValueError("iter_epochs() requires a pipeline created with repeat()")
        it = self.iter_datasets()
        e = 0
        while max_epoch < 0 or e < max_epoch:
            chunk = list(itertools.islice(it, self._epoch_len))
            if not chunk:
                return
            yield DatasetPipeline([lambda d=d: d for d in chunk], length=len(chunk))
            e += 1

    def split(self, n: int, *, equal: bool = False, locality_hints=None) -> List["DatasetPipeline"]:
        """n pipelines over shards of each window (materialised window by window)."""
        shards: List[List[Callable]] = [[] for _ in range(n)]
        for ds in self.iter_datasets():
            for i, part in enumerate(ds.split(n, equal=equal, locality_hints=locality_hints)):
                shards[i].append(lambda p=part: p)
        return [DatasetPipeline(s, length=len(s)) for s in shards]

    def split_at_indices(self, indices: List[int]) -> List["DatasetPipeline"]:
        """len(indices)+1 pipelines over the index-split shards of every window."""
        shards: List[List[Callable]] = [[] for _ in range(len(indices) + 1)]
        for ds in self.iter_datasets():
            for i, part in enumerate(ds.split_at_indices(indices)):
                shards[i].append(lambda p=part: p)
        return [DatasetPipeline(s, length=len(s)) for s in shards]

    @staticmethod
    def from_iterable(iterable) -> "DatasetPipeline":
        """A pipeline over zero-arg callables that each produce one window's Dataset."""
        items = list(iterable)
        return DatasetPipeline(items, length=len(items))

    def take(self, limit: int = 20) -> List[Any]:
        return list(itertools.islice(self.iter_rows(), limit))

    def take_all(self, limit: Optional[int] = None) -> List[Any]:
        if self._length == float("inf"):
            raise ValueError("Cannot take_all of a pipeline of infinite length.")
        out = list(self.iter_rows())
        if limit is not None and len(out) > limit:
            raise ValueError(f"The pipeline has more than the given limit of {limit} records.")
        return out

    def show_windows(self, limit_per_dataset: int = 10) -> None:
        for i, ds in enumerate(self.iter_datasets()):
            print(f"=== Window {i} ===")
            for r in ds.take(limit_per_dataset):
                print(r)

    def to_torch(self, **kw):
        """An iterable over the torch batches of every window (reference DatasetPipeline.to_torch)."""
        pipe = self

        class _It:
            def __iter__(self_inner):
                for ds in pipe.iter_datasets():
                    yield from ds.to_torch(**kw)

        return _It()

    def _write_each(self, method: str, path: str, **kw):
        import os

        for i, ds in enumerate(self.iter_datasets()):
            getattr(ds, method)(os.path.join(path, f"window_{i:06d}"), **kw)

    def write_json(self, path: str, **kw):
        self._write_each("write_json", path, **kw)

    def write_csv(self, path: str, **kw):
        self._write_each("write_csv", path, **kw)

    def write_parquet(self, path: str, **kw):
        self._write_each("write_parquet", path, **kw)

    def write_datasource(self, datasource, **kw):
        for ds in self.iter_datasets():
            ds.write_datasource(datasource, **kw)

    def show(self, limit: int = 20) -> None:
        for r in self.take(limit):
            print(r)

    def count(self) -> int:
        if self._length == float("inf"):
            raise ValueError("Cannot count a pipeline of infinite length.")
        return sum(ds.count() for ds in self.iter_datasets())

    def sum(self):
        if self._length == float("inf"):
            raise ValueError("Cannot sum a pipeline of infinite length.")
        return sum((ds.sum() or 0) for ds in self.iter_datasets())

    def schema(self):
        for ds in self.iter_datasets():
            return ds.schema()

    def stats(self) -> str:
        return f"DatasetPipeline(num_stages={len(self._stages)}, length={self._length})"

    def __repr__(self):
        return f"DatasetPipeline(num_windows={self._length}, num_stages={len(self._stages) + 1})"
