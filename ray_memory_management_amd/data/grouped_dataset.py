"""groupby(key).aggregate / count / sum / min / max / mean / std / map_groups.

Parity: reference python/ray/data/grouped_dataset.py. Sort-based: range-partition the dataset on
the key (sampled boundaries, like sort), then each partition task walks its sorted rows and
folds every group with the AggregateFns; output is sorted by key (as in the reference).
"""
from __future__ import annotations

import itertools
from typing import Any, Callable, List, Optional

import ray_memory_management_amd as ray
from ray_memory_management_amd.data import _internal as I
from ray_memory_management_amd.data.aggregate import AggregateFn, Count, Max, Mean, Min, Std, Sum
from ray_memory_management_amd.data.block import BlockAccessor, BlockBuilder, _key_of, concat_blocks


def _agg_out_row(key_name, key, names, values, simple: bool):
    if key_name is None:
        return tuple(values) if simple else dict(zip(names, values))
    if simple:
        return (key,) + tuple(values)
    return {key_name if isinstance(key_name, str) else "key": key, **dict(zip(names, values))}


@ray.remote
def _aggregate_partition(key, aggs, *parts):
    block = concat_blocks(list(parts))
    acc = BlockAccessor.for_block(block)
    simple = isinstance(block, list)
    rows = list(acc.iter_rows())
    names = [a.name for a in aggs]
    b = BlockBuilder()
    if key is None:  # global aggregate: one partial row
        if rows or True:
            vals = [a.accumulate_rows(None, rows) for a in aggs]
            b.add(("__partial__", vals))
        out = b.build()
        return out, BlockAccessor.for_block(out).get_metadata()
    for k, grp in itertools.groupby(rows, key=lambda r: _key_of(r, key)):
        grp = list(grp)
        vals = [a.finalize(a.accumulate_rows(k, grp)) for a in aggs]
        b.add(_agg_out_row(key if isinstance(key, str) else None, k, names, vals, simple or callable(key)))
    out = b.build() if b.num_rows() else []
    return out, BlockAccessor.for_block(out).get_metadata()


@ray.remote
def _map_groups_partition(key, fn, batch_format, *parts):
    block = concat_blocks(list(parts))
    acc = BlockAccessor.for_block(block)
    from ray_memory_management_amd.data.block import batch_to_block

    n = acc.num_rows()
    outs = []
    if n:
        keys = [_key_of(r, key) for r in acc.iter_rows()]
        start = 0
        for i in range(1, n + 1):
            if i == n or keys[i] != keys[start]:
                batch = BlockAccessor.for_block(acc.slice(start, i)).to_batch(batch_format)
                outs.append(batch_to_block(fn(batch)))
                start = i
    out = concat_blocks(outs) if outs else acc.slice(0, 0)
    return out, BlockAccessor.for_block(out).get_metadata()


class GroupedDataset:
    def __init__(self, dataset, key):
        self._dataset = dataset
        self._key = key

    def __repr__(self):
        return f"GroupedDataset(dataset={self._dataset}, key={self._key!r})"

    def _partitions(self):
        blocks = self._dataset._blocks()
        if self._key is None:
            return [[b] for b in blocks]
        num_out = max(len(blocks), 1)
        boundaries = I.sample_boundaries(blocks, self._key, num_out, False)
        n_parts = len(boundaries) + 1
        parts = []
        for b in blocks:
            r = I._sort_partition.options(num_returns=n_parts).remote(b, self._key, boundaries, False)
            parts.append(r if n_parts > 1 else [r])
        return [[p[j] for p in parts] for j in range(n_parts)]

    def aggregate(self, *aggs: AggregateFn):
        from ray_memory_management_amd.data.dataset import Dataset, ExecutionPlan

        if not aggs:
            raise ValueError("Aggregate requires at least one aggregation")
        parts = self._partitions()
        out_b, out_m = [], []
        for p in parts:
            rb, rm = _aggregate_partition.options(num_returns=2).remote(self._key, list(aggs), *p)
            out_b.append(rb)
            out_m.append(rm)
        if self._key is None:  # merge the per-block partials on the driver
            partials = [row[1] for blk in ray.get(out_b) for row in blk]
            if not partials or self._dataset.count() == 0:
                return Dataset(ExecutionPlan([ray.put([])], [BlockAccessor.for_block([]).get_metadata()]))
            vals = partials[0]
            for pv in partials[1:]:
                vals = [a.merge(x, y) for a, x, y in zip(aggs, vals, pv)]
            fin = [a.finalize(v) for a, v in zip(aggs, vals)]
            simple = isinstance(ray.get(self._dataset._blocks()[0]), list)
            row = tuple(fin) if simple else dict(zip([a.name for a in aggs], fin))
            blk = [row] if simple else BlockBuilder()
            if not simple:
                blk.add(row)
                blk = blk.build()
            return Dataset(ExecutionPlan([ray.put(blk)], [BlockAccessor.for_block(blk).get_metadata()]))
        return Dataset(ExecutionPlan(out_b, out_m))

    def map_groups(self, fn: Callable, *, compute=None, batch_format: str = "native", **ray_remote_args):
        from ray_memory_management_amd.data.dataset import Dataset, ExecutionPlan

        out_b, out_m = [], []
        for p in self._partitions():
            rb, rm = _map_groups_partition.options(num_returns=2, **ray_remote_args).remote(
                self._key, fn, batch_format, *p)
            out_b.append(rb)
            out_m.append(rm)
        return Dataset(ExecutionPlan(out_b, out_m))

    def _agg(self, cls, on, ignore_nulls=True, **kw):
        if isinstance(on, list):
            return self.aggregate(*[cls(c, ignore_nulls=ignore_nulls, **kw) for c in on])
        return self.aggregate(cls(on, ignore_nulls=ignore_nulls, **kw))

    def count(self):
        return self.aggregate(Count())

    def sum(self, on=None, ignore_nulls: bool = True):
        return self._agg(Sum, on, ignore_nulls)

    def min(self, on=None, ignore_nulls: bool = True):
        return self._agg(Min, on, ignore_nulls)

    def max(self, on=None, ignore_nulls: bool = True):
        return self._agg(Max, on, ignore_nulls)

    def mean(self, on=None, ignore_nulls: bool = True):
        return self._agg(Mean, on, ignore_nulls)

    def std(self, on=None, ddof: int = 1, ignore_nulls: bool = True):
        return self._agg(Std, on, ignore_nulls, ddof=ddof)
