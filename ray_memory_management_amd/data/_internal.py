"""Execution internals for Dataset: per-block remote tasks, stage fusion, actor-pool compute,
all-to-all exchanges (shuffle / sort / repartition / groupby).

Parity: reference python/ray/data/_internal/{plan.py (ExecutionPlan, stage fusion),
compute.py (TaskPoolStrategy / ActorPoolStrategy), shuffle.py + push_based_shuffle.py,
sort.py (sample boundaries → range partition → merge), fast_repartition.py, stats.py}.

Every block task returns TWO objects — the block and its BlockMetadata — so the driver learns
row counts / sizes / schemas without fetching blocks (`num_returns=2`).
"""
from __future__ import annotations

import time
from typing import Any, Callable, List, Optional, Sequence

import numpy as np

import ray_memory_management_amd as ray
from ray_memory_management_amd.data.block import (BlockAccessor, BlockBuilder, BlockMetadata, batch_to_block,
                                                  concat_blocks, merge_sorted_blocks, partition_by_boundaries,
                                                  random_split_block)

# ---------------------------------------------------------------------- compute strategies


class ComputeStrategy:
    pass


class TaskPoolStrategy(ComputeStrategy):
    def __repr__(self):
        return "TaskPoolStrategy()"


class ActorPoolStrategy(ComputeStrategy):
    """Run a stage on an autoscaling pool of actors (reference compute.py ActorPoolStrategy)."""

    def __init__(self, min_size: int = 1, max_size: Optional[int] = None, max_tasks_in_flight_per_actor: int = 2):
        if min_size < 1:
            raise ValueError("min_size must be > 1", min_size)
        if max_size is not None and min_size > max_size:
            raise ValueError("min_size must be <= max_size", min_size, max_size)
        self.min_size = min_size
        self.max_size = max_size or min_size
        self.max_tasks_in_flight_per_actor = max_tasks_in_flight_per_actor

    def __repr__(self):
        return f"ActorPoolStrategy(min_size={self.min_size}, max_size={self.max_size})"


def get_compute(compute) -> ComputeStrategy:
    if compute is None or compute == "tasks":
        return TaskPoolStrategy()
    if compute == "actors":
        return ActorPoolStrategy()
    if isinstance(compute, ComputeStrategy):
        return compute
    raise ValueError(f"compute must be 'tasks', 'actors' or a ComputeStrategy, got {compute!r}")


# ---------------------------------------------------------------------- block transforms


class BlockTransform:
    """One one-to-one stage: a picklable block -> block function."""

    def __init__(self, kind: str, fn, batch_size=None, batch_format="native", fn_args=(), fn_kwargs=None,
                 fn_constructor_args=(), fn_constructor_kwargs=None, name=None):
        self.kind, self.fn, self.batch_size, self.batch_format = kind, fn, batch_size, batch_format
        self.fn_args, self.fn_kwargs = tuple(fn_args or ()), dict(fn_kwargs or {})
        self.ctor_args, self.ctor_kwargs = tuple(fn_constructor_args or ()), dict(fn_constructor_kwargs or {})
        self.name = name or kind
        self._inst = None

    def _callable(self):
        if isinstance(self.fn, type):  # callable class: one instance per worker/actor
            if self._inst is None:
                self._inst = self.fn(*self.ctor_args, **self.ctor_kwargs)
            return self._inst
        return self.fn

    def __call__(self, block):
        fn = self._callable()
        acc = BlockAccessor.for_block(block)
        a, kw = self.fn_args, self.fn_kwargs
        if self.kind == "map":
            b = BlockBuilder()
            for r in acc.iter_rows():
                b.add(fn(r, *a, **kw))
            return b.build() if b.num_rows() else acc.slice(0, 0)
        if self.kind == "flat_map":
            b = BlockBuilder()
            for r in acc.iter_rows():
                for x in fn(r, *a, **kw):
                    b.add(x)
            return b.build() if b.num_rows() else acc.slice(0, 0)
        if self.kind == "filter":
            keep = [i for i, r in enumerate(acc.iter_rows()) if fn(r, *a, **kw)]
            return acc.take(keep)
        if self.kind == "map_batches":
            n = acc.num_rows()
            bs = n if self.batch_size is None else max(int(self.batch_size), 1)
            outs = []
            for s in range(0, max(n, 1), max(bs, 1)):
                if n == 0:
                    break
                batch = BlockAccessor.for_block(acc.slice(s, min(s + bs, n))).to_batch(self.batch_format)
                outs.append(batch_to_block(fn(batch, *a, **kw)))
            return concat_blocks(outs) if outs else acc.slice(0, 0)
        if self.kind == "block":  # raw block -> block
            return fn(block, *a, **kw)
        raise ValueError(self.kind)


def _exec_transforms(block, transforms: Sequence[BlockTransform]):
    t0 = time.perf_counter()
    for t in transforms:
        block = t(block)
    meta = BlockAccessor.for_block(block).get_metadata(exec_stats={"wall_s": time.perf_counter() - t0})
    return block, meta


@ray.remote
def _stage_task(block, transforms):
    return _exec_transforms(block, transforms)


class _BlockWorker:
    def __init__(self, transforms):
        self.transforms = transforms

    def ready(self):
        return True

    def process(self, block):
        return _exec_transforms(block, self.transforms)


def run_transforms(blocks: List[Any], transforms: List[BlockTransform], compute: ComputeStrategy,
                   remote_args: dict):
    """Apply fused transforms to every block. Returns (block_refs, meta_refs)."""
    remote_args = dict(remote_args or {})
    if isinstance(compute, TaskPoolStrategy):
        out_b, out_m = [], []
        task = _stage_task.options(num_returns=2, **remote_args)
        for b in blocks:
            rb, rm = task.remote(b, transforms)
            out_b.append(rb)
            out_m.append(rm)
        return out_b, out_m
    # actor pool: start min_size actors, grow toward max_size while work is queued
    cls = ray.remote(_BlockWorker).options(**remote_args)
    actors = [cls.remote(transforms) for _ in range(compute.min_size)]
    ray.get([a.ready.remote() for a in actors])
    per = compute.max_tasks_in_flight_per_actor
    results: List[Any] = [None] * len(blocks)
    inflight = {}
    load = {id(a): 0 for a in actors}
    nxt = 0
    while nxt < len(blocks) or inflight:
        while nxt < len(blocks):
            free = [a for a in actors if load[id(a)] < per]
            if not free and len(actors) < compute.max_size:
                a = cls.remote(transforms)
                actors.append(a)
                load[id(a)] = 0
                free = [a]
            if not free:
                break
            a = min(free, key=lambda x: load[id(x)])
            rb, rm = a.process.options(num_returns=2).remote(blocks[nxt])
            inflight[rm] = (nxt, a, rb)
            load[id(a)] += 1
            nxt += 1
        ready, _ = ray.wait(list(inflight), num_returns=1)
        for r in ready:
            i, a, rb = inflight.pop(r)
            load[id(a)] -= 1
            results[i] = (rb, r)
    for a in actors:
        ray.kill(a)
    return [r[0] for r in results], [r[1] for r in results]


# ---------------------------------------------------------------------- all-to-all exchanges
@ray.remote
def _split_random(block, n, seed):
    parts = random_split_block(block, n, seed)
    return tuple(parts) if n > 1 else parts[0]


@ray.remote
def _concat_shuffle(seed, *parts):
    b = concat_blocks(list(parts))
    out = BlockAccessor.for_block(b).random_shuffle(seed)
    return out, BlockAccessor.for_block(out).get_metadata()


@ray.remote
def _merge_parts(*parts):
    """Push-based shuffle merge stage: pre-combine one reducer's parts from a round of mappers."""
    return concat_blocks(list(parts))


def shuffle_blocks(blocks, num_out: int, seed: Optional[int], push_based: bool = False,
                   merge_factor: int = 4):
    """Random shuffle: map (split each block randomly into num_out parts) → [merge] → reduce."""
    m = len(blocks)
    if m == 0:
        return [], []
    parts = []
    for i, b in enumerate(blocks):
        r = _split_random.options(num_returns=num_out).remote(b, num_out, None if seed is None else seed + i)
        parts.append(r if num_out > 1 else [r])
    if push_based and m > merge_factor:
        # merge rounds: combine every `merge_factor` mappers' outputs per reducer so reducers
        # read O(m / merge_factor) objects (reference push_based_shuffle.py)
        merged = []
        for g in range(0, m, merge_factor):
            grp = parts[g:g + merge_factor]
            merged.append([_merge_parts.remote(*[p[j] for p in grp]) for j in range(num_out)])
        parts = merged
    out_b, out_m = [], []
    for j in range(num_out):
        rb, rm = _concat_shuffle.options(num_returns=2).remote(None if seed is None else seed * 7919 + j,
                                                               *[p[j] for p in parts])
        out_b.append(rb)
        out_m.append(rm)
    return out_b, out_m


@ray.remote
def _sample_block(block, n, key):
    return BlockAccessor.for_block(block).sample(n, key)


@ray.remote
def _sort_partition(block, key, boundaries, descending):
    acc = BlockAccessor.for_block(block)
    s = acc.sort(key, descending) if acc.num_rows() else block
    parts = partition_by_boundaries(s, key, boundaries, descending)
    return tuple(parts) if len(parts) > 1 else parts[0]


@ray.remote
def _merge_sorted(key, descending, *parts):
    b = merge_sorted_blocks(list(parts), key, descending)
    return b, BlockAccessor.for_block(b).get_metadata()


def sample_boundaries(blocks, key, num_out: int, descending: bool) -> list:
    n_samples = max(10, 2 * num_out)
    samples = [s for lst in ray.get([_sample_block.remote(b, n_samples, key) for b in blocks]) for s in lst]
    if not samples:
        return []
    samples.sort()
    qs = [samples[min(len(samples) - 1, int(len(samples) * i / num_out))] for i in range(1, num_out)]
    if descending:
        qs = qs[::-1]
    return qs


def sort_blocks(blocks, key, descending: bool):
    if not blocks:
        return [], []
    num_out = len(blocks)
    boundaries = sample_boundaries(blocks, key, num_out, descending)
    n_parts = len(boundaries) + 1
    parts = []
    for b in blocks:
        r = _sort_partition.options(num_returns=n_parts).remote(b, key, boundaries, descending)
        parts.append(r if n_parts > 1 else [r])
    out_b, out_m = [], []
    for j in range(n_parts):
        rb, rm = _merge_sorted.options(num_returns=2).remote(key, descending, *[p[j] for p in parts])
        out_b.append(rb)
        out_m.append(rm)
    return out_b, out_m


@ray.remote
def _slice_block(block, start, end):
    return BlockAccessor.for_block(block).slice(start, end, copy=True)


@ray.remote
def _concat_with_meta(*parts):
    b = concat_blocks(list(parts))
    return b, BlockAccessor.for_block(b).get_metadata()


def repartition_blocks(blocks, counts: List[int], num_out: int, split_sizes: Optional[List[int]] = None):
    """Split/combine blocks (order preserving) into num_out blocks of near-equal rows, or into
    blocks of exactly `split_sizes` rows."""
    total = sum(counts)
    if split_sizes is None:
        base, extra = divmod(total, max(num_out, 1))
        split_sizes = [base + (1 if i < extra else 0) for i in range(num_out)]
    out_b, out_m = [], []
    bi, off = 0, 0  # cursor: block index, row offset inside it
    for size in split_sizes:
        pieces = []
        need = size
        while need > 0 and bi < len(blocks):
            avail = counts[bi] - off
            take = min(avail, need)
            if take == counts[bi] and off == 0:
                pieces.append(blocks[bi])
            elif take > 0:
                pieces.append(_slice_block.remote(blocks[bi], off, off + take))
            off += take
            need -= take
            if off >= counts[bi]:
                bi += 1
                off = 0
        if not pieces and blocks:
            pieces = [_slice_block.remote(blocks[0], 0, 0)]
        rb, rm = _concat_with_meta.options(num_returns=2).remote(*pieces)
        out_b.append(rb)
        out_m.append(rm)
    return out_b, out_m


# ---------------------------------------------------------------------- stats
class DatasetStats:
    def __init__(self, parent: Optional["DatasetStats"] = None):
        self.stages: List[tuple] = list(parent.stages) if parent else []

    def record(self, name: str, num_blocks: int, wall_s: float):
        self.stages.append((name, num_blocks, wall_s))

    def summary_string(self) -> str:
        lines = []
        for i, (name, nb, t) in enumerate(self.stages):
            lines.append(f"Stage {i} {name}: {nb} blocks executed in {t:.3f}s")
        return "\n".join(lines) if lines else "No stages executed"
