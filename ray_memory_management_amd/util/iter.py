"""Parallel iterators over actor-held shards.

Parity: reference python/ray/util/iter.py — from_items / from_range / from_iterators /
from_actors, ParallelIterator (for_each, filter, batch, flatten, combine, local_shuffle,
repartition, gather_sync, gather_async, batch_across_shards, union, select_shards, num_shards,
shards, get_shard, take, show) and LocalIterator (for_each, filter, batch, flatten, combine,
shuffle, take, show, union, duplicate).

Design: each shard is an actor holding a generator factory plus a list of per-item transforms
that the actor applies itself (so for_each/filter run next to the data); the driver pulls items
in small batches (``fetch_batch``) to amortise round trips, either in lock-step over shards
(gather_sync) or with one request in flight per shard, harvested in completion order
(gather_async).
"""
from __future__ import annotations

import collections
import itertools
import random
import threading
from typing import Any, Callable, Iterable, List, Optional

import ray_memory_management_amd as ray
from ray_memory_management_amd.util.iter_metrics import MetricsContext, SharedMetrics

_NEXT_BATCH = 32


# ---------------------------------------------------------------------- transforms (picklable)
def _apply(transforms, it):
    for kind, fn in transforms:
        if kind == "map":
            it = map(fn, it)
        elif kind == "filter":
            it = filter(fn, it)
        elif kind == "batch":
            it = _batched(it, fn)
        elif kind == "flatten":
            it = (y for x in it for y in x)
        elif kind == "shuffle":
            it = _shuffled(it, *fn)
        elif kind == "combine":
            it = (y for x in it for y in fn(x))
    return it


def _batched(it, n):
    buf = []
    for x in it:
        buf.append(x)
        if len(buf) >= n:
            yield buf
            buf = []
    if buf:
        yield buf


def _shuffled(it, buffer_size, seed):
    rng = random.Random(seed)
    buf = []
    for x in it:
        buf.append(x)
        if len(buf) >= buffer_size:
            yield buf.pop(rng.randrange(len(buf)))
    rng.shuffle(buf)
    yield from buf


class ParallelIteratorWorker:
    """Actor body for one shard (reference iter.py ParallelIteratorWorker)."""

    def __init__(self, item_generator, repeat: bool):
        self.item_generator = item_generator
        self.repeat = repeat
        self.local_it = None
        self.transforms = None

    def _base(self):
        g = self.item_generator
        while True:
            yield from (g() if callable(g) else g)
            if not self.repeat:
                return

    def par_iter_init(self, transforms):
        self.transforms = transforms
        self.local_it = _apply(transforms, self._base())

    def par_iter_next_batch(self, n):
        if self.local_it is None:
            raise ValueError("par_iter_init() must be called first")
        out = list(itertools.islice(self.local_it, n))
        return out, len(out) < n  # (items, exhausted)

    def par_iter_slice(self, step, start, transforms):
        it = _apply(transforms, self._base())
        return list(itertools.islice(it, start, None, step))


_Worker = None


def _worker_cls():
    global _Worker
    if _Worker is None:
        _Worker = ray.remote(num_cpus=0)(ParallelIteratorWorker)
    return _Worker


# ---------------------------------------------------------------------- constructors
def from_items(items: List[Any], num_shards: int = 2, repeat: bool = False) -> "ParallelIterator":
    shards = [[] for _ in range(num_shards)]
    for i, item in enumerate(items):
        shards[i % num_shards].append(item)
    name = f"from_items[{type(items[0]).__name__ if items else 'None'}, {len(items)}, shards={num_shards}" \
           f"{', repeat=True' if repeat else ''}]"
    return from_iterators(shards, repeat=repeat, name=name)


class _Range:
    def __init__(self, a, b):
        self.a, self.b = a, b

    def __call__(self):
        return iter(range(self.a, self.b))


def from_range(n: int, num_shards: int = 2, repeat: bool = False) -> "ParallelIterator":
    gens = []
    for i in range(num_shards):
        start = i * (n // num_shards)
        end = n if i == num_shards - 1 else (i + 1) * (n // num_shards)
        gens.append(_Range(start, end))
    return from_iterators(gens, repeat=repeat, name=f"from_range[{n}, shards={num_shards}"
                                                    f"{', repeat=True' if repeat else ''}]")


def from_iterators(generators: List[Iterable], repeat: bool = False, name=None) -> "ParallelIterator":
    gens = [list(g) if not callable(g) and not isinstance(g, (list, tuple)) else g for g in generators]
    if name is None:
        name = f"from_iterators[shards={len(gens)}{', repeat=True' if repeat else ''}]"
    actors = [_worker_cls().remote(g, repeat) for g in gens]
    return from_actors(actors, name=name)


def from_actors(actors: List[Any], name=None) -> "ParallelIterator":
    return ParallelIterator([_ActorSet(actors, [])], name or f"from_actors[shards={len(actors)}]", [])


class _ActorSet:
    def __init__(self, actors, transforms):
        self.actors = actors
        self.transforms = transforms

    def init(self):
        ray.get([a.par_iter_init.remote(self.transforms) for a in self.actors])

    def with_transform(self, t):
        return _ActorSet(self.actors, self.transforms + [t])


class ParallelIterator:
    def __init__(self, actor_sets: List[_ActorSet], name: str, parent_iterators: list):
        self.actor_sets = actor_sets
        self.name = name
        self.parent_iterators = parent_iterators

    def __iter__(self):
        raise TypeError("You must use it.gather_sync() or it.gather_async() to iterate over the results "
                        "of a ParallelIterator.")

    def __str__(self):
        return repr(self)

    def __repr__(self):
        return f"ParallelIterator[{self.name}]"

    def _with(self, t, label):
        return ParallelIterator([s.with_transform(t) for s in self.actor_sets], self.name + label,
                                self.parent_iterators)

    # transforms run inside the shard actors
    def for_each(self, fn: Callable, max_concurrency: int = 1, resources=None) -> "ParallelIterator":
        return self._with(("map", fn), ".for_each()")

    def filter(self, fn: Callable) -> "ParallelIterator":
        return self._with(("filter", fn), ".filter()")

    def batch(self, n: int) -> "ParallelIterator":
        return self._with(("batch", n), f".batch({n})")

    def flatten(self) -> "ParallelIterator":
        return self._with(("flatten", None), ".flatten()")

    def combine(self, fn: Callable) -> "ParallelIterator":
        return self._with(("combine", fn), ".combine()")

    def local_shuffle(self, shuffle_buffer_size: int, seed: Optional[int] = None) -> "ParallelIterator":
        return self._with(("shuffle", (shuffle_buffer_size, seed)),
                          f".local_shuffle(shuffle_buffer_size={shuffle_buffer_size}, seed={seed})")

    def repartition(self, num_partitions: int, batch_ms: int = 0) -> "ParallelIterator":
        """Round-robin items of all shards into num_partitions new shards (materialises)."""
        it = from_items(list(self.gather_sync()), num_shards=num_partitions)
        it.name = self.name + f".repartition[num_partitions={num_partitions}]"
        return it

    def union(self, other: "ParallelIterator") -> "ParallelIterator":
        if not isinstance(other, ParallelIterator):
            raise TypeError(f"other must be of type ParallelIterator, got {type(other)}")
        return ParallelIterator(self.actor_sets + other.actor_sets, f"ParallelUnion[{self}, {other}]",
                                self.parent_iterators + other.parent_iterators)

    def num_shards(self) -> int:
        return sum(len(s.actors) for s in self.actor_sets)

    def shards(self) -> List["LocalIterator"]:
        return [self.get_shard(i) for i in range(self.num_shards())]

    def select_shards(self, shards_to_keep: List[int]) -> "ParallelIterator":
        sets, i = [], 0
        for s in self.actor_sets:
            keep = [a for j, a in enumerate(s.actors) if i + j in shards_to_keep]
            i += len(s.actors)
            if keep:
                sets.append(_ActorSet(keep, s.transforms))
        return ParallelIterator(sets, self.name + f".select_shards({len(shards_to_keep)} total)", self.parent_iterators)

    def _flat_actors(self):
        return [(a, s.transforms) for s in self.actor_sets for a in s.actors]

    def get_shard(self, shard_index: int, batch_ms: int = 0, num_async: int = 1) -> "LocalIterator":
        a, tr = self._flat_actors()[shard_index]

        def gen():
            ray.get(a.par_iter_init.remote(tr))
            while True:
                items, done = ray.get(a.par_iter_next_batch.remote(_NEXT_BATCH))
                yield from items
                if done:
                    return

        return LocalIterator(gen, name=self.name + f".shard[{shard_index}]")

    def gather_sync(self) -> "LocalIterator":
        """Round-robin over shards, one item from each in turn (deterministic order)."""

        def gen():
            for s in self.actor_sets:
                s.init()
            actors = [a for a, _ in self._flat_actors()]
            bufs = [collections.deque() for _ in actors]
            done = [False] * len(actors)
            while True:
                live = False
                for i, a in enumerate(actors):
                    if not bufs[i] and not done[i]:
                        items, done[i] = ray.get(a.par_iter_next_batch.remote(_NEXT_BATCH))
                        bufs[i].extend(items)
                    if bufs[i]:
                        live = True
                        yield bufs[i].popleft()
                if not live:
                    return

        return LocalIterator(gen, name=self.name + ".gather_sync()")

    def gather_async(self, batch_ms: int = 0, num_async: int = 1) -> "LocalIterator":
        """Items in completion order with `num_async` fetches in flight per shard."""
        if num_async < 1:
            raise ValueError("queue depth must be positive")

        def gen():
            for s in self.actor_sets:
                s.init()
            inflight = {}
            for a, _ in self._flat_actors():
                for _ in range(num_async):
                    inflight[a.par_iter_next_batch.remote(_NEXT_BATCH)] = a
            finished = set()
            while inflight:
                ready, _ = ray.wait(list(inflight), num_returns=1)
                a = inflight.pop(ready[0])
                items, done = ray.get(ready[0])
                for x in items:
                    stack = getattr(_metrics_tls, "stack", None)
                    if stack:  # the consumer's metrics: which shard produced this item
                        stack[-1].current_actor = a
                    yield x
                if done:
                    finished.add(id(a))
                elif id(a) not in finished:
                    inflight[a.par_iter_next_batch.remote(_NEXT_BATCH)] = a

        return LocalIterator(gen, name=self.name + ".gather_async()")

    def batch_across_shards(self) -> "LocalIterator":
        """One list per round holding the next item of every shard."""

        def gen():
            for s in self.actor_sets:
                s.init()
            actors = [a for a, _ in self._flat_actors()]
            while True:
                res = ray.get([a.par_iter_next_batch.remote(1) for a in actors])
                items = [r[0][0] for r in res if r[0]]
                if not items:
                    return
                yield items

        return LocalIterator(gen, name=self.name + ".batch_across_shards()")

    def take(self, n: int) -> List[Any]:
        return self.gather_sync().take(n)

    def show(self, n: int = 20):
        for i, x in enumerate(self.gather_sync()):
            if i >= n:
                break
            print(x)


_metrics_tls = threading.local()


class LocalIterator:
    """Driver-side iterator with lazy transforms (reference iter.py LocalIterator). Every operator of
    a chain shares one MetricsContext (util.iter_metrics), readable from inside the operators'
    functions through ``LocalIterator.get_metrics()``."""

    def __init__(self, base_iterator: Callable[[], Iterable], name: Optional[str] = None,
                 shared_metrics: Optional[SharedMetrics] = None):
        self.base_iterator = base_iterator
        self.built_iterator = None
        self.name = name or "LocalIterator"
        self.shared_metrics = shared_metrics or SharedMetrics()

    def _build(self):
        if self.built_iterator is None:
            self.built_iterator = iter(self.base_iterator())

    def __iter__(self):
        self._build()
        return self

    def __next__(self):
        self._build()
        stack = getattr(_metrics_tls, "stack", None)
        if stack is None:
            stack = _metrics_tls.stack = []
        stack.append(self.shared_metrics.get())
        try:
            return next(self.built_iterator)
        finally:
            stack.pop()

    @staticmethod
    def get_metrics() -> MetricsContext:
        """The metrics context of the iterator whose item is being computed (call it only from inside
        an operator function of a LocalIterator chain)."""
        stack = getattr(_metrics_tls, "stack", None)
        if not stack:
            raise ValueError("get_metrics() may only be called from inside a LocalIterator operator")
        return stack[-1]

    def __repr__(self):
        return f"LocalIterator[{self.name}]"

    def _chain(self, f, label):
        parent = self
        return LocalIterator(lambda: f(iter(parent)), self.name + label, shared_metrics=self.shared_metrics)

    def for_each(self, fn: Callable, max_concurrency: int = 1, resources=None) -> "LocalIterator":
        return self._chain(lambda it: map(fn, it), ".for_each()")

    def filter(self, fn: Callable) -> "LocalIterator":
        return self._chain(lambda it: filter(fn, it), ".filter()")

    def batch(self, n: int) -> "LocalIterator":
        return self._chain(lambda it: _batched(it, n), f".batch({n})")

    def flatten(self) -> "LocalIterator":
        return self._chain(lambda it: (y for x in it for y in x), ".flatten()")

    def combine(self, fn: Callable) -> "LocalIterator":
        return self._chain(lambda it: (y for x in it for y in fn(x)), ".combine()")

    def shuffle(self, shuffle_buffer_size: int, seed: Optional[int] = None) -> "LocalIterator":
        return self._chain(lambda it: _shuffled(it, shuffle_buffer_size, seed),
                           f".shuffle(shuffle_buffer_size={shuffle_buffer_size}, seed={seed})")

    def take(self, n: int) -> List[Any]:
        return list(itertools.islice(iter(self), n))

    def show(self, n: int = 20):
        for x in self.take(n):
            print(x)

    def union(self, *others: "LocalIterator", deterministic: bool = False, round_robin_weights=None):
        its = [self] + list(others)
        weights = round_robin_weights or [1] * len(its)

        def gen():
            live = [iter(i) for i in its]
            w = list(weights)
            while live:
                nxt_live, nxt_w = [], []
                for it, k in zip(live, w):
                    alive = True
                    n = 1 if k == "*" else k
                    for _ in range(n):
                        try:
                            yield next(it)
                        except StopIteration:
                            alive = False
                            break
                    if alive:
                        nxt_live.append(it)
                        nxt_w.append(k)
                live, w = nxt_live, nxt_w

        return LocalIterator(gen, f"LocalUnion[{', '.join(i.name for i in its)}]",
                             shared_metrics=SharedMetrics(parents=[i.shared_metrics for i in its]))

    def duplicate(self, n: int) -> List["LocalIterator"]:
        """n iterators over the same items (buffers what the slowest has not consumed)."""
        src = iter(self)
        queues = [collections.deque() for _ in range(n)]

        def make(i):
            def gen():
                while True:
                    if not queues[i]:
                        try:
                            x = next(src)
                        except StopIteration:
                            return
                        for q in queues:
                            q.append(x)
                    yield queues[i].popleft()
            return gen

        return [LocalIterator(make(i), self.name + f".duplicate[{i}]", shared_metrics=self.shared_metrics)
                for i in range(n)]
