"""ActorPool: run work over a fixed set of actors.

Parity: reference python/ray/util/actor_pool.py (map / map_unordered / submit / has_next /
get_next / get_next_unordered / has_free / pop_idle / push). Ordered results are tracked by a
submission index; unordered results are harvested with ``wait`` over the in-flight futures.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Tuple

import ray_memory_management_amd as ray


class ActorPool:
    def __init__(self, actors: list):
        self._idle: List[Any] = list(actors)
        self._future_to_actor: Dict[Any, Tuple[int, Any]] = {}
        self._index_to_future: Dict[int, Any] = {}
        self._next_task_index = 0
        self._next_return_index = 0
        self._pending: List[Tuple[Callable, Any]] = []  # submitted while no actor was free

    # ------------------------------------------------------------------ submission
    def submit(self, fn: Callable[[Any, Any], Any], value: Any) -> None:
        """Schedule fn(actor, value) on a free actor (queued until one frees up)."""
        if self._idle:
            actor = self._idle.pop()
            fut = fn(actor, value)
            self._future_to_actor[fut] = (self._next_task_index, actor)
            self._index_to_future[self._next_task_index] = fut
            self._next_task_index += 1
        else:
            self._pending.append((fn, value))

    def map(self, fn: Callable[[Any, Any], Any], values):
        """Ordered results of fn(actor, v) for every v (a generator)."""
        while self.has_next():  # drain results from previous calls first
            try:
                self.get_next_unordered(timeout=0)
            except TimeoutError:
                pass
        for v in values:
            self.submit(fn, v)
        while self.has_next():
            yield self.get_next()

    def map_unordered(self, fn: Callable[[Any, Any], Any], values):
        while self.has_next():
            try:
                self.get_next_unordered(timeout=0)
            except TimeoutError:
                pass
        for v in values:
            self.submit(fn, v)
        while self.has_next():
            yield self.get_next_unordered()

    # ------------------------------------------------------------------ results
    def has_next(self) -> bool:
        return bool(self._future_to_actor) or bool(self._pending)

    def get_next(self, timeout=None, ignore_if_timedout: bool = False):
        """Next result in submission order."""
        if not self.has_next():
            raise StopIteration("No more results to get")
        if self._next_return_index >= self._next_task_index:
            raise ValueError("It is not allowed to call get_next() after get_next_unordered().")
        fut = self._index_to_future[self._next_return_index]
        if timeout is not None:
            ready, _ = ray.wait([fut], timeout=timeout)
            if not ready:
                if ignore_if_timedout:
                    return None
                raise TimeoutError("Timed out waiting for result")
        del self._index_to_future[self._next_return_index]
        self._next_return_index += 1
        _, actor = self._future_to_actor.pop(fut)
        self._return_actor(actor)
        return ray.get(fut)

    def get_next_unordered(self, timeout=None, ignore_if_timedout: bool = False):
        """Any finished result (completion order)."""
        if not self.has_next():
            raise StopIteration("No more results to get")
        ready, _ = ray.wait(list(self._future_to_actor), num_returns=1, timeout=timeout)
        if not ready:
            if ignore_if_timedout:
                return None
            raise TimeoutError("Timed out waiting for result")
        fut = ready[0]
        i, actor = self._future_to_actor.pop(fut)
        self._index_to_future.pop(i, None)
        self._next_return_index = max(self._next_return_index, i + 1)
        self._return_actor(actor)
        return ray.get(fut)

    def _return_actor(self, actor):
        self._idle.append(actor)
        if self._pending:
            fn, value = self._pending.pop(0)
            self.submit(fn, value)

    # ------------------------------------------------------------------ pool management
    def has_free(self) -> bool:
        return bool(self._idle) and not self._pending

    def pop_idle(self):
        return self._idle.pop() if self.has_free() else None

    def push(self, actor):
        busy = {a for _, a in self._future_to_actor.values()}
        if actor in self._idle or actor in busy:
            raise ValueError("Actor already belongs to current ActorPool")
        self._return_actor(actor)
