"""Distributed FIFO queue backed by an async actor.

Parity: reference python/ray/util/queue.py (Queue with put/get blocking + timeouts, *_nowait,
*_nowait_batch, put_async/get_async, size/qsize/empty/full, shutdown; Empty/Full exceptions).
"""
from __future__ import annotations

import asyncio
import queue as _stdq
from typing import Any, Dict, Iterable, List, Optional

import ray_memory_management_amd as ray


class Empty(_stdq.Empty):
    pass


class Full(_stdq.Full):
    pass


class _QueueActor:
    def __init__(self, maxsize):
        self.maxsize = maxsize
        self.queue = asyncio.Queue(maxsize)

    def qsize(self):
        return self.queue.qsize()

    def empty(self):
        return self.queue.empty()

    def full(self):
        return self.queue.full()

    async def put(self, item, timeout=None):
        try:
            await asyncio.wait_for(self.queue.put(item), timeout)
        except asyncio.TimeoutError:
            raise Full

    async def get(self, timeout=None):
        try:
            return await asyncio.wait_for(self.queue.get(), timeout)
        except asyncio.TimeoutError:
            raise Empty

    def put_nowait(self, item):
        self.queue.put_nowait(item)

    def put_nowait_batch(self, items):
        if self.maxsize > 0 and len(items) + self.qsize() > self.maxsize:
            raise Full(f"Cannot add {len(items)} items to queue of size {self.qsize()} and maxsize {self.maxsize}.")
        for item in items:
            self.queue.put_nowait(item)

    def get_nowait(self):
        return self.queue.get_nowait()

    def get_nowait_batch(self, num_items):
        if num_items > self.qsize():
            raise Empty(f"Cannot get {num_items} items from queue of size {self.qsize()}.")
        return [self.queue.get_nowait() for _ in range(num_items)]


class Queue:
    def __init__(self, maxsize: int = 0, actor_options: Optional[Dict] = None) -> None:
        actor_options = actor_options or {}
        self.maxsize = maxsize
        self.actor = ray.remote(_QueueActor).options(**actor_options).remote(self.maxsize)

    def __len__(self) -> int:
        return self.size()

    def size(self) -> int:
        return ray.get(self.actor.qsize.remote())

    def qsize(self) -> int:
        return self.size()

    def empty(self) -> bool:
        return ray.get(self.actor.empty.remote())

    def full(self) -> bool:
        return ray.get(self.actor.full.remote())

    def put(self, item: Any, block: bool = True, timeout: Optional[float] = None) -> None:
        if not block:
            try:
                ray.get(self.actor.put_nowait.remote(item))
            except asyncio.QueueFull:
                raise Full
            except ray.exceptions.RayTaskError as e:
                raise Full from e
        else:
            if timeout is not None and timeout < 0:
                raise ValueError("'timeout' must be a non-negative number")
            try:
                ray.get(self.actor.put.remote(item, timeout))
            except ray.exceptions.RayTaskError as e:
                raise Full from e

    async def put_async(self, item: Any, block: bool = True, timeout: Optional[float] = None) -> None:
        loop = asyncio.get_event_loop()
        await loop.run_in_executor(None, lambda: self.put(item, block, timeout))

    def get(self, block: bool = True, timeout: Optional[float] = None) -> Any:
        if not block:
            try:
                return ray.get(self.actor.get_nowait.remote())
            except ray.exceptions.RayTaskError as e:
                raise Empty from e
        if timeout is not None and timeout < 0:
            raise ValueError("'timeout' must be a non-negative number")
        try:
            return ray.get(self.actor.get.remote(timeout))
        except ray.exceptions.RayTaskError as e:
            raise Empty from e

    async def get_async(self, block: bool = True, timeout: Optional[float] = None) -> Any:
        loop = asyncio.get_event_loop()
        return await loop.run_in_executor(None, lambda: self.get(block, timeout))

    def put_nowait(self, item: Any) -> None:
        return self.put(item, block=False)

    def put_nowait_batch(self, items: Iterable) -> None:
        if not isinstance(items, Iterable):
            raise TypeError("Argument 'items' must be an Iterable")
        try:
            ray.get(self.actor.put_nowait_batch.remote(list(items)))
        except ray.exceptions.RayTaskError as e:
            raise Full(str(e)) from e

    def get_nowait(self) -> Any:
        return self.get(block=False)

    def get_nowait_batch(self, num_items: int) -> List[Any]:
        if not isinstance(num_items, int):
            raise TypeError("Argument 'num_items' must be an int")
        if num_items < 0:
            raise ValueError("'num_items' must be nonnegative")
        try:
            return ray.get(self.actor.get_nowait_batch.remote(num_items))
        except ray.exceptions.RayTaskError as e:
            raise Empty(str(e)) from e

    def shutdown(self, force: bool = False, grace_period_s: int = 5) -> None:
        if self.actor is not None:
            if force:
                ray.kill(self.actor, no_restart=True)
            else:
                done = self.actor.__ray_terminate__.remote()
                ready, _ = ray.wait([done], timeout=grace_period_s)
                if not ready:
                    ray.kill(self.actor, no_restart=True)
        self.actor = None
