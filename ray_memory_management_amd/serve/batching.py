"""@serve.batch. Parity: reference python/ray/serve/batching.py — concurrent calls to an async
method are queued and executed as ONE call on a list of inputs (max_batch_size, waiting at most
batch_wait_timeout_s for the batch to fill); each caller gets its own element of the result."""
from __future__ import annotations

import asyncio
import functools
from typing import Callable, Optional


class _BatchQueue:
    def __init__(self, max_batch_size: int, timeout_s: float, handler: Callable):
        self.max_batch_size, self.timeout_s, self.handler = max_batch_size, timeout_s, handler
        self.queue: asyncio.Queue = asyncio.Queue()
        self.task = asyncio.get_event_loop().create_task(self._loop())

    async def _loop(self):
        while True:
            first = await self.queue.get()
            batch = [first]
            deadline = asyncio.get_event_loop().time() + self.timeout_s
            while len(batch) < self.max_batch_size:
                left = deadline - asyncio.get_event_loop().time()
                if left <= 0:
                    break
                try:
                    batch.append(await asyncio.wait_for(self.queue.get(), left))
                except asyncio.TimeoutError:
                    break
            args = [b[0] for b in batch]
            futs = [b[1] for b in batch]
            selfs = batch[0][2]
            try:
                res = await (self.handler(selfs, args) if selfs is not None else self.handler(args))
                if not isinstance(res, (list, tuple)) or len(res) != len(args):
                    raise TypeError(f"Batched function returned {type(res).__name__} of length "
                                    f"{len(res) if hasattr(res, '__len__') else '?'}; expected a list of length "
                                    f"{len(args)} (one result per input).")
                for f, r in zip(futs, res):
                    if not f.done():
                        f.set_result(r)
            except Exception as e:
                for f in futs:
                    if not f.done():
                        f.set_exception(e)


def batch(_func: Optional[Callable] = None, max_batch_size: int = 10, batch_wait_timeout_s: float = 0.0):
    if max_batch_size < 1:
        raise ValueError("max_batch_size must be an integer >= 1")
    if batch_wait_timeout_s < 0:
        raise ValueError("batch_wait_timeout_s must be a float >= 0")

    def deco(fn):
        if not asyncio.iscoroutinefunction(fn):
            raise TypeError("Functions decorated with @serve.batch must be 'async def'")
        is_method = "self" in fn.__code__.co_varnames[:1]
        attr = f"__serve_batch_queue_{fn.__name__}"

        if is_method:
            @functools.wraps(fn)
            async def wrapper(self, arg):
                q = getattr(self, attr, None)
                if q is None:
                    q = _BatchQueue(max_batch_size, batch_wait_timeout_s, fn)
                    setattr(self, attr, q)
                fut = asyncio.get_event_loop().create_future()
                await q.queue.put((arg, fut, self))
                return await fut
        else:
            state = {}

            @functools.wraps(fn)
            async def wrapper(arg):
                q = state.get("q")
                if q is None:
                    q = state["q"] = _BatchQueue(max_batch_size, batch_wait_timeout_s, fn)
                fut = asyncio.get_event_loop().create_future()
                await q.queue.put((arg, fut, None))
                return await fut
        wrapper._serve_batch = True
        return wrapper

    return deco(_func) if callable(_func) else deco
