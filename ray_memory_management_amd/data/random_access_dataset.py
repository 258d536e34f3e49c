"""Random access by key over a sorted Dataset. Parity: reference
python/ray/data/random_access_dataset.py (sort on key, range-partitioned serving actors,
get_async / multiget)."""
from __future__ import annotations

import bisect
from typing import Any, List, Optional

import ray_memory_management_amd as ray
from ray_memory_management_amd.data.block import BlockAccessor, concat_blocks


class _RandomAccessWorker:
    def __init__(self, key):
        self.key = key
        self.rows = []
        self.keys = []

    def assign_blocks(self, *blocks):
        b = concat_blocks(list(blocks))
        self.rows = list(BlockAccessor.for_block(b).iter_rows())
        self.keys = [r[self.key] for r in self.rows]
        return len(self.rows)

    def get(self, k):
        i = bisect.bisect_left(self.keys, k)
        if i < len(self.keys) and self.keys[i] == k:
            return self.rows[i]
        return None

    def multiget(self, ks):
        return [self.get(k) for k in ks]


class RandomAccessDataset:
    def __init__(self, dataset, key: str, num_workers: Optional[int] = None):
        ds = dataset.sort(key)
        blocks = ds._blocks()
        metas = ds._metas()
        nw = max(1, min(num_workers or len(blocks), len(blocks)))
        groups = [list(range(i, len(blocks), nw)) for i in range(nw)]
        # contiguous assignment keeps each worker's key range contiguous
        per = -(-len(blocks) // nw)
        groups = [list(range(i * per, min((i + 1) * per, len(blocks)))) for i in range(nw)]
        cls = ray.remote(_RandomAccessWorker)
        self._workers = [cls.remote(key) for _ in groups]
        ray.get([w.assign_blocks.remote(*[blocks[i] for i in g]) for w, g in zip(self._workers, groups)])
        # lower bound key of each worker
        firsts = []
        for g in groups:
            lo = None
            for i in g:
                if metas[i].num_rows:
                    lo = ray.get(_first_key.remote(blocks[i], key))
                    break
            firsts.append(lo)
        self._bounds = [(f, w) for f, w in zip(firsts, self._workers) if f is not None]
        self._keys = [f for f, _ in self._bounds]

    def _worker_for(self, k):
        i = max(bisect.bisect_right(self._keys, k) - 1, 0)
        return self._bounds[i][1] if self._bounds else None

    def get_async(self, key: Any):
        w = self._worker_for(key)
        return w.get.remote(key) if w is not None else ray.put(None)

    def multiget(self, keys: List[Any]) -> List[Any]:
        by_worker = {}
        for i, k in enumerate(keys):
            w = self._worker_for(k)
            by_worker.setdefault(id(w), (w, []))[1].append((i, k))
        out = [None] * len(keys)
        refs = [(items, w.multiget.remote([k for _, k in items])) for w, items in by_worker.values() if w is not None]
        for items, r in refs:
            for (i, _), v in zip(items, ray.get(r)):
                out[i] = v
        return out

    def stats(self) -> str:
        return f"RandomAccessDataset(num_workers={len(self._workers)})"


@ray.remote
def _first_key(block, key):
    for r in BlockAccessor.for_block(block).iter_rows():
        return r[key]
    return None
