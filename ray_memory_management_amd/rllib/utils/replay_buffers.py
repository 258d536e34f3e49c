"""Replay buffers. Parity: reference rllib/utils/replay_buffers/{replay_buffer,
prioritized_replay_buffer,reservoir_replay_buffer}.py and rllib/execution/segment_tree.py
(ReplayBuffer(capacity, storage_unit="timesteps") add / sample / stats / get_state / set_state;
PrioritizedReplayBuffer(alpha) sample(n, beta) with importance weights + update_priorities).

Storage is COLUMNAR and preallocated (one ring array per column, allocated on the first add),
not a list of per-step SampleBatches: ``add`` is one slice assignment per column and ``sample`` is
one gather per column. With ``device="cuda"`` the columns live in HBM next to the learner and the
sample is the K2 row-gather kernel (ops.gather_rows) — no host round trip per training batch.
The prioritized variant keeps its sum / min segment trees as flat numpy arrays (vectorised
prefix-sum search for a whole batch at once).
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np

from ray_memory_management_amd.rllib.sample_batch import SampleBatch


class ReplayBuffer:
    def __init__(self, capacity: int = 10000, storage_unit: str = "timesteps", device: Optional[str] = None,
                 seed: Optional[int] = None, **kwargs):
        if storage_unit not in ("timesteps",):
            raise ValueError("only storage_unit='timesteps' is supported")
        self.capacity = int(capacity)
        self.device = device
        self._cols: Dict[str, Any] = {}
        self._next = 0
        self._size = 0
        self._added = 0
        self._sampled = 0
        self._rng = np.random.default_rng(seed)

    def __len__(self):
        return self._size

    def _alloc(self, k, v):
        shape = (self.capacity,) + tuple(np.shape(v)[1:])
        if self.device and self.device != "cpu":
            import torch

            dt = v.dtype if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v[:1])).dtype
            return torch.empty(shape, dtype=dt, device=self.device)
        return np.empty(shape, dtype=np.asarray(v[:1]).dtype)

    def _write(self, dst, start, v):
        if self.device and self.device != "cpu":
            import torch

            src = v if isinstance(v, torch.Tensor) else torch.as_tensor(np.asarray(v))
            dst[start:start + len(v)] = src.to(self.device, non_blocking=True)
        else:
            dst[start:start + len(v)] = np.asarray(v)

    def add(self, batch: SampleBatch, **kwargs) -> np.ndarray:
        """Append a batch of timesteps (ring overwrite when full). Returns the slots written."""
        n = batch.count
        if n == 0:
            return np.zeros(0, dtype=np.int64)
        if n > self.capacity:
            batch = batch.slice(n - self.capacity, n)
            n = self.capacity
        for k, v in batch.items():
            if k not in self._cols:
                self._cols[k] = self._alloc(k, v)
        slots = (self._next + np.arange(n)) % self.capacity
        first = min(n, self.capacity - self._next)
        for k, v in batch.items():
            self._write(self._cols[k], self._next, v[:first])
            if first < n:
                self._write(self._cols[k], 0, v[first:])
        self._next = (self._next + n) % self.capacity
        self._size = min(self.capacity, self._size + n)
        self._added += n
        return slots

    def _gather(self, idx: np.ndarray) -> SampleBatch:
        out = SampleBatch()
        if self.device and self.device != "cpu":
            import torch

            from ray_memory_management_amd import ops

            ti = torch.as_tensor(idx, dtype=torch.int64, device=self.device)
            for k, v in self._cols.items():
                dict.__setitem__(out, k, ops.gather_rows(v, ti) if v.is_cuda else v[ti.cpu()])
        else:
            for k, v in self._cols.items():
                dict.__setitem__(out, k, v[idx])
        out.count = len(idx)
        return out

    def sample(self, num_items: int, **kwargs) -> Optional[SampleBatch]:
        if self._size == 0:
            return None
        idx = self._rng.integers(0, self._size, size=num_items)
        self._sampled += num_items
        b = self._gather(idx)
        dict.__setitem__(b, "batch_indexes", idx)
        return b

    def stats(self, debug: bool = False) -> dict:
        return {"added_count": self._added, "sampled_count": self._sampled, "num_entries": self._size,
                "est_size_bytes": int(sum((v.nbytes if hasattr(v, "nbytes") else v.numel() * v.element_size())
                                          for v in self._cols.values()))}

    def get_state(self) -> Dict[str, Any]:
        cols = {k: (v[:self._size].cpu().numpy() if hasattr(v, "cpu") else v[:self._size].copy())
                for k, v in self._cols.items()}
        return {"cols": cols, "next": self._next, "size": self._size, "added": self._added}

    def set_state(self, state: Dict[str, Any]) -> None:
        self._cols = {}
        b = SampleBatch(state["cols"])
        self._next = self._size = 0
        if b.count:
            self.add(b)
        self._next, self._size, self._added = state["next"], state["size"], state["added"]


class _SegmentTrees:
    """Sum + min trees over `cap` (power of two) leaves as flat arrays; batched updates/queries."""

    def __init__(self, cap: int):
        self.cap = cap
        self.sum = np.zeros(2 * cap, dtype=np.float64)
        self.min = np.full(2 * cap, np.inf, dtype=np.float64)

    def update(self, idx: np.ndarray, val: np.ndarray):
        for i, v in zip(np.asarray(idx), np.asarray(val, dtype=np.float64)):
            j = int(i) + self.cap
            self.sum[j] = v
            self.min[j] = v
            j //= 2
            while j >= 1:
                self.sum[j] = self.sum[2 * j] + self.sum[2 * j + 1]
                self.min[j] = min(self.min[2 * j], self.min[2 * j + 1])
                j //= 2

    def total(self) -> float:
        return float(self.sum[1])

    def find_prefixsum(self, mass: np.ndarray) -> np.ndarray:
        """Leaf index with cumulative sum >= mass, for a whole vector of masses (descends the tree
        for every query at once)."""
        idx = np.ones(len(mass), dtype=np.int64)
        mass = np.asarray(mass, dtype=np.float64).copy()
        while idx[0] < self.cap:
            left = 2 * idx
            ls = self.sum[left]
            go_right = mass > ls
            mass = np.where(go_right, mass - ls, mass)
            idx = np.where(go_right, left + 1, left)
        return idx - self.cap


class PrioritizedReplayBuffer(ReplayBuffer):
    def __init__(self, capacity: int = 10000, storage_unit: str = "timesteps", alpha: float = 1.0, **kwargs):
        super().__init__(capacity, storage_unit, **kwargs)
        if alpha <= 0:
            raise ValueError("alpha must be > 0")
        self._alpha = alpha
        cap = 1
        while cap < self.capacity:
            cap *= 2
        self._trees = _SegmentTrees(cap)
        self._max_priority = 1.0

    def add(self, batch: SampleBatch, weight: Optional[float] = None, **kwargs) -> np.ndarray:
        slots = super().add(batch)
        w = self._max_priority if weight is None else weight
        self._trees.update(slots, np.full(len(slots), w ** self._alpha))
        return slots

    def sample(self, num_items: int, beta: float = 0.4, **kwargs) -> Optional[SampleBatch]:
        if self._size == 0:
            return None
        total = self._trees.total()
        mass = (self._rng.random(num_items) + np.arange(num_items)) * (total / num_items)  # stratified
        idx = np.minimum(self._trees.find_prefixsum(mass), self._size - 1)
        p_min = self._trees.min[1] / total
        max_w = (p_min * self._size) ** (-beta)
        p = self._trees.sum[idx + self._trees.cap] / total
        weights = (p * self._size) ** (-beta) / max_w
        self._sampled += num_items
        b = self._gather(idx)
        dict.__setitem__(b, "weights", weights.astype(np.float32))
        dict.__setitem__(b, "batch_indexes", idx)
        return b

    def update_priorities(self, idxes, priorities) -> None:
        pr = np.asarray(priorities, dtype=np.float64)
        if np.any(pr <= 0):
            raise ValueError("priorities must be > 0")
        self._trees.update(np.asarray(idxes), pr ** self._alpha)
        self._max_priority = max(self._max_priority, float(pr.max()))


class ReservoirReplayBuffer(ReplayBuffer):
    """Reservoir sampling over everything ever added (uniform over the stream)."""

    def add(self, batch: SampleBatch, **kwargs) -> np.ndarray:
        out = []
        for i in range(batch.count):
            row = batch.slice(i, i + 1)
            if self._size < self.capacity:
                out.append(super().add(row))
                continue
            self._added += 1
            j = int(self._rng.integers(0, self._added))
            if j < self.capacity:
                saved = self._next
                self._next = j
                super().add(row)
                self._added -= 1
                self._next = saved
                out.append(np.array([j]))
        return np.concatenate(out) if out else np.zeros(0, dtype=np.int64)
