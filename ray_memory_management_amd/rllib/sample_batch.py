"""SampleBatch. Parity: reference rllib/policy/sample_batch.py (column dict, concat_samples,
slicing, shuffle, timeslices/minibatches, MultiAgentBatch).

Columns may be numpy arrays (CPU rollout workers) or torch tensors. GPU columns are concatenated
with ONE multi-segment copy launch per column (ops.concat, kernel K1) and minibatches are gathered
with the row-gather kernel (ops.gather_rows, K2)."""
from __future__ import annotations

from typing import Dict, Iterator, List

import numpy as np


def _is_torch(x):
    return type(x).__module__.startswith("torch")


class SampleBatch(dict):
    OBS = "obs"
    NEXT_OBS = "new_obs"
    ACTIONS = "actions"
    REWARDS = "rewards"
    DONES = "dones"
    INFOS = "infos"
    EPS_ID = "eps_id"
    AGENT_INDEX = "agent_index"
    T = "t"
    ACTION_LOGP = "action_logp"
    ACTION_DIST_INPUTS = "action_dist_inputs"
    VF_PREDS = "vf_preds"
    ADVANTAGES = "advantages"
    VALUE_TARGETS = "value_targets"

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.count = self._infer_count()

    def _infer_count(self):
        for v in self.values():
            if hasattr(v, "shape") and len(v.shape) > 0:
                return int(v.shape[0])
            if isinstance(v, list):
                return len(v)
        return 0

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        if not self.count:
            self.count = self._infer_count()

    def __len__(self):  # reference: len(batch) == number of rows
        return self.count

    @property
    def env_steps(self):
        return self.count

    def copy(self):
        return SampleBatch({k: (v.clone() if _is_torch(v) else np.array(v, copy=True)) for k, v in self.items()})

    def slice(self, start: int, end: int) -> "SampleBatch":
        return SampleBatch({k: v[start:end] for k, v in self.items()})

    def __getitem__(self, key):
        if isinstance(key, slice):
            return self.slice(key.start or 0, key.stop if key.stop is not None else self.count)
        return dict.__getitem__(self, key)

    def rows(self) -> Iterator[dict]:
        for i in range(self.count):
            yield {k: v[i] for k, v in self.items()}

    def columns(self, keys: List[str]):
        return [self[k] for k in keys]

    def shuffle(self, seed=None) -> "SampleBatch":
        perm = _perm(self.count, self, seed)
        for k in list(self.keys()):
            dict.__setitem__(self, k, _take(dict.__getitem__(self, k), perm))
        return self

    def take(self, idx) -> "SampleBatch":
        return SampleBatch({k: _take(v, idx) for k, v in self.items()})

    def timeslices(self, size: int) -> List["SampleBatch"]:
        return [self.slice(i, min(i + size, self.count)) for i in range(0, self.count, size)]

    def minibatches(self, size: int, shuffle: bool = True, seed=None) -> Iterator["SampleBatch"]:
        """Yield minibatches of `size` rows; shuffled minibatches gather rows on-device."""
        if not shuffle:
            yield from self.timeslices(size)
            return
        perm = _perm(self.count, self, seed)
        for i in range(0, self.count - size + 1 if self.count >= size else 1, size):
            yield self.take(perm[i:i + size])

    def to_device(self, device):
        import torch

        out = SampleBatch()
        for k, v in self.items():
            if isinstance(v, np.ndarray) and v.dtype != object:
                dict.__setitem__(out, k, torch.from_numpy(np.ascontiguousarray(v)).to(device, non_blocking=True))
            elif _is_torch(v):
                dict.__setitem__(out, k, v.to(device, non_blocking=True))
            else:
                dict.__setitem__(out, k, v)
        out.count = self.count
        return out

    def size_bytes(self) -> int:
        return int(sum(v.nbytes if isinstance(v, np.ndarray) else (v.numel() * v.element_size() if _is_torch(v) else 0)
                       for v in self.values()))

    def __repr__(self):
        return f"SampleBatch({self.count}: {list(self.keys())})"

    def __reduce__(self):
        return (SampleBatch, (dict(self),))


def _perm(n, batch, seed):
    for v in batch.values():
        if _is_torch(v) and v.is_cuda:
            import torch

            g = None
            if seed is not None:
                g = torch.Generator(device=v.device)
                g.manual_seed(seed)
            return torch.randperm(n, device=v.device, generator=g)
    rng = np.random.default_rng(seed)
    return rng.permutation(n)


def _take(v, idx):
    if _is_torch(v):
        import torch

        if v.is_cuda:
            from ray_memory_management_amd import ops

            if not _is_torch(idx):
                idx = torch.as_tensor(np.asarray(idx), device=v.device)
            return ops.gather_rows(v, idx)
        if not _is_torch(idx):
            idx = torch.as_tensor(np.asarray(idx))
        return v[idx.cpu()]
    if isinstance(v, np.ndarray):
        if _is_torch(idx):
            idx = idx.cpu().numpy()
        return v[idx]
    if isinstance(v, list):
        if _is_torch(idx):
            idx = idx.cpu().numpy()
        return [v[int(i)] for i in idx]
    return v


def concat_samples(batches: List[SampleBatch]) -> SampleBatch:
    batches = [b for b in batches if b is not None and b.count > 0]
    if not batches:
        return SampleBatch()
    out = SampleBatch()
    for k in batches[0].keys():
        vals = [dict.__getitem__(b, k) for b in batches]
        v0 = vals[0]
        if _is_torch(v0):
            from ray_memory_management_amd import ops

            dict.__setitem__(out, k, ops.concat(vals))
        elif isinstance(v0, np.ndarray):
            dict.__setitem__(out, k, np.concatenate(vals))
        elif isinstance(v0, list):
            dict.__setitem__(out, k, sum(vals, []))
        else:
            dict.__setitem__(out, k, v0)
    out.count = sum(b.count for b in batches)
    return out


SampleBatch.concat_samples = staticmethod(concat_samples)


class MultiAgentBatch:
    def __init__(self, policy_batches: Dict[str, SampleBatch], env_steps: int):
        self.policy_batches = policy_batches
        self.count = env_steps

    def env_steps(self):
        return self.count

    def agent_steps(self):
        return sum(b.count for b in self.policy_batches.values())

    @staticmethod
    def concat_samples(samples: List["MultiAgentBatch"]) -> "MultiAgentBatch":
        """Concatenate per policy (reference MultiAgentBatch.concat_samples)."""
        per: Dict[str, List[SampleBatch]] = {}
        steps = 0
        for s in samples:
            if isinstance(s, SampleBatch):
                s = MultiAgentBatch({DEFAULT_POLICY_ID: s}, s.count)
            steps += s.count
            for pid, b in s.policy_batches.items():
                per.setdefault(pid, []).append(b)
        return MultiAgentBatch({pid: concat_samples(bs) for pid, bs in per.items()}, steps)

    def __len__(self):
        return self.count


DEFAULT_POLICY_ID = "default_policy"
