"""Row-wise sample-batch builders. Parity: reference rllib/evaluation/sample_batch_builder.py
(SampleBatchBuilder, MultiAgentSampleBatchBuilder). Columns accumulate as Python lists and become
numpy arrays once in build_and_reset."""
from __future__ import annotations

import collections
from typing import Any, Dict, Optional

import numpy as np

from ray_memory_management_amd.rllib.sample_batch import MultiAgentBatch, SampleBatch


def _to_array(v):
    try:
        return np.asarray(v)
    except Exception:
        out = np.empty(len(v), dtype=object)
        out[:] = v
        return out


class SampleBatchBuilder:
    def __init__(self):
        self.buffers: Dict[str, list] = collections.defaultdict(list)
        self.count = 0

    def add_values(self, **values: Any) -> None:
        for k, v in values.items():
            self.buffers[k].append(v)
        self.count += 1

    def add_batch(self, batch: SampleBatch) -> None:
        for k, v in batch.items():
            self.buffers[k].extend(list(v))
        self.count += batch.count

    def build_and_reset(self) -> SampleBatch:
        b = SampleBatch({k: _to_array(v) for k, v in self.buffers.items()})
        self.buffers.clear()
        self.count = 0
        return b


class MultiAgentSampleBatchBuilder:
    """Per-agent builders; ``postprocess_batch_so_far`` runs each policy's postprocess_trajectory
    on its agents' trajectories (with the other agents' batches) and moves them into per-policy
    builders; ``build_and_reset`` returns a MultiAgentBatch."""

    def __init__(self, policy_map: Dict[str, Any], clip_rewards: bool = False, callbacks=None):
        self.policy_map = policy_map
        self.clip_rewards = clip_rewards
        self.callbacks = callbacks
        self.policy_builders = {pid: SampleBatchBuilder() for pid in policy_map}
        self.agent_builders: Dict[Any, SampleBatchBuilder] = {}
        self.agent_to_policy: Dict[Any, str] = {}
        self.count = 0

    def total(self) -> int:
        return sum(b.count for b in self.agent_builders.values())

    def has_pending_agent_data(self) -> bool:
        return bool(self.agent_builders)

    def add_values(self, agent_id, policy_id: str, **values: Any) -> None:
        if agent_id not in self.agent_builders:
            self.agent_builders[agent_id] = SampleBatchBuilder()
            self.agent_to_policy[agent_id] = policy_id
        if self.clip_rewards and "rewards" in values:
            values["rewards"] = float(np.sign(values["rewards"]))
        self.agent_builders[agent_id].add_values(**values)

    def postprocess_batch_so_far(self, episode=None) -> None:
        pre = {a: b.build_and_reset() for a, b in self.agent_builders.items()}
        for agent_id, batch in pre.items():
            pid = self.agent_to_policy[agent_id]
            others = {a: (self.agent_to_policy[a], self.policy_map[self.agent_to_policy[a]], b)
                      for a, b in pre.items() if a != agent_id}
            pol = self.policy_map[pid]
            post = pol.postprocess_trajectory(batch, others, episode) if hasattr(pol, "postprocess_trajectory") \
                else batch
            self.policy_builders[pid].add_batch(post)
        self.agent_builders.clear()
        self.agent_to_policy.clear()

    def build_and_reset(self, episode=None) -> MultiAgentBatch:
        self.postprocess_batch_so_far(episode)
        batches = {pid: b.build_and_reset() for pid, b in self.policy_builders.items() if b.count > 0}
        n = self.count
        self.count = 0
        return MultiAgentBatch(batches, n)
