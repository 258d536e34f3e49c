"""Ape-X DQN: distributed prioritized experience replay.

Parity: reference rllib/algorithms/apex_dqn/apex_dqn.py (ApexDQNConfig: many rollout workers with
PerWorkerEpsilonGreedy exploration, `num_replay_buffer_shards` replay ACTORS, asynchronous sampling
with `max_requests_in_flight_per_sampler_worker`, asynchronous replay sampling by the learner,
priority updates sent back to the owning shard, weight broadcast to a worker once it has sampled
`max_weight_sync_delay` steps since its last sync, target network update every
`target_network_update_freq` trained steps) and rllib/utils/replay_buffers/replay_buffer actors.

Data path here: a worker's sample batch is an object in the shared-memory store; the driver passes
the ObjectRef straight on to a replay shard (`shard.add.remote(ref)`), so rollout rows go worker →
store → shard without ever being deserialised by the driver. Replay batches come back the same way
and feed the learner (on the GPU with ``num_gpus > 0``). `ApexMixin` carries the loop; Ape-X DDPG
reuses it with the DDPG learner.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np

import ray_memory_management_amd as ray
from ray_memory_management_amd.rllib.algorithms.dqn import DQN, DQNConfig
from ray_memory_management_amd.rllib.sample_batch import SampleBatch
from ray_memory_management_amd.rllib.utils.replay_buffers import PrioritizedReplayBuffer, ReplayBuffer

_KEEP = (SampleBatch.OBS, SampleBatch.NEXT_OBS, SampleBatch.ACTIONS, SampleBatch.REWARDS, SampleBatch.DONES)


class ReplayActor:
    """One replay shard (reference apex ReplayActor / MultiAgentPrioritizedReplayBuffer shard)."""

    def __init__(self, capacity: int, prioritized: bool, alpha: float = 0.6, seed=None):
        self.prioritized = prioritized
        self.buf = (PrioritizedReplayBuffer(capacity, alpha=alpha, seed=seed) if prioritized
                    else ReplayBuffer(capacity, seed=seed))

    def add(self, batch: SampleBatch) -> int:
        b = SampleBatch({k: np.asarray(batch[k]) for k in _KEEP if k in batch})
        self.buf.add(b)
        return b.count

    def sample(self, n: int, beta: float = 0.4):
        if len(self.buf) < n:
            return None
        return self.buf.sample(n, beta=beta) if self.prioritized else self.buf.sample(n)

    def update_priorities(self, idx, prio) -> None:
        if self.prioritized:
            self.buf.update_priorities(np.asarray(idx), np.asarray(prio))

    def stats(self) -> Dict:
        return self.buf.stats()

    def size(self) -> int:
        return len(self.buf)


class ApexMixin:
    """Asynchronous sampling → replay shards → learner loop shared by Ape-X DQN / DDPG."""

    def _setup_apex(self):
        c = self.algo_config
        rb = dict(c.replay_buffer_config)
        n_shards = max(1, int(c.num_replay_buffer_shards))
        prioritized = "Prioritized" in str(rb.get("type", "MultiAgentPrioritizedReplayBuffer"))
        cls = ray.remote(ReplayActor).options(num_cpus=0)
        cap = max(1, int(rb.get("capacity", 100000)) // n_shards)
        self.replay_actors: List = [cls.remote(cap, prioritized, rb.get("prioritized_replay_alpha", 0.6),
                                               None if c.seed is None else c.seed + i) for i in range(n_shards)]
        self._prioritized = prioritized
        self._sample_inflight: Dict = {}  # sample ref -> worker
        self._replay_inflight: Dict = {}  # replay-sample ref -> shard
        self._steps_since_sync: Dict = {}
        self._shard_rr = 0
        self._rows_per_sample = int(c.rollout_fragment_length) * int(c.num_envs_per_worker)
        self._trained_since_target = 0
        self._weights_ref = None
        self._weights_dirty = True

    def _weights(self):
        if self._weights_dirty or self._weights_ref is None:
            self._weights_ref = ray.put(self._learner_weights())
            self._weights_dirty = False
        return self._weights_ref

    def _apex_step(self) -> Dict:
        c = self.algo_config
        workers = self.workers.remote_workers()
        if not workers:
            raise ValueError(f"{type(self).__name__} needs num_rollout_workers >= 1")
        per = max(1, int(c.max_requests_in_flight_per_sampler_worker))
        for w in workers:  # keep `per` sample requests in flight on every worker
            have = sum(1 for x in self._sample_inflight.values() if x is w)
            for _ in range(per - have):
                self._sample_inflight[w.sample.remote()] = w
        ready, _ = ray.wait(list(self._sample_inflight), num_returns=len(self._sample_inflight), timeout=0)
        if not ready:
            ready, _ = ray.wait(list(self._sample_inflight), num_returns=1, timeout=60)
        adds = []
        for ref in ready:
            w = self._sample_inflight.pop(ref)
            shard = self.replay_actors[self._shard_rr % len(self.replay_actors)]
            self._shard_rr += 1
            adds.append(shard.add.remote(ref))  # rows never pass through the driver
            n = self._rows_per_sample
            self._counters["num_env_steps_sampled"] += n
            self._timesteps_total += n
            self._steps_since_sync[w] = self._steps_since_sync.get(w, 0) + n
            if self._steps_since_sync[w] >= c.max_weight_sync_delay:
                w.set_weights.remote(self._weights())
                self._steps_since_sync[w] = 0
                self._counters["num_weight_broadcasts"] += 1
            self._sample_inflight[w.sample.remote()] = w
        stats: Dict = {}
        if self._counters["num_env_steps_sampled"] > c.num_steps_sampled_before_learning_starts:
            ray.get(adds)
            beta = c.replay_buffer_config.get("prioritized_replay_beta", 0.4)
            for shard in self.replay_actors:
                if shard not in self._replay_inflight.values():
                    self._replay_inflight[shard.sample.remote(c.train_batch_size, beta)] = shard
            eps = c.replay_buffer_config.get("prioritized_replay_eps", 1e-6)
            # `training_intensity` (trained / sampled rows) paces the learner against the samplers;
            # without it the learner takes whatever replay batches are ready (as the reference's
            # learner thread trains as fast as it can)
            intensity = getattr(c, "training_intensity", None)
            want = intensity * (self._counters["num_env_steps_sampled"] - c.num_steps_sampled_before_learning_starts) \
                if intensity else 0
            rready, _ = ray.wait(list(self._replay_inflight), num_returns=len(self._replay_inflight), timeout=0.05)
            while rready:
                ref = rready.pop(0)
                shard = self._replay_inflight.pop(ref)
                tb = ray.get(ref)
                self._replay_inflight[shard.sample.remote(c.train_batch_size, beta)] = shard
                if tb is None:
                    continue
                out = self.learner.update(tb)
                self._weights_dirty = True
                if self._prioritized:
                    shard.update_priorities.remote(np.asarray(tb["batch_indexes"]), out["td_error"] + eps)
                stats.update({k: v for k, v in out.items() if k != "td_error"})
                self._counters["num_env_steps_trained"] += c.train_batch_size
                self._trained_since_target += c.train_batch_size
                if self._trained_since_target >= c.target_network_update_freq:
                    self._apex_target_update()
                    self._trained_since_target = 0
                    self._counters["num_target_updates"] += 1
                if not rready and self._counters["num_env_steps_trained"] < want:
                    rready, _ = ray.wait(list(self._replay_inflight), num_returns=1, timeout=10)
        if self._weights_dirty and self.workers.local_worker() is not None:
            # the driver's local policy (evaluate / compute_single_action) follows the learner
            self.workers.local_worker().set_weights(self._learner_weights())
        stats["num_samples_in_flight"] = len(self._sample_inflight)
        stats["num_replay_shards"] = len(self.replay_actors)
        return stats

    def replay_stats(self) -> List[Dict]:
        return ray.get([a.stats.remote() for a in self.replay_actors])

    def _stop_apex(self):
        for a in getattr(self, "replay_actors", []):
            try:
                ray.kill(a)
            except Exception:
                pass
        self.replay_actors = []


class ApexDQNConfig(DQNConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or ApexDQN)
        self.num_workers = 32
        self.num_envs_per_worker = 1
        self.rollout_fragment_length = 50
        self.train_batch_size = 512
        self.n_step = 3
        self.target_network_update_freq = 500000
        self.num_steps_sampled_before_learning_starts = 50000
        self.max_requests_in_flight_per_sampler_worker = 2
        self.max_weight_sync_delay = 400
        self.num_replay_buffer_shards = 4
        self.min_time_s_per_iteration = 30
        self.min_sample_timesteps_per_iteration = 25000
        self.replay_buffer_config = {"type": "MultiAgentPrioritizedReplayBuffer", "capacity": 2000000,
                                     "prioritized_replay_alpha": 0.6, "prioritized_replay_beta": 0.4,
                                     "prioritized_replay_eps": 1e-6}
        self.exploration_config = {"type": "PerWorkerEpsilonGreedy"}

    def training(self, *, num_replay_buffer_shards=None, max_requests_in_flight_per_sampler_worker=None,
                 max_weight_sync_delay=None, **kwargs) -> "ApexDQNConfig":
        for k, v in dict(num_replay_buffer_shards=num_replay_buffer_shards, max_weight_sync_delay=max_weight_sync_delay,
                         max_requests_in_flight_per_sampler_worker=max_requests_in_flight_per_sampler_worker).items():
            if v is not None:
                setattr(self, k, v)
        return super().training(**kwargs)


class ApexDQN(ApexMixin, DQN):
    _config_class = ApexDQNConfig

    def _setup_learner(self):
        super()._setup_learner()
        self.buffer = None  # replay lives in the shard actors
        self._setup_apex()

    def _learner_weights(self):
        return self.learner.get_weights()

    def _apex_target_update(self):
        self.learner.sync_target()

    def training_step(self) -> Dict:
        return self._apex_step()

    def cleanup(self):
        self._stop_apex()
        super().cleanup()


DEFAULT_CONFIG = ApexDQNConfig().to_dict()
