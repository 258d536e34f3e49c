"""Algorithm / rollout callbacks. Parity: reference rllib/algorithms/callbacks.py (DefaultCallbacks:
on_algorithm_init, on_episode_start / on_episode_step / on_episode_end, on_sample_end,
on_learn_on_batch, on_train_result; MultiCallbacks) and rllib/evaluation/episode.py (Episode:
episode_id, length, total_reward, custom_metrics, user_data, hist_data). Custom metrics recorded in
`episode.custom_metrics` are aggregated into ``result["custom_metrics"]`` as <name>_mean/_min/_max.
"""
from __future__ import annotations

from typing import Dict, List


class Episode:
    """Per-episode scratch space handed to the episode callbacks."""

    def __init__(self, episode_id: int, env_index: int = 0):
        self.episode_id = episode_id
        self.env_id = env_index
        self.length = 0
        self.total_reward = 0.0
        self.custom_metrics: Dict[str, float] = {}
        self.user_data: Dict = {}
        self.hist_data: Dict[str, List[float]] = {}
        self.media: Dict = {}
        self._last_obs = None
        self._last_action = None
        self._last_reward = None

    def last_observation_for(self, agent_id=None):
        return self._last_obs

    def last_action_for(self, agent_id=None):
        return self._last_action

    def last_reward_for(self, agent_id=None):
        return self._last_reward


class DefaultCallbacks:
    def on_algorithm_init(self, *, algorithm, **kw):
        pass

    def on_episode_start(self, *, worker, base_env, policies, episode: Episode, env_index=None, **kw):
        pass

    def on_episode_step(self, *, worker, base_env, policies=None, episode: Episode, env_index=None, **kw):
        pass

    def on_episode_end(self, *, worker, base_env, policies, episode: Episode, env_index=None, **kw):
        pass

    def on_sample_end(self, *, worker, samples, **kw):
        pass

    def on_learn_on_batch(self, *, policy, train_batch, result, **kw):
        pass

    def on_train_result(self, *, algorithm, result: dict, **kw):
        pass


class MultiCallbacks(DefaultCallbacks):
    """Fan every hook out to several callback classes (reference MultiCallbacks)."""

    def __init__(self, callback_class_list):
        self._classes = list(callback_class_list)
        self._cbs = [c() for c in self._classes]

    def __call__(self):  # used as a "class" by configs: MultiCallbacks([...]) then instantiated
        return MultiCallbacks(self._classes)

    def _each(self, name, **kw):
        for c in self._cbs:
            getattr(c, name)(**kw)

    def on_algorithm_init(self, **kw):
        self._each("on_algorithm_init", **kw)

    def on_episode_start(self, **kw):
        self._each("on_episode_start", **kw)

    def on_episode_step(self, **kw):
        self._each("on_episode_step", **kw)

    def on_episode_end(self, **kw):
        self._each("on_episode_end", **kw)

    def on_sample_end(self, **kw):
        self._each("on_sample_end", **kw)

    def on_learn_on_batch(self, **kw):
        self._each("on_learn_on_batch", **kw)

    def on_train_result(self, **kw):
        self._each("on_train_result", **kw)


def summarize_custom_metrics(values: Dict[str, List[float]]) -> Dict[str, float]:
    import numpy as np

    out = {}
    for k, v in values.items():
        if v:
            out[f"{k}_mean"] = float(np.mean(v))
            out[f"{k}_min"] = float(np.min(v))
            out[f"{k}_max"] = float(np.max(v))
    return out
