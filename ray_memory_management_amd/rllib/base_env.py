"""BaseEnv / ExternalEnv. Parity: reference rllib/env/base_env.py (BaseEnv.poll / send_actions /
try_reset over {env_id: {agent_id: ...}} dicts, convert_to_base_env for Env / VectorEnv /
MultiAgentEnv) and rllib/env/external_env.py (ExternalEnv: the application owns the loop and calls
start_episode / get_action / log_action / log_returns / end_episode from its own thread; the
sampler polls observations and answers with actions).

The ExternalEnv bridge is two condition-guarded queues per episode (observation out, action in);
`ExternalEnvBase.poll()` blocks until at least one episode has an observation ready."""
from __future__ import annotations

import queue
import threading
import uuid
from typing import Any, Dict, Optional, Tuple

_DUMMY_AGENT = "agent0"


class BaseEnv:
    """Async, batched, multi-agent env interface every sampler can drive."""

    observation_space = action_space = None

    def poll(self) -> Tuple[Dict, Dict, Dict, Dict, Dict]:
        """(obs, rewards, dones, infos, off_policy_actions), each {env_id: {agent_id: value}}."""
        raise NotImplementedError

    def send_actions(self, action_dict: Dict[Any, Dict[Any, Any]]) -> None:
        raise NotImplementedError

    def try_reset(self, env_id=None) -> Optional[Dict]:
        return None

    def get_sub_environments(self):
        return []

    def stop(self) -> None:
        pass


class _VectorBaseEnv(BaseEnv):
    """BaseEnv over N single-agent envs (a VectorEnv or a list of Env); episodes auto-reset."""

    def __init__(self, envs):
        self.envs = list(envs)
        self.observation_space = self.envs[0].observation_space
        self.action_space = self.envs[0].action_space
        self._obs = {i: e.reset() for i, e in enumerate(self.envs)}
        self._rew = {i: 0.0 for i in self._obs}
        self._done = {i: False for i in self._obs}
        self._info = {i: {} for i in self._obs}

    def poll(self):
        obs = {i: {_DUMMY_AGENT: o} for i, o in self._obs.items()}
        rew = {i: {_DUMMY_AGENT: self._rew[i]} for i in self._obs}
        done = {i: {_DUMMY_AGENT: self._done[i], "__all__": self._done[i]} for i in self._obs}
        info = {i: {_DUMMY_AGENT: self._info[i]} for i in self._obs}
        self._obs = {}
        return obs, rew, done, info, {}

    def send_actions(self, action_dict):
        for i, acts in action_dict.items():
            o, r, d, inf = self.envs[i].step(acts[_DUMMY_AGENT])
            self._obs[i], self._rew[i], self._done[i], self._info[i] = o, r, d, inf

    def try_reset(self, env_id=None):
        o = self.envs[env_id].reset()
        self._obs[env_id], self._rew[env_id], self._done[env_id] = o, 0.0, False
        return {env_id: {_DUMMY_AGENT: o}}

    def get_sub_environments(self):
        return self.envs


class _MultiAgentBaseEnv(BaseEnv):
    def __init__(self, envs):
        self.envs = list(envs)
        self.observation_space = self.envs[0].observation_space
        self.action_space = self.envs[0].action_space
        self._pending = {i: (e.reset(), {}, {"__all__": False}, {}) for i, e in enumerate(self.envs)}

    def poll(self):
        obs, rew, done, info = {}, {}, {}, {}
        for i, (o, r, d, inf) in self._pending.items():
            obs[i], rew[i], done[i], info[i] = o, r, d, inf
        self._pending = {}
        return obs, rew, done, info, {}

    def send_actions(self, action_dict):
        for i, acts in action_dict.items():
            self._pending[i] = self.envs[i].step(acts)

    def try_reset(self, env_id=None):
        o = self.envs[env_id].reset()
        self._pending[env_id] = (o, {}, {"__all__": False}, {})
        return {env_id: o}

    def get_sub_environments(self):
        return self.envs


def convert_to_base_env(env, make_env=None, num_envs: int = 1) -> BaseEnv:
    """Env / VectorEnv / MultiAgentEnv / ExternalEnv / BaseEnv → BaseEnv (reference
    base_env.convert_to_base_env)."""
    from ray_memory_management_amd.rllib.env import MultiAgentEnv, VectorEnv

    if isinstance(env, BaseEnv):
        return env
    if isinstance(env, ExternalEnv):
        return env.to_base_env()
    if isinstance(env, VectorEnv):
        return _VectorBaseEnv(env.envs)
    envs = [env] + [make_env(i) for i in range(1, num_envs)] if make_env else [env]
    if isinstance(env, MultiAgentEnv):
        return _MultiAgentBaseEnv(envs)
    return _VectorBaseEnv(envs)


class _Episode:
    def __init__(self, eid: str, training_enabled: bool):
        self.episode_id, self.training_enabled = eid, training_enabled
        self.obs_q: "queue.Queue" = queue.Queue(maxsize=1)
        self.act_q: "queue.Queue" = queue.Queue(maxsize=1)
        self.reward = 0.0
        self.off_policy_action = None
        self.done = False


class ExternalEnv(threading.Thread):
    """An env that drives itself: subclass and implement ``run()``, calling the episode API."""

    def __init__(self, action_space, observation_space, max_concurrent: int = 100):
        super().__init__(daemon=True)
        self.action_space, self.observation_space = action_space, observation_space
        self._max_concurrent = max_concurrent
        self._episodes: Dict[str, _Episode] = {}
        self._ready = threading.Condition()
        self._outbox: Dict[str, Tuple] = {}

    def run(self):  # pragma: no cover - user code
        raise NotImplementedError

    # --- application-side episode API -------------------------------------------------------
    def start_episode(self, episode_id: Optional[str] = None, training_enabled: bool = True) -> str:
        eid = episode_id or uuid.uuid4().hex
        if eid in self._episodes:
            raise ValueError(f"episode {eid} already started")
        if len(self._episodes) >= self._max_concurrent:
            raise ValueError(f"more than max_concurrent={self._max_concurrent} episodes")
        self._episodes[eid] = _Episode(eid, training_enabled)
        return eid

    def _publish(self, ep: _Episode, obs, done: bool):
        with self._ready:
            self._outbox[ep.episode_id] = (obs, ep.reward, done, ep.off_policy_action)
            ep.reward, ep.off_policy_action = 0.0, None
            self._ready.notify_all()

    def get_action(self, episode_id: str, observation):
        ep = self._episodes[episode_id]
        self._publish(ep, observation, False)
        return ep.act_q.get()

    def log_action(self, episode_id: str, observation, action) -> None:
        ep = self._episodes[episode_id]
        ep.off_policy_action = action
        self._publish(ep, observation, False)
        ep.act_q.get()  # the sampler acknowledges with the logged action

    def log_returns(self, episode_id: str, reward: float, info=None) -> None:
        self._episodes[episode_id].reward += float(reward)

    def end_episode(self, episode_id: str, observation) -> None:
        ep = self._episodes.pop(episode_id)
        self._publish(ep, observation, True)

    # --- sampler side ----------------------------------------------------------------------
    def to_base_env(self) -> BaseEnv:
        return _ExternalBaseEnv(self)


class _ExternalBaseEnv(BaseEnv):
    def __init__(self, ext: ExternalEnv, timeout: float = 60.0):
        self.ext, self.timeout = ext, timeout
        self.observation_space, self.action_space = ext.observation_space, ext.action_space
        if not ext.is_alive():
            ext.start()

    def poll(self):
        ext = self.ext
        with ext._ready:
            if not ext._ready.wait_for(lambda: bool(ext._outbox), timeout=self.timeout):
                raise TimeoutError("ExternalEnv produced no observation")
            box, ext._outbox = ext._outbox, {}
        obs, rew, done, info, off = {}, {}, {}, {}, {}
        for eid, (o, r, d, a) in box.items():
            obs[eid] = {_DUMMY_AGENT: o}
            rew[eid] = {_DUMMY_AGENT: r}
            done[eid] = {_DUMMY_AGENT: d, "__all__": d}
            info[eid] = {_DUMMY_AGENT: {}}
            if a is not None:
                off[eid] = {_DUMMY_AGENT: a}
        return obs, rew, done, info, off

    def send_actions(self, action_dict):
        for eid, acts in action_dict.items():
            ep = self.ext._episodes.get(eid)
            if ep is not None:
                ep.act_q.put(acts[_DUMMY_AGENT])
