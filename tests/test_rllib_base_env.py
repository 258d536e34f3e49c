"""BaseEnv / ExternalEnv / Policy API. Mirrors reference rllib/env/tests/test_external_env.py
(an application-driven env sampled through poll / send_actions) and base_env conversion tests."""
import numpy as np
import pytest

from ray_memory_management_amd import rllib
from ray_memory_management_amd.rllib.base_env import convert_to_base_env
from ray_memory_management_amd.rllib.env import CartPoleEnv, MultiAgentCartPole, VectorEnv


class CartPoleServing(rllib.ExternalEnv):
    def __init__(self, episodes):
        env = CartPoleEnv()
        super().__init__(env.action_space, env.observation_space)
        self.env, self.episodes, self.returns = env, episodes, []

    def run(self):
        for k in range(self.episodes):
            eid = self.start_episode()
            obs, total, done = self.env.reset(), 0.0, False
            while not done:
                if k % 2:  # odd episodes: the application picks the action and logs it
                    a = int(obs[2] > 0)
                    self.log_action(eid, obs, a)
                else:
                    a = self.get_action(eid, obs)
                obs, r, done, _ = self.env.step(a)
                self.log_returns(eid, r)
                total += r
            self.end_episode(eid, obs)
            self.returns.append(total)


def test_external_env_sampled_through_base_env():
    ext = CartPoleServing(episodes=4)
    base = convert_to_base_env(ext)
    policy_rng = np.random.default_rng(0)
    rewards, off_policy, finished = 0.0, 0, 0
    while finished < 4:
        obs, rew, done, info, off = base.poll()
        acts = {}
        for eid, o in obs.items():
            rewards += rew[eid]["agent0"]
            if done[eid]["__all__"]:
                finished += 1
                continue
            if eid in off:
                off_policy += 1
                acts[eid] = {"agent0": off[eid]["agent0"]}
            else:
                acts[eid] = {"agent0": int(policy_rng.integers(2))}
        base.send_actions(acts)
    ext.join(timeout=10)
    assert len(ext.returns) == 4 and abs(rewards - sum(ext.returns)) < 1e-6 and off_policy > 0


def test_convert_vector_and_multi_agent_envs():
    v = convert_to_base_env(VectorEnv(lambda i: CartPoleEnv(), 3))
    obs, rew, done, _, _ = v.poll()
    assert sorted(obs) == [0, 1, 2] and not done[0]["__all__"]
    v.send_actions({i: {"agent0": 0} for i in obs})
    obs2, rew2, _, _, _ = v.poll()
    assert sorted(obs2) == [0, 1, 2] and rew2[1]["agent0"] == 1.0
    m = convert_to_base_env(MultiAgentCartPole({"num_agents": 2}))
    obs, _, _, _, _ = m.poll()
    assert sorted(obs[0]) == [0, 1]
    m.send_actions({0: {0: 1, 1: 0}})
    obs, rew, done, _, _ = m.poll()
    assert set(rew[0]) == {0, 1} and done[0]["__all__"] is False


def test_policy_base_classes():
    env = CartPoleEnv()
    p = rllib.TorchPolicy(env.observation_space, env.action_space, {})
    assert isinstance(p, rllib.Policy)
    st = p.get_state()
    p.set_state(st)
    assert p.compute_single_action(env.reset()) in (0, 1)
    with pytest.raises(ImportError):
        rllib.TFPolicy(env.observation_space, env.action_space, {})
