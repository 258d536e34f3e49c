"""RLlib-equivalent reinforcement learning library (PPO first). Parity: reference rllib/."""
from ray_memory_management_amd.rllib.env import (  # noqa: F401
    Box, CartPoleEnv, Discrete, Env, GPUSyntheticAtariVectorEnv, SyntheticAtariEnv, VectorEnv, make_env,
    register_env)
from ray_memory_management_amd.rllib.sample_batch import (  # noqa: F401
    DEFAULT_POLICY_ID, MultiAgentBatch, SampleBatch, concat_samples)


def __getattr__(name):
    import importlib

    if name in ("PPO", "PPOConfig"):
        return getattr(importlib.import_module("ray_memory_management_amd.rllib.ppo"), name)
    if name in ("DQN", "DQNConfig"):
        return getattr(importlib.import_module("ray_memory_management_amd.rllib.algorithms.dqn"), name)
    if name in ("RolloutWorker", "WorkerSet"):
        return getattr(importlib.import_module("ray_memory_management_amd.rllib.rollout_worker"), name)
    raise AttributeError(name)
