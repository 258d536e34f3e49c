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
    if name in ("Policy", "TorchPolicy", "TFPolicy"):
        return getattr(importlib.import_module("ray_memory_management_amd.rllib.policy"), name)
    if name in ("BaseEnv", "ExternalEnv", "convert_to_base_env"):
        return getattr(importlib.import_module("ray_memory_management_amd.rllib.base_env"), name)
    if name == "MultiAgentEnv":
        return importlib.import_module("ray_memory_management_amd.rllib.env").MultiAgentEnv
    if name in ("RolloutWorker", "WorkerSet"):
        return getattr(importlib.import_module("ray_memory_management_amd.rllib.rollout_worker"), name)
    raise AttributeError(name)
