"""Parity: reference rllib/algorithms/registry.py (get_algorithm_class)."""
from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm  # noqa: F401
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig  # noqa: F401


def get_algorithm_class(name: str):
    if name == "PPO":
        from ray_memory_management_amd.rllib.algorithms.ppo import PPO

        return PPO
    raise ValueError(f"Unknown algorithm {name!r}")
