"""Parity: reference rllib/algorithms/registry.py (get_algorithm_class)."""
import importlib

from ray_memory_management_amd.rllib.algorithms.algorithm import Algorithm  # noqa: F401
from ray_memory_management_amd.rllib.algorithms.algorithm_config import AlgorithmConfig  # noqa: F401

ALGORITHMS = {
    "PPO": ("ppo", "PPO"),
    "DQN": ("dqn", "DQN"),
    "IMPALA": ("impala", "Impala"),
    "APPO": ("appo", "APPO"),
    "PG": ("pg", "PG"),
    "A2C": ("a2c", "A2C"),
    "MARWIL": ("marwil", "MARWIL"),
    "BC": ("bc", "BC"),
    "DDPG": ("ddpg", "DDPG"),
    "TD3": ("td3", "TD3"),
    "SAC": ("sac", "SAC"),
    "SimpleQ": ("simple_q", "SimpleQ"),
    "APEX": ("apex_dqn", "ApexDQN"),
    "APEX_DDPG": ("apex_ddpg", "ApexDDPG"),
    "A3C": ("a3c", "A3C"),
    "R2D2": ("r2d2", "R2D2"),
    "DT": ("dt", "DT"),
    "AlphaZero": ("alpha_zero", "AlphaZero"),
    "SlateQ": ("slateq", "SlateQ"),
    "MAML": ("maml", "MAML"),
    "Dreamer": ("dreamer", "Dreamer"),
    "MBMPO": ("mbmpo", "MBMPO"),
    "AlphaStar": ("alpha_star", "AlphaStar"),
    "QMIX": ("qmix", "QMix"),
    "MADDPG": ("maddpg", "MADDPG"),
    "CQL": ("cql", "CQL"),
    "CRR": ("crr", "CRR"),
    "DDPPO": ("ddppo", "DDPPO"),
    "ES": ("es", "ES"),
    "ARS": ("ars", "ARS"),
    "BanditLinUCB": ("bandit", "BanditLinUCB"),
    "BanditLinTS": ("bandit", "BanditLinTS"),
}


def get_algorithm_class(name: str):
    if name not in ALGORITHMS:
        raise ValueError(f"Unknown algorithm {name!r}")
    mod, cls = ALGORITHMS[name]
    return getattr(importlib.import_module(f"ray_memory_management_amd.rllib.algorithms.{mod}"), cls)
