"""Compat alias (reference rllib/agents/ppo)."""
from ray_memory_management_amd.rllib.algorithms.ppo import DEFAULT_CONFIG, PPO, PPOConfig  # noqa: F401
