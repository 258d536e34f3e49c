"""Compat alias."""
from ray_memory_management_amd.rllib.evaluation import RolloutWorker, WorkerSet  # noqa: F401
