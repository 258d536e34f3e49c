"""Utilities. Parity: reference python/ray/util/__init__.py."""
from ray_memory_management_amd.util.placement_group import (  # noqa: F401
    get_current_placement_group, get_placement_group, placement_group, placement_group_table,
    remove_placement_group)
from ray_memory_management_amd.util import scheduling_strategies  # noqa: F401


def __getattr__(name):
    import importlib

    if name == "ActorPool":
        return importlib.import_module("ray_memory_management_amd.util.actor_pool").ActorPool
    if name in ("collective", "queue", "metrics", "multiprocessing", "state", "iter", "actor_pool", "annotations"):
        return importlib.import_module(f"ray_memory_management_amd.util.{name}")
    raise AttributeError(name)
