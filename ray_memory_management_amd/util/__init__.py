"""Utilities. Parity: reference python/ray/util/__init__.py."""
from ray_memory_management_amd.util.placement_group import (  # noqa: F401
    get_current_placement_group, get_placement_group, placement_group, placement_group_table,
    remove_placement_group)
from ray_memory_management_amd.util import scheduling_strategies  # noqa: F401


def __getattr__(name):
    import importlib

    if name == "ActorPool":
        return importlib.import_module("ray_memory_management_amd.util.actor_pool").ActorPool
    if name in ("collective", "queue", "metrics", "multiprocessing", "state", "iter", "actor_pool", "annotations",
                "serialization", "check_serialize", "debug", "accelerators", "rpdb"):
        return importlib.import_module(f"ray_memory_management_amd.util.{name}")
    if name in ("register_serializer", "deregister_serializer"):
        return getattr(importlib.import_module("ray_memory_management_amd.util.serialization"), name)
    if name == "inspect_serializability":
        return importlib.import_module("ray_memory_management_amd.util.check_serialize").inspect_serializability
    if name == "log_once":
        return importlib.import_module("ray_memory_management_amd.util.debug").log_once
    if name == "pdb":
        return importlib.import_module("ray_memory_management_amd.util.rpdb")
    raise AttributeError(name)
