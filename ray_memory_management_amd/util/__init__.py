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
    if name in ("disable_log_once_globally", "enable_periodic_logging"):
        return getattr(importlib.import_module("ray_memory_management_amd.util.debug"), name)
    if name in ("connect", "disconnect"):
        return globals()["_client_" + name]
    raise AttributeError(name)


def get_node_ip_address(address: str = "127.0.0.1:80") -> str:
    """IP of this node as other nodes see it (reference ray.util.get_node_ip_address): the source
    address the kernel picks toward `address` (no packet is sent); loopback on a single node."""
    import socket

    host, _, port = address.rpartition(":")
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        s.connect((host or "127.0.0.1", int(port or 80)))
        return s.getsockname()[0]
    except OSError:
        return "127.0.0.1"
    finally:
        s.close()


def list_named_actors(all_namespaces: bool = False):
    """Names of live named actors: in the current namespace, or every namespace as
    {"name", "namespace"} dicts (reference ray.util.list_named_actors)."""
    from ray_memory_management_amd.runtime_context import get_runtime_context
    from ray_memory_management_amd.util import state

    live = [a for a in state.list_actors() if a.get("name") and a.get("state") != "DEAD"]
    if all_namespaces:
        return [{"name": a["name"], "namespace": a["namespace"]} for a in live]
    ns = get_runtime_context().namespace
    return [a["name"] for a in live if a["namespace"] == ns]


def _client_connect(conn_str: str, namespace=None, **_kw):
    """ray.util.connect (legacy Ray Client entry): same as ray.init("ray://...")."""
    from ray_memory_management_amd._private import worker

    return worker.init(conn_str if conn_str.startswith("ray://") else "ray://" + conn_str, namespace=namespace)


def _client_disconnect():
    from ray_memory_management_amd._private import worker

    worker.shutdown()
