"""ray_memory_management_amd — an MI355X-native distributed runtime with Ray's task / actor /
object API (``init``, ``@remote``, ``get``/``put``/``wait``), a native shared-memory object store
with spilling, an HBM GPU object store, RCCL collectives and the Train / Tune / RLlib / Data /
Serve / Workflow libraries.

Usage mirrors the reference: ``import ray_memory_management_amd as ray``.
"""
from __future__ import annotations

__version__ = "0.1.0"

from ray_memory_management_amd import exceptions  # noqa: F401
from ray_memory_management_amd._private.ids import (  # noqa: F401
    ActorID, FunctionID, JobID, NodeID, ObjectID, PlacementGroupID, TaskID, UniqueID, WorkerID)
from ray_memory_management_amd._private.worker import (  # noqa: F401
    LOCAL_MODE, SCRIPT_MODE, WORKER_MODE, available_resources, cancel, cluster_resources, get, get_actor,
    get_gpu_ids, init, is_initialized, kill, nodes, put, remote, shutdown, timeline, wait)
from ray_memory_management_amd.actor import ActorClass, ActorHandle, exit_actor, method  # noqa: F401
from ray_memory_management_amd.object_ref import ObjectRef, ObjectRefGenerator  # noqa: F401
from ray_memory_management_amd.remote_function import RemoteFunction  # noqa: F401
from ray_memory_management_amd.runtime_context import get_runtime_context  # noqa: F401
from ray_memory_management_amd.client_builder import ClientBuilder, client  # noqa: F401
from ray_memory_management_amd.cross_language import (  # noqa: F401
    Language, cpp_function, java_actor_class, java_function)
from ray_memory_management_amd._private.ids import ActorClassID  # noqa: F401

__all__ = [
    "__version__", "init", "shutdown", "is_initialized", "remote", "get", "put", "wait", "kill", "cancel",
    "get_actor", "get_gpu_ids", "method", "nodes", "cluster_resources", "available_resources", "timeline",
    "get_runtime_context", "ObjectRef", "ObjectRefGenerator", "ActorHandle", "ActorClass", "exceptions",
    "exit_actor", "client", "ClientBuilder", "Language", "java_function", "java_actor_class", "cpp_function",
    "show_in_dashboard", "_config", "LOCAL_MODE", "SCRIPT_MODE", "WORKER_MODE",
]


def show_in_dashboard(message: str, key: str = "", dtype: str = "text") -> None:
    """Publish a message for this actor / task in the dashboard (reference ray.show_in_dashboard):
    stored in the internal KV under the current actor's (or driver's) id and served by the
    dashboard's state endpoints."""
    if dtype not in ("text", "html"):
        raise ValueError("dtype accepts only: text, html")
    import json

    from ray_memory_management_amd import internal

    ctx = get_runtime_context()
    owner = ctx.get_actor_id() or "driver"
    internal._internal_kv_put(f"dashboard_msg:{owner}:{key}",
                              json.dumps({"message": message, "dtype": dtype}).encode(), overwrite=True,
                              namespace="dashboard")


class _SystemConfig:
    """`ray._config`: read access to the system config of the running cluster (reference
    ray._config = the RayConfig singleton)."""

    def __getattr__(self, name):
        from ray_memory_management_amd._private import worker as _w

        cfg = _w._system_config_used
        if name in cfg:
            return cfg[name]
        raise AttributeError(name)


_config = _SystemConfig()


def __getattr__(name):
    # lazily import heavier subpackages (reference exposes ray.util / ray.data / ...)
    import importlib

    if name in ("util", "data", "train", "tune", "rllib", "serve", "workflow", "dag", "air", "ops",
                "experimental", "models", "parallel", "utils", "internal", "cluster_utils", "job_config",
                "autoscaler", "widgets", "dashboard", "job_submission", "scripts"):
        return importlib.import_module(f"ray_memory_management_amd.{name}")
    raise AttributeError(name)
