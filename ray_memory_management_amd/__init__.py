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

__all__ = [
    "__version__", "init", "shutdown", "is_initialized", "remote", "get", "put", "wait", "kill", "cancel",
    "get_actor", "get_gpu_ids", "method", "nodes", "cluster_resources", "available_resources", "timeline",
    "get_runtime_context", "ObjectRef", "ObjectRefGenerator", "ActorHandle", "ActorClass", "exceptions",
    "exit_actor",
]


def __getattr__(name):
    # lazily import heavier subpackages (reference exposes ray.util / ray.data / ...)
    import importlib

    if name in ("util", "data", "train", "tune", "rllib", "serve", "workflow", "dag", "air", "ops",
                "experimental", "models", "parallel", "utils", "internal", "cluster_utils", "job_config"):
        return importlib.import_module(f"ray_memory_management_amd.{name}")
    raise AttributeError(name)
