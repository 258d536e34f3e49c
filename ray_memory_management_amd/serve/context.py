"""Replica context. Parity: reference python/ray/serve/context.py (get_replica_context:
deployment, replica_tag, servable_object)."""
from __future__ import annotations

import dataclasses
from typing import Any, Optional


@dataclasses.dataclass
class ReplicaContext:
    deployment: str
    replica_tag: str
    servable_object: Any = None
    app_name: str = "default"


_ctx: Optional[ReplicaContext] = None


def _set_replica_context(ctx: Optional[ReplicaContext]):
    global _ctx
    _ctx = ctx


def get_replica_context() -> ReplicaContext:
    if _ctx is None:
        from ray_memory_management_amd.serve.exceptions import RayServeException

        raise RayServeException("`serve.get_replica_context()` may only be called from within a Ray Serve "
                                "deployment.")
    return _ctx
