"""Serializers for third-party types that plain pickling handles badly, registered on demand.

Role parity: reference python/ray/util/serialization_addons.py (``apply`` registers pydantic model
classes and starlette requests so Serve can pass them between processes). Here they go through the
runtime's custom-serializer registry (util/serialization.py): pydantic models travel as
(class, field dict), starlette requests as (scope, body).
"""
from __future__ import annotations


def register_pydantic_serializer(serialization_context=None) -> bool:
    try:
        import pydantic
    except ImportError:
        return False
    from ray_memory_management_amd.util.serialization import register_serializer

    def _ser(m):
        return type(m), m.model_dump() if hasattr(m, "model_dump") else m.dict()

    def _de(v):
        cls, fields = v
        return cls(**fields)

    register_serializer(pydantic.BaseModel, serializer=_ser, deserializer=_de)
    return True


def register_starlette_serializer(serialization_context=None) -> bool:
    try:
        from starlette.requests import Request
    except ImportError:
        return False
    from ray_memory_management_amd.util.serialization import register_serializer

    def _ser(req):
        scope = {k: v for k, v in req.scope.items() if k not in ("app", "router", "endpoint", "state")}
        return scope, getattr(req, "_body", b"")

    def _de(v):
        scope, body = v

        async def receive():
            return {"type": "http.request", "body": body, "more_body": False}

        return Request(scope, receive)

    register_serializer(Request, serializer=_ser, deserializer=_de)
    return True


def apply(serialization_context=None) -> None:
    register_pydantic_serializer(serialization_context)
    register_starlette_serializer(serialization_context)


__all__ = ["apply", "register_pydantic_serializer", "register_starlette_serializer"]
