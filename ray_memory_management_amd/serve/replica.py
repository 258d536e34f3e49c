"""Replica actor: hosts one copy of a deployment's callable.

Parity: reference python/ray/serve/_private/replica.py (RayServeReplica: handle_request with
max_concurrent_queries, reconfigure(user_config), check_health, prepare_for_shutdown, ongoing
request metrics) and http_util.py (ASGI request/response plumbing).

The replica is an async actor: async user methods run on its event loop (so @serve.batch can
coalesce concurrent calls); sync methods run on a thread pool so they do not serialise the loop.
HTTP requests arrive as (ASGI scope, body) and are executed through ASGI here, so FastAPI
ingress apps and plain `__call__(request)` deployments share one path.
"""
from __future__ import annotations

import asyncio
import inspect
import json
import time
from typing import Any, Dict, List, Optional, Tuple

from ray_memory_management_amd.serve.context import ReplicaContext, _set_replica_context


class ServeReplica:
    def __init__(self, deployment_name: str, replica_tag: str, func_or_class, init_args, init_kwargs,
                 user_config=None, ingress_app=None):
        from ray_memory_management_amd.serve.handle import _resolve_handles

        self._name, self._tag = deployment_name, replica_tag
        init_args = _resolve_handles(init_args)
        init_kwargs = _resolve_handles(init_kwargs)
        if inspect.isclass(func_or_class):
            self._callable = func_or_class(*init_args, **init_kwargs)
            self._is_function = False
        else:
            self._callable = func_or_class
            self._is_function = True
        self._ingress_app = ingress_app
        if ingress_app is not None:
            self._ingress_app = _bind_ingress_instance(ingress_app, None if self._is_function else self._callable)
        _set_replica_context(ReplicaContext(deployment_name, replica_tag, self._callable))
        self._ongoing = 0
        self._total = 0
        self._user_config = None
        if user_config is not None:
            self._reconfigure_sync(user_config)

    def _reconfigure_sync(self, user_config):
        self._user_config = user_config
        fn = getattr(self._callable, "reconfigure", None)
        if fn is None:
            raise ValueError("user_config specified but deployment doesn't have a reconfigure method")
        r = fn(user_config)
        if inspect.iscoroutine(r):
            asyncio.get_event_loop().run_until_complete(r) if not asyncio.get_event_loop().is_running() else None

    async def reconfigure(self, user_config):
        self._user_config = user_config
        fn = getattr(self._callable, "reconfigure", None)
        if fn is None:
            raise ValueError("user_config specified but deployment doesn't have a reconfigure method")
        r = fn(user_config)
        if inspect.iscoroutine(r):
            await r
        return True

    async def ready(self):
        return self._tag

    async def check_health(self):
        fn = getattr(self._callable, "check_health", None)
        if fn is not None:
            r = fn()
            if inspect.iscoroutine(r):
                await r
        return True

    async def get_metrics(self):
        return {"ongoing": self._ongoing, "total": self._total}

    async def _call(self, fn, args, kwargs):
        if inspect.iscoroutinefunction(fn) or getattr(fn, "_serve_batch", False):
            return await fn(*args, **kwargs)
        loop = asyncio.get_event_loop()
        r = await loop.run_in_executor(None, lambda: fn(*args, **kwargs))
        if inspect.iscoroutine(r):
            r = await r
        return r

    async def handle_request(self, method_name: str, args, kwargs):
        self._ongoing += 1
        self._total += 1
        try:
            if self._is_function:
                fn = self._callable
            else:
                fn = getattr(self._callable, method_name or "__call__")
            return await self._call(fn, list(args), dict(kwargs))
        finally:
            self._ongoing -= 1

    async def handle_http(self, scope: Dict, body: bytes) -> Tuple[int, List, bytes]:
        """Run one HTTP request through ASGI; returns (status, headers, body)."""
        self._ongoing += 1
        self._total += 1
        try:
            sent = {"status": 500, "headers": [], "body": b""}

            async def receive():
                return {"type": "http.request", "body": body, "more_body": False}

            async def send(msg):
                if msg["type"] == "http.response.start":
                    sent["status"] = msg["status"]
                    sent["headers"] = [(bytes(k), bytes(v)) for k, v in msg.get("headers", [])]
                elif msg["type"] == "http.response.body":
                    sent["body"] += msg.get("body", b"")

            if self._ingress_app is not None:
                await self._ingress_app(scope, receive, send)
                return sent["status"], sent["headers"], sent["body"]
            from starlette.requests import Request

            req = Request(scope, receive)
            fn = self._callable if self._is_function else getattr(self._callable, "__call__")
            try:
                result = await self._call(fn, [req], {})
            except Exception as e:  # surface as 500 like the reference proxy
                import traceback

                return 500, [(b"content-type", b"text/plain")], traceback.format_exc().encode()
            await _to_response(result)(scope, receive, send)
            return sent["status"], sent["headers"], sent["body"]
        finally:
            self._ongoing -= 1

    async def prepare_for_shutdown(self, timeout_s: float = 2.0):
        t0 = time.time()
        while self._ongoing > 0 and time.time() - t0 < timeout_s:
            await asyncio.sleep(0.02)
        fn = getattr(self._callable, "__del__", None)
        return True


def _to_response(result):
    from starlette.responses import JSONResponse, PlainTextResponse, Response

    if isinstance(result, Response):
        return result
    if isinstance(result, (bytes, bytearray)):
        return Response(bytes(result), media_type="application/octet-stream")
    if isinstance(result, str):
        return PlainTextResponse(result)
    try:
        import numpy as np

        if isinstance(result, np.ndarray):
            result = result.tolist()
        elif isinstance(result, np.generic):
            result = result.item()
    except ImportError:  # pragma: no cover
        pass
    return JSONResponse(result)


class IngressSpec:
    """Picklable description of a FastAPI app: its API routes (path, endpoint, methods, ...)."""

    def __init__(self, title, routes):
        self.title, self.routes = title, routes

    @classmethod
    def from_app(cls, app):
        from fastapi.routing import APIRoute

        routes = []
        for r in app.routes:
            if isinstance(r, APIRoute):
                routes.append(dict(path=r.path, endpoint=r.endpoint, methods=sorted(r.methods or ["GET"]),
                                   status_code=r.status_code, name=r.name))
        return cls(getattr(app, "title", "FastAPI"), routes)

    def build(self, instance=None):
        import functools

        from fastapi import FastAPI

        app = FastAPI(title=self.title)
        for r in self.routes:
            ep = r["endpoint"]
            params = list(inspect.signature(ep).parameters.values())
            if instance is not None and params and params[0].name == "self":
                bound = functools.partial(ep, instance)
                functools.update_wrapper(bound, ep)
                bound.__signature__ = inspect.signature(ep).replace(parameters=params[1:])
                ep = bound
            app.add_api_route(r["path"], ep, methods=r["methods"], status_code=r["status_code"], name=r["name"])
        return app


def _bind_ingress_instance(app, instance):
    if isinstance(app, IngressSpec):
        return app.build(instance)
    """@serve.ingress(FastAPI app) on a class: build a per-replica app whose routes call the
    replica's instance methods (reference api.py ingress: class-based views)."""
    import functools

    try:
        from fastapi import FastAPI
        from fastapi.routing import APIRoute
    except ImportError:  # pragma: no cover
        return app
    if not isinstance(app, FastAPI):
        return app
    new = FastAPI(title=app.title)
    for r in app.routes:
        if isinstance(r, APIRoute):
            ep = r.endpoint
            params = list(inspect.signature(ep).parameters)
            if params and params[0] == "self":
                ep = functools.partial(ep, instance)
                functools.update_wrapper(ep, r.endpoint)
                ep.__signature__ = inspect.signature(r.endpoint).replace(
                    parameters=list(inspect.signature(r.endpoint).parameters.values())[1:])
            new.add_api_route(r.path, ep, methods=list(r.methods or ["GET"]), response_model=r.response_model,
                              status_code=r.status_code, name=r.name)
        else:
            new.router.routes.append(r)
    return new
