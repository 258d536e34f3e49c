"""DAGDriver: the HTTP ingress of a deployment graph.
Parity: reference python/ray/serve/drivers.py (DAGDriver.bind(dag_or_route_dict,
http_adapter=...): one DAG or a {route: dag} table, the adapter converts the request, `predict`
/ `predict_with_route` for handle callers)."""
from __future__ import annotations

import asyncio
import inspect
from typing import Any, Dict, Union

from ray_memory_management_amd.serve.api import deployment
from ray_memory_management_amd.serve.http_adapters import resolve


async def _call(handle, *args, **kwargs):
    return await handle.remote(*args, **kwargs)  # ObjectRefs are awaitable inside the replica's loop


@deployment(route_prefix="/")
class DAGDriver:
    def __init__(self, dags: Union[Any, Dict[str, Any]], http_adapter=None):
        self.adapter = resolve(http_adapter)
        self.routes = dict(dags) if isinstance(dags, dict) else None
        self.dag = None if isinstance(dags, dict) else dags

    async def _adapt(self, request):
        out = self.adapter(request)
        return await out if inspect.isawaitable(out) else out

    async def __call__(self, request):
        inp = await self._adapt(request)
        if self.routes is None:
            return await _call(self.dag, inp)
        path = request.url.path.rstrip("/") or "/"
        for route, h in sorted(self.routes.items(), key=lambda kv: -len(kv[0])):
            if path == route or path.endswith(route):
                return await _call(h, inp)
        from starlette.responses import PlainTextResponse

        return PlainTextResponse(f"no route for {path}; known: {sorted(self.routes)}", status_code=404)

    async def predict(self, *args, **kwargs):
        if self.routes is not None:
            raise ValueError("this driver serves several routes: use predict_with_route")
        return await _call(self.dag, *args, **kwargs)

    async def predict_with_route(self, route: str, *args, **kwargs):
        return await _call(self.routes[route], *args, **kwargs)

    def get_routes(self):
        return sorted(self.routes) if self.routes is not None else ["/"]
