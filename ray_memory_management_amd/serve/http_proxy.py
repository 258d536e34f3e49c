"""HTTP ingress. Parity: reference python/ray/serve/_private/http_proxy.py (uvicorn ASGI server
in an actor; longest-prefix route matching against the controller's route table; request
forwarded to a replica; 404 for unknown routes) and http_util.py.

The proxy forwards (ASGI scope, body) and the replica runs the request through ASGI itself
(see replica.py), so the proxy never needs user code."""
from __future__ import annotations

import asyncio
import threading
import time
from typing import Dict, Optional

import ray_memory_management_amd as ray
from ray_memory_management_amd.serve.handle import _controller, _Router

_SCOPE_KEYS = ("type", "asgi", "http_version", "method", "scheme", "path", "raw_path", "root_path", "query_string",
               "headers", "server", "client")


class HTTPProxyActor:
    def __init__(self, host: str = "127.0.0.1", port: int = 8000, root_path: str = ""):
        self.host, self.port, self.root_path = host, port, root_path
        self._routes: Dict[str, str] = {}
        self._routes_t = 0.0
        self._started = threading.Event()
        self._error: Optional[BaseException] = None
        self._t = threading.Thread(target=self._serve, daemon=True, name="serve-http")
        self._t.start()

    def _serve(self):
        import uvicorn

        try:
            config = uvicorn.Config(self._app, host=self.host, port=self.port, log_level="warning", lifespan="off",
                                    access_log=False)
            self._server = uvicorn.Server(config)
            loop = asyncio.new_event_loop()
            asyncio.set_event_loop(loop)

            async def watch():
                while not self._server.started:
                    await asyncio.sleep(0.01)
                for s in getattr(self._server, "servers", []) or []:
                    for sock in s.sockets:
                        self.port = sock.getsockname()[1]
                self._started.set()

            async def run():
                w = asyncio.ensure_future(watch())
                await self._server.serve()
                w.cancel()

            loop.run_until_complete(run())
        except BaseException as e:  # noqa: B902
            self._error = e
            self._started.set()

    def ready(self):
        self._started.wait(30)
        if self._error is not None:
            raise self._error
        return self.port

    def _route_for(self, path: str):
        now = time.time()
        if now - self._routes_t > 0.2:
            self._routes = ray.get(_controller().get_route_table.remote())
            self._routes_t = now
        best = None
        for prefix, name in self._routes.items():
            p = prefix.rstrip("/") or "/"
            if path == p or path.startswith(p if p.endswith("/") else p + "/") or p == "/":
                if best is None or len(p) > len(best[0]):
                    best = (p, name)
        return best

    @property
    def _app(self):
        # a closure, not an `async def` method: the actor must stay a plain threaded actor
        async def app(scope, receive, send):
            try:
                await _asgi(self, scope, receive, send)
            except Exception:
                import traceback

                await send({"type": "http.response.start", "status": 500,
                            "headers": [(b"content-type", b"text/plain")]})
                await send({"type": "http.response.body", "body": traceback.format_exc().encode()})

        return app

    def _forward(self, name, scope, body):
        r = _Router.get(name)
        last = None
        for _ in range(3):
            i = r.choose()
            try:
                ref = r.replicas[i].handle_http.remote(scope, body)
                r.record(i, ref)
                return ray.get(ref)
            except Exception as e:  # replica died: refresh and retry
                last = e
                r.refresh(force=True)
        import traceback

        return 500, [(b"content-type", b"text/plain")], "".join(traceback.format_exception_only(type(last), last)
                                                                 ).encode()

    def shutdown(self):
        if getattr(self, "_server", None) is not None:
            self._server.should_exit = True
        return True


async def _asgi(self, scope, receive, send):
        if scope["type"] != "http":
            return
        path = scope.get("path", "/")
        loop = asyncio.get_event_loop()
        route = await loop.run_in_executor(None, self._route_for, path)
        if route is None:
            body = f'Path "{path}" not found. Please ping http://.../-/routes for route table.'.encode()
            await send({"type": "http.response.start", "status": 404,
                        "headers": [(b"content-type", b"text/plain")]})
            await send({"type": "http.response.body", "body": body})
            return
        prefix, name = route
        chunks = []
        more = True
        while more:
            msg = await receive()
            chunks.append(msg.get("body", b""))
            more = msg.get("more_body", False)
        fwd = {k: scope[k] for k in _SCOPE_KEYS if k in scope}
        fwd["headers"] = [(bytes(k), bytes(v)) for k, v in scope.get("headers", [])]
        fwd["root_path"] = (prefix if prefix != "/" else "")
        status, headers, body = await loop.run_in_executor(None, self._forward, name, fwd, b"".join(chunks))
        await send({"type": "http.response.start", "status": status, "headers": headers})
        await send({"type": "http.response.body", "body": body})
