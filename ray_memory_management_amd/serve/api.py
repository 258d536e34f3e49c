"""Serve public API. Parity: reference python/ray/serve/api.py + deployment.py (serve.start /
shutdown / run / deployment decorator / Deployment.deploy / options / bind / get_handle /
delete / get_deployment / list_deployments / ingress / get_replica_context / batch) and
deployment_graph (bind → Application; bound deployments passed as init args become handles).
"""
from __future__ import annotations

import inspect
from typing import Any, Callable, Dict, Optional, Union

import ray_memory_management_amd as ray
from ray_memory_management_amd.serve.config import AutoscalingConfig, DeploymentConfig, HTTPOptions
from ray_memory_management_amd.serve.handle import (CONTROLLER_NAME, SERVE_NAMESPACE, RayServeHandle,
                                                    _HandlePlaceholder)

_state = {"controller": None, "proxy": None, "port": None}


def _get_controller(create: bool = True, http_options=None, detached: bool = False):
    from ray_memory_management_amd.serve.controller import ServeController

    if not ray.is_initialized():
        ray.init()
    if _state["controller"] is not None:
        return _state["controller"]
    try:
        c = ray.get_actor(CONTROLLER_NAME, namespace=SERVE_NAMESPACE)
    except ValueError:
        if not create:
            return None
        opts = dict(name=CONTROLLER_NAME, namespace=SERVE_NAMESPACE, num_cpus=0, max_concurrency=64,
                     get_if_exists=True)
        if detached:
            opts["lifetime"] = "detached"
        c = ray.remote(ServeController).options(**opts).remote(http_options, detached)
        ray.get(c.ping.remote())
    _state["controller"] = c
    return c


def start(detached: bool = False, http_options: Optional[Union[dict, HTTPOptions]] = None, **kw):
    """Start the controller (and the HTTP proxy when http_options has a port)."""
    if isinstance(http_options, HTTPOptions):
        http_options = {"host": http_options.host, "port": http_options.port, "root_path": http_options.root_path}
    c = _get_controller(True, http_options, detached)
    if http_options is not None and http_options.get("port") is not None and http_options.get("location") != "NoServer":
        _start_proxy(http_options.get("host", "127.0.0.1"), http_options.get("port", 8000), detached)
    return c


def _start_proxy(host: str, port: int, detached: bool = False):
    from ray_memory_management_amd.serve.http_proxy import HTTPProxyActor

    if _state["proxy"] is not None:
        return _state["port"]
    opts = dict(name="SERVE_PROXY_ACTOR", namespace=SERVE_NAMESPACE, num_cpus=0, max_concurrency=64,
                get_if_exists=True)
    if detached:  # `serve deploy` from a CLI: the proxy outlives the deploying driver
        opts["lifetime"] = "detached"
    p = ray.remote(HTTPProxyActor).options(**opts).remote(host, port)
    _state["port"] = ray.get(p.ready.remote())
    _state["proxy"] = p
    return _state["port"]


def http_port() -> Optional[int]:
    return _state["port"]


def shutdown():
    c = _state["controller"]
    if c is None:
        try:
            c = ray.get_actor(CONTROLLER_NAME, namespace=SERVE_NAMESPACE)
        except Exception:
            c = None
    if c is not None:
        try:
            ray.get(c.shutdown.remote(), timeout=30)
        except Exception:
            pass
        ray.kill(c)
    if _state["proxy"] is not None:
        try:
            ray.get(_state["proxy"].shutdown.remote(), timeout=5)
        except Exception:
            pass
        ray.kill(_state["proxy"])
    from ray_memory_management_amd.serve.handle import _Router

    _Router._routers.clear()
    _state.update(controller=None, proxy=None, port=None)


class Application:
    """A bound deployment (deployment graph node)."""

    def __init__(self, deployment: "Deployment", args, kwargs):
        self.deployment, self.args, self.kwargs = deployment, args, kwargs

    def _collect(self, out: Dict[str, "Application"]):
        def walk(a):  # bound deployments may be nested in lists / tuples / dicts (DAGDriver routes)
            if isinstance(a, Application):
                a._collect(out)
            elif isinstance(a, (list, tuple)):
                for x in a:
                    walk(x)
            elif isinstance(a, dict):
                for x in a.values():
                    walk(x)

        for a in list(self.args) + list(self.kwargs.values()):
            walk(a)
        out[self.deployment.name] = self
        return out


def _placeholders(obj):
    if isinstance(obj, Application):
        return _HandlePlaceholder(obj.deployment.name)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_placeholders(x) for x in obj)
    if isinstance(obj, dict):
        return {k: _placeholders(v) for k, v in obj.items()}
    return obj


class Deployment:
    def __init__(self, func_or_class, name: str, config: DeploymentConfig, version: Optional[str] = None,
                 init_args=(), init_kwargs=None, route_prefix: Optional[str] = None,
                 ray_actor_options: Optional[dict] = None, ingress_app=None, _internal=False):
        if not _internal:
            raise RuntimeError("The Deployment constructor should not be called directly. Use `@serve.deployment` "
                               "instead.")
        self.func_or_class = func_or_class
        self._name = name
        self._config = config
        self._version = version
        self._init_args = tuple(init_args or ())
        self._init_kwargs = dict(init_kwargs or {})
        if route_prefix is not None and route_prefix != "/" and (not route_prefix.startswith("/") or
                                                                 route_prefix.endswith("/")):
            if not route_prefix.startswith("/"):
                raise ValueError("The route_prefix must start with a forward slash ('/')")
            if route_prefix.endswith("/"):
                raise ValueError("The route_prefix cannot end with a forward slash ('/')")
        self._route_prefix = route_prefix if route_prefix is not None else f"/{name}"
        self._ray_actor_options = dict(ray_actor_options or {})
        self._ingress_app = ingress_app or getattr(func_or_class, "_serve_asgi_app", None)

    # ---- properties
    @property
    def name(self):
        return self._name

    @property
    def version(self):
        return self._version

    @property
    def num_replicas(self):
        return self._config.num_replicas

    @property
    def user_config(self):
        return self._config.user_config

    @property
    def max_concurrent_queries(self):
        return self._config.max_concurrent_queries

    @property
    def route_prefix(self):
        return self._route_prefix

    @property
    def ray_actor_options(self):
        return self._ray_actor_options

    @property
    def init_args(self):
        return self._init_args

    @property
    def init_kwargs(self):
        return self._init_kwargs

    @property
    def url(self):
        port = _state["port"] or 8000
        return f"http://127.0.0.1:{port}{self._route_prefix}" if self._route_prefix else None

    # ---- API
    def options(self, func_or_class=None, name=None, version=None, init_args=None, init_kwargs=None,
                route_prefix=-1, num_replicas=None, ray_actor_options=None, user_config=None,
                max_concurrent_queries=None, autoscaling_config=None, graceful_shutdown_timeout_s=None,
                health_check_period_s=None, health_check_timeout_s=None, **kw) -> "Deployment":
        import copy

        cfg = copy.deepcopy(self._config)
        if num_replicas is not None:
            if autoscaling_config is not None:
                raise ValueError("Manually setting num_replicas is not allowed when autoscaling_config is provided.")
            cfg.num_replicas = num_replicas
        if user_config is not None:
            cfg.user_config = user_config
        if max_concurrent_queries is not None:
            cfg.max_concurrent_queries = max_concurrent_queries
        if autoscaling_config is not None:
            cfg.autoscaling_config = autoscaling_config if isinstance(autoscaling_config, AutoscalingConfig) \
                else AutoscalingConfig(**autoscaling_config)
        for k, v in (("graceful_shutdown_timeout_s", graceful_shutdown_timeout_s),
                     ("health_check_period_s", health_check_period_s),
                     ("health_check_timeout_s", health_check_timeout_s)):
            if v is not None:
                setattr(cfg, k, v)
        new_name = name or self._name
        rp = self._route_prefix if route_prefix == -1 else route_prefix
        if name is not None and route_prefix == -1 and self._route_prefix == f"/{self._name}":
            rp = f"/{name}"
        return Deployment(func_or_class or self.func_or_class, new_name, cfg, version or self._version,
                          init_args if init_args is not None else self._init_args,
                          init_kwargs if init_kwargs is not None else self._init_kwargs, rp,
                          ray_actor_options if ray_actor_options is not None else self._ray_actor_options,
                          self._ingress_app, _internal=True)

    def set_options(self, **kw):
        d = self.options(**kw)
        self.__dict__.update(d.__dict__)

    def bind(self, *args, **kwargs) -> Application:
        return Application(self, args, kwargs)

    def deploy(self, *init_args, _blocking: bool = True, **init_kwargs):
        if init_args or init_kwargs:
            return self.options(init_args=init_args, init_kwargs=init_kwargs).deploy(_blocking=_blocking)
        c = _get_controller()
        spec = {"func_or_class": self.func_or_class, "init_args": _placeholders(self._init_args),
                "init_kwargs": _placeholders(self._init_kwargs), "config": self._config, "version": self._version,
                "route_prefix": self._route_prefix, "ray_actor_options": self._ray_actor_options,
                "ingress_app": self._ingress_app}
        ray.get(c.deploy.remote(self._name, spec))
        if _blocking:
            ray.get(c.wait_ready.remote(self._name, 120.0))
        return None

    def delete(self):
        c = _get_controller(create=False)
        if c is not None:
            ray.get(c.delete_deployment.remote(self._name))
            ray.get(c.wait_deleted.remote(self._name, 60.0))

    def get_handle(self, sync: bool = True) -> RayServeHandle:
        return RayServeHandle(self._name, _sync=sync)

    def __call__(self, *a, **k):
        raise RuntimeError("Deployments cannot be constructed directly. Use `deployment.deploy()` instead.")

    def __repr__(self):
        return f"Deployment(name={self._name}, version={self._version}, route_prefix={self._route_prefix})"


def deployment(_func_or_class=None, name: Optional[str] = None, version: Optional[str] = None,
               num_replicas: Optional[int] = None, init_args=None, init_kwargs=None, route_prefix=-1,
               ray_actor_options: Optional[dict] = None, user_config=None, max_concurrent_queries: Optional[int] = None,
               autoscaling_config=None, graceful_shutdown_timeout_s=None, health_check_period_s=None,
               health_check_timeout_s=None, **kw):
    if num_replicas is not None and autoscaling_config is not None:
        raise ValueError("Manually setting num_replicas is not allowed when autoscaling_config is provided.")
    if num_replicas == 0:
        raise ValueError("num_replicas is expected to larger than 0")

    def deco(fc):
        cfg = DeploymentConfig()
        if num_replicas is not None:
            cfg.num_replicas = num_replicas
        if user_config is not None:
            cfg.user_config = user_config
        if max_concurrent_queries is not None:
            cfg.max_concurrent_queries = max_concurrent_queries
        if autoscaling_config is not None:
            cfg.autoscaling_config = autoscaling_config if isinstance(autoscaling_config, AutoscalingConfig) \
                else AutoscalingConfig(**autoscaling_config)
        for k, v in (("graceful_shutdown_timeout_s", graceful_shutdown_timeout_s),
                     ("health_check_period_s", health_check_period_s),
                     ("health_check_timeout_s", health_check_timeout_s)):
            if v is not None:
                setattr(cfg, k, v)
        nm = name or fc.__name__
        return Deployment(fc, nm, cfg, version, init_args, init_kwargs,
                          None if route_prefix == -1 else route_prefix, ray_actor_options, _internal=True)

    return deco(_func_or_class) if callable(_func_or_class) else deco


def ingress(app):
    """Mark a class deployment as serving an ASGI (FastAPI / Starlette) app."""

    from ray_memory_management_amd.serve.replica import IngressSpec

    def deco(cls):
        # ship the route table, not the app object (FastAPI apps do not pickle); each replica
        # rebuilds the app around its own instance
        cls._serve_asgi_app = IngressSpec.from_app(app)
        return cls

    return deco


def run(target: Union[Application, Deployment], _blocking: bool = True, *, host: str = "127.0.0.1",
        port: Optional[int] = None, route_prefix: Optional[str] = "/", name: str = "default") -> RayServeHandle:
    """Deploy an application (a bound deployment graph) and return a handle to its ingress."""
    if isinstance(target, Deployment):
        target = target.bind()
    start(http_options={"host": host, "port": port} if port is not None else None)
    nodes = target._collect({})
    ingress_name = target.deployment.name
    for dname, node in nodes.items():
        d = node.deployment
        rp = route_prefix if dname == ingress_name else None
        if dname == ingress_name and route_prefix is None:
            rp = d.route_prefix
        d = d.options(init_args=node.args, init_kwargs=node.kwargs, route_prefix=rp)
        d.deploy(_blocking=False)
    c = _get_controller()
    for dname in nodes:
        ray.get(c.wait_ready.remote(dname, 120.0))
    return RayServeHandle(ingress_name)


def get_deployment(name: str) -> Deployment:
    c = _get_controller(create=False)
    spec = ray.get(c.get_deployment_spec.remote(name)) if c is not None else None
    if spec is None:
        raise KeyError(f"Deployment {name} was not found. Did you call Deployment.deploy()?")
    return Deployment(spec["func_or_class"], name, spec["config"], spec.get("version"), spec.get("init_args"),
                      spec.get("init_kwargs"), spec.get("route_prefix"), spec.get("ray_actor_options"),
                      spec.get("ingress_app"), _internal=True)


def list_deployments() -> Dict[str, Deployment]:
    c = _get_controller(create=False)
    if c is None:
        return {}
    return {n: get_deployment(n) for n in ray.get(c.list_deployments.remote())}


def status() -> Dict[str, dict]:
    c = _get_controller(create=False)
    return ray.get(c.list_deployments.remote()) if c is not None else {}


def delete(name: str, _blocking: bool = True):
    c = _get_controller(create=False)
    if c is not None:
        ray.get(c.delete_deployment.remote(name))
        if _blocking:
            ray.get(c.wait_deleted.remote(name, 60.0))


def get_deployment_handle(name: str) -> RayServeHandle:
    return RayServeHandle(name)
