"""RayServeHandle: call a deployment from Python.

Parity: reference python/ray/serve/handle.py (RayServeHandle / RayServeSyncHandle: .remote()
returns an ObjectRef, .options(method_name=...), attribute access `handle.method.remote()`,
picklable so handles can be passed to other deployments) and _private/router.py (replica set
from the controller, power-of-two-choices on in-flight counts, retry on replica failure).
"""
from __future__ import annotations

import random
import threading
import time
from typing import Any, Dict, List, Optional

import ray_memory_management_amd as ray

CONTROLLER_NAME = "SERVE_CONTROLLER_ACTOR"
SERVE_NAMESPACE = "serve"
_REFRESH_S = 0.5


def _controller():
    return ray.get_actor(CONTROLLER_NAME, namespace=SERVE_NAMESPACE)


class _Router:
    """Per-process replica view for one deployment."""

    _routers: Dict[str, "_Router"] = {}
    _lock = threading.Lock()

    @classmethod
    def get(cls, name: str) -> "_Router":
        with cls._lock:
            r = cls._routers.get(name)
            if r is None:
                r = cls._routers[name] = _Router(name)
            return r

    def __init__(self, name: str):
        self.name = name
        self.replicas: List[Any] = []
        self.version = -1
        self.last_refresh = 0.0
        self.inflight: Dict[int, list] = {}   # replica index -> outstanding refs
        self.lock = threading.Lock()
        self._reported = 0.0

    def refresh(self, force=False):
        now = time.time()
        if not force and self.replicas and now - self.last_refresh < _REFRESH_S:
            return
        ver, reps = ray.get(_controller().get_replicas.remote(self.name, self.version))
        self.last_refresh = now
        if ver != self.version and reps is not None:
            self.version = ver
            self.replicas = list(reps)
            self.inflight = {}

    def _load(self, i):
        lst = self.inflight.get(i, [])
        if lst:
            done, pending = ray.wait(lst, num_returns=len(lst), timeout=0)
            self.inflight[i] = pending
            return len(pending)
        return 0

    def choose(self):
        deadline = time.time() + 30
        while True:
            self.refresh()
            if self.replicas:
                break
            if time.time() > deadline:
                raise RuntimeError(f"Deployment {self.name!r} has no running replicas")
            time.sleep(0.05)
            self.refresh(force=True)
        n = len(self.replicas)
        if n == 1:
            return 0
        a, b = random.sample(range(n), 2)  # power of two choices
        return a if self._load(a) <= self._load(b) else b

    def record(self, i, ref):
        with self.lock:
            self.inflight.setdefault(i, []).append(ref)
        self._maybe_report()

    def _maybe_report(self):
        now = time.time()
        if now - self._reported > 0.25:
            self._reported = now
            total = sum(len(v) for v in self.inflight.values())
            try:
                _controller().record_handle_metrics.remote(self.name, total, now)
            except Exception:
                pass


class RayServeHandle:
    def __init__(self, deployment_name: str, method_name: Optional[str] = None, _sync: bool = True):
        self.deployment_name = deployment_name
        self.method_name = method_name
        self._sync = _sync

    def options(self, *, method_name: Optional[str] = None, **kw) -> "RayServeHandle":
        return RayServeHandle(self.deployment_name, method_name or self.method_name, self._sync)

    def remote(self, *args, **kwargs):
        r = _Router.get(self.deployment_name)
        for attempt in range(3):
            i = r.choose()
            replica = r.replicas[i]
            try:
                ref = replica.handle_request.remote(self.method_name or "__call__", args, kwargs)
            except Exception:
                r.refresh(force=True)
                continue
            r.record(i, ref)
            return ref
        raise RuntimeError(f"could not reach a replica of {self.deployment_name!r}")

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return self.options(method_name=name)

    def __reduce__(self):
        return (RayServeHandle, (self.deployment_name, self.method_name, self._sync))

    def __repr__(self):
        return f"RayServeHandle(deployment={self.deployment_name!r})"


RayServeSyncHandle = RayServeHandle


class _HandlePlaceholder:
    """A bound deployment passed as an init arg: replaced by a handle inside the replica."""

    def __init__(self, name):
        self.name = name


def _resolve_handles(obj):
    if isinstance(obj, _HandlePlaceholder):
        return RayServeHandle(obj.name)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_resolve_handles(x) for x in obj)
    if isinstance(obj, dict):
        return {k: _resolve_handles(v) for k, v in obj.items()}
    return obj
